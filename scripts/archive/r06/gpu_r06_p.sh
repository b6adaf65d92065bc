# Round 6: a random sample of 160 lengths 129 <= n <= 8192 with a prime
# factor above 31 (the lengths the reference and the smooth kernels leave to
# chirp-z; scripts/sweep_nonsmooth.py, production plans only) for the
# distribution of plan kinds and HBM fractions; and the PCIe-inclusive rate
# of the host-pointer API on the BASELINE shapes (scripts/bench_host_batch.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06p
cd $R
timeout -k 10 500 python3 scripts/sweep_nonsmooth.py --no-chirpz --samples 67108864 $(cat scripts/nonsmooth_sample.txt) > gpurun_out/r06p/sample.jsonl 2> gpurun_out/r06p/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06p/sweep.err; exit $rc; }
timeout -k 10 300 python3 scripts/bench_host_batch.py > gpurun_out/r06p/host_batch.json 2> gpurun_out/r06p/host.err; rc=$?
echo "host rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06p/host.err; exit $rc; }
cat gpurun_out/r06p/host_batch.json
