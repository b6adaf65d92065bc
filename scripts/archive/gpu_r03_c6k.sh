# M = 6144 chirp-z (chirpz6k.hip): its parity tests and the chirp-z tests
# around it, then the chirpz3000 bench line (with the M = 8192 time beside it)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "chirpz or primes or random" > gpurun_out/c6k_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/c6k_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload chirpz3000 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/c6k_bench.json 2> gpurun_out/c6k_bench.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/c6k_bench.json; [ $rc -eq 0 ] || tail -20 gpurun_out/c6k_bench.err
exit $rc
