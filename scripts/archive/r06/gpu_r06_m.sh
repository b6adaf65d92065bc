# Round 6: the large-batch chirp-z properties on the new pass-B radices, and
# the chirp-z lengths below 1025 (primes whose p - 1 is not smooth), for the
# next candidate range.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06m
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "large_batch_properties" > gpurun_out/r06m/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06m/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/sweep_nonsmooth.py 227 311 389 509 523 607 709 787 887 983 1019 > gpurun_out/r06m/small.jsonl 2> gpurun_out/r06m/sweep.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06m/sweep.err; exit $rc; }
