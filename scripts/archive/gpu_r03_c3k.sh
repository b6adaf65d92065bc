# M = 3072 / 6144 chirp-z: parity tests, then ms per 2^27 samples against the
# power-of-2 M (scripts/bench_c6k.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "chirpz or primes" > gpurun_out/c3k_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/c3k_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_c6k.py > gpurun_out/c3k_sizes.jsonl 2> gpurun_out/c3k_sizes.err; rc=$?
echo "sizes rc=$rc"; cat gpurun_out/c3k_sizes.jsonl; [ $rc -eq 0 ] || tail -20 gpurun_out/c3k_sizes.err
exit $rc
