# Four-step rows on the output-split chirp-z: parity tests, then ms per 2^27
# samples with and without the parts (GDSP_BLU_NOPARTS=1); FFT2 out-of-place A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parts or plan_kinds or convolution_length or fourstep" > gpurun_out/parts_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/parts_pytest.log; [ $rc -eq 0 ] || exit $rc
L="525376 20014 36867 16418 24627"
timeout -k 10 300 python scripts/bench_sizes.py $L > gpurun_out/rows_parts.jsonl 2>&1; rc=$?; [ $rc -eq 0 ] || { tail gpurun_out/rows_parts.jsonl; exit $rc; }
GDSP_BLU_NOPARTS=1 timeout -k 10 300 python scripts/bench_sizes.py $L > gpurun_out/rows_noparts.jsonl 2>&1; rc=$?; [ $rc -eq 0 ] || { tail gpurun_out/rows_noparts.jsonl; exit $rc; }
paste <(grep '"chirpz": false' gpurun_out/rows_parts.jsonl | python -c "import sys,json;[print(json.loads(l)['n'],json.loads(l)['plan_kind'],json.loads(l)['ms']) for l in sys.stdin]") <(grep '"chirpz": false' gpurun_out/rows_noparts.jsonl | python -c "import sys,json;[print(json.loads(l)['plan_kind'],json.loads(l)['ms']) for l in sys.stdin]")
bash scripts/gpu_ab.sh fft2_8192 "default env:GDSP_FFT2_OOP=1" 3
