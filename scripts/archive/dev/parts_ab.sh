# Output-split chirp-z: parity tests, then ms per 2^27 samples for the parts
# lengths with the parts kernel and with the composed chirp-z (GDSP_BLU_NOPARTS=1).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parts or plan_kinds or convolution_length" > gpurun_out/parts_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/parts_pytest.log; [ $rc -eq 0 ] || exit $rc
L="8209 10007 10909 11003 12281 12289 13999 14563"
timeout -k 10 300 python scripts/bench_sizes.py $L > gpurun_out/parts_sizes.jsonl 2>&1; rc=$?; [ $rc -eq 0 ] || { tail gpurun_out/parts_sizes.jsonl; exit $rc; }
GDSP_BLU_NOPARTS=1 timeout -k 10 300 python scripts/bench_sizes.py $L > gpurun_out/noparts_sizes.jsonl 2>&1; rc=$?; [ $rc -eq 0 ] || { tail gpurun_out/noparts_sizes.jsonl; exit $rc; }
paste <(grep '"chirpz": false' gpurun_out/parts_sizes.jsonl | python -c "import sys,json;[print(json.loads(l)['n'],json.loads(l)['ms']) for l in sys.stdin]") <(grep '"chirpz": false' gpurun_out/noparts_sizes.jsonl | python -c "import sys,json;[print(json.loads(l)['ms']) for l in sys.stdin]")
