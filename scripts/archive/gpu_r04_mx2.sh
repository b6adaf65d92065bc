# Two-pass mixed four-step (columns + power-of-2 rows with the transpose in
# their store): parity, then per 2^27 samples against GDSP_MX3=1 (dev build).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread \
  -k "mixed or smooth or random or fourstep or sizes or beyond" > gpurun_out/mx2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/mx2_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/mx2_pytest.log | head; exit $rc; }
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
SZ="10000 12000 20000 48000 96000 196608 160000"
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_sizes_default.py $SZ > gpurun_out/mx2_new_$r.jsonl 2>> gpurun_out/mx2.err || exit $?
  GDSP_LIB=$DEV GDSP_MX3=1 timeout -k 10 300 python scripts/bench_sizes_default.py $SZ > gpurun_out/mx2_old_$r.jsonl 2>> gpurun_out/mx2.err || exit $?
  python3 -c "
import json
for tag in ('new','old'):
    for l in open('gpurun_out/mx2_%s_$r.jsonl' % tag):
        d=json.loads(l); print(tag, d['n'], d['batch'], d['plan_kind'], d['ms'], d['alg_tb_s'])
"
done
