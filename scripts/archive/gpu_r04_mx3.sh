# Two-pass mixed four-step with smooth (non-power-of-2) rows by the runtime-
# compiled rowt_fixed_kernel: parity, then per 2^27 samples against GDSP_MX3=1.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export GDSP_JIT_VERBOSE=1
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread \
  -k "mixed or smooth or random or fourstep or sizes or beyond" > gpurun_out/mx3_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/mx3_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert|hipRTC" gpurun_out/mx3_pytest.log | head -20; exit $rc; }
unset GDSP_JIT_VERBOSE
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
SZ="9000 27000 30000 44100 50000 60000 72000 88200 100000 200000 600000 1000000 4961250"
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_sizes_default.py $SZ > gpurun_out/mx3_new_$r.jsonl 2>> gpurun_out/mx3.err || exit $?
  GDSP_LIB=$DEV GDSP_MX3=1 timeout -k 10 300 python scripts/bench_sizes_default.py $SZ > gpurun_out/mx3_old_$r.jsonl 2>> gpurun_out/mx3.err || exit $?
  python3 -c "
import json
for tag in ('new','old'):
    for l in open('gpurun_out/mx3_%s_$r.jsonl' % tag):
        d=json.loads(l); print(tag, d['n'], d['batch'], d['plan_kind'], d['ms'], d['alg_tb_s'])
"
done
