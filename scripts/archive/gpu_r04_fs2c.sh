# Composed chirp-z on the two-pass FFT_M (rowfft_t modes 2/3): parity, then per
# 2^27 samples against the three-pass form (GDSP_FS3=1, development build).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread \
  -k "chirpz or random or beyond or fourstep or parts" > gpurun_out/fs2c_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/fs2c_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/fs2c_pytest.log | head; exit $rc; }
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_sizes_default.py 16381 16411 40009 65537 200003 262147 > gpurun_out/fs2c_new_$r.jsonl 2>> gpurun_out/fs2c.err || exit $?
  GDSP_LIB=$DEV GDSP_FS3=1 timeout -k 10 300 python scripts/bench_sizes_default.py 16381 16411 40009 65537 200003 262147 > gpurun_out/fs2c_old_$r.jsonl 2>> gpurun_out/fs2c.err || exit $?
  python3 -c "
import json
for tag in ('new','old'):
    for l in open('gpurun_out/fs2c_%s_$r.jsonl' % tag):
        d=json.loads(l); print(tag, d['n'], d['batch'], d['plan_kind'], d['ms'], d['alg_tb_s'])
"
done
