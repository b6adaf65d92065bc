# Two-pass four-step (2^15..2^18): parity, then per-2^27-sample times against
# the three-pass form (GDSP_FS3=1 on the development build), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "fourstep or fft_sizes or fft_real" > gpurun_out/fs2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/fs2_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/fs2_pytest.log | head; exit $rc; }
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for r in 1 2; do
  timeout -k 10 300 python scripts/bench_sizes_default.py 32768 65536 131072 262144 524288 > gpurun_out/fs2_new_$r.jsonl 2>> gpurun_out/fs2.err || exit $?
  GDSP_LIB=$DEV GDSP_FS3=1 timeout -k 10 300 python scripts/bench_sizes_default.py 32768 65536 131072 262144 524288 > gpurun_out/fs2_old_$r.jsonl 2>> gpurun_out/fs2.err || exit $?
  python3 -c "
import json
for tag in ('new','old'):
    for l in open('gpurun_out/fs2_%s_$r.jsonl' % tag):
        d=json.loads(l); print(tag, d['n'], d['batch'], d['ms'], d['alg_tb_s'])
"
done
