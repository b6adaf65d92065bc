# Two-pass four-step extended to 2^19 / 2^20 (rows or columns of 1024: 64-128-B
# segments; dev build GDSP_FS2_MAX=20) against the three-pass form.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
GDSP_LIB=$DEV GDSP_FS2_MAX=20 timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "fourstep or fft_sizes or fft_real" > gpurun_out/fs2b_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/fs2b_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/fs2b_pytest.log | head; exit $rc; }
for r in 1 2; do
  GDSP_LIB=$DEV GDSP_FS2_MAX=20 timeout -k 10 300 python scripts/bench_sizes_default.py 524288 1048576 > gpurun_out/fs2b_new_$r.jsonl 2>> gpurun_out/fs2b.err || exit $?
  timeout -k 10 300 python scripts/bench_sizes_default.py 524288 1048576 > gpurun_out/fs2b_old_$r.jsonl 2>> gpurun_out/fs2b.err || exit $?
  python3 -c "
import json
for tag in ('new','old'):
    for l in open('gpurun_out/fs2b_%s_$r.jsonl' % tag):
        d=json.loads(l); print(tag, d['n'], d['batch'], d['ms'], d['alg_tb_s'])
"
done
GDSP_LIB=$DEV GDSP_FS2_MAX=20 timeout -k 10 300 python bench.py --workload fft_2p20 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/fs2b_2p20_new.json 2>> gpurun_out/fs2b.err || exit $?
timeout -k 10 300 python bench.py --workload fft_2p20 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/fs2b_2p20_old.json 2>> gpurun_out/fs2b.err || exit $?
for t in new old; do python3 -c "import json;d=json.load(open('gpurun_out/fs2b_2p20_$t.json'));print('fft_2p20 $t', d['ms_per_step'], d['value'], (d.get('parity') or {}).get('max_nrel_vs_oracle'))"; done
