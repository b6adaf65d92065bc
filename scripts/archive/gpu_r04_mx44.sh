# 44100 (and 30000) with forced smooth-row lengths (GDSP_MXROW_C, dev build)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for C in 630 490 441 420 350 300 252 225 210 180 175 150 147 126 100; do
  GDSP_LIB=$DEV GDSP_MXROW_C=$C timeout -k 10 120 python scripts/bench_sizes_default.py 44100 > gpurun_out/mx44_$C.jsonl 2>> gpurun_out/mx44.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mx44_$C.jsonl').read()); print('44100 C=$C', d['plan_kind'], d['ms'])"
done
timeout -k 10 120 python scripts/bench_sizes_default.py 44100 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('44100 default', d['plan_kind'], d['ms'])"
for C in 1000 600 500 400 375 300 250 200 150 120 100; do
  GDSP_LIB=$DEV GDSP_MXROW_C=$C timeout -k 10 120 python scripts/bench_sizes_default.py 30000 > gpurun_out/mx30_$C.jsonl 2>> gpurun_out/mx44.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mx30_$C.jsonl').read()); print('30000 C=$C', d['plan_kind'], d['ms'])"
done
