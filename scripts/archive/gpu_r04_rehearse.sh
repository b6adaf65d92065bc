# The default bench line (every nested config) at N = 2 and 4 through the plain
# command, ranks sharing the box's one GPU over gloo: the path the driver's
# 8-GPU run takes, minus RCCL.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_mirror.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/replay.log 2>&1; echo "replay rc=$? $(tail -1 gpurun_out/replay.log)"
for N in 2 4; do
  GDSP_DIST_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus $N --steps 3 --warmup 1 > gpurun_out/rehearse_default_$N.json 2> gpurun_out/rehearse_default_$N.err; rc=$?
  echo "N=$N rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse_default_$N.err; exit $rc; }
  python3 -c "import json;d=json.load(open('gpurun_out/rehearse_default_$N.json'));print(d['n_gpus'],d['value'],d['ms_per_step'],d['config']['parallelism'],sorted(d['configs']),{k:v['value'] for k,v in d['configs'].items()}, d.get('weak_scaling',{}).get('value'))"
done
