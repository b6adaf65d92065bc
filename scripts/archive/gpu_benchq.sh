# bench lines (no CPU baseline) for the workloads given as arguments
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/bq_$w.json 2> gpurun_out/bq_$w.err; rc=$?
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bq_$w.err; exit $rc; }
  python -c "import json; d=json.loads(open('gpurun_out/bq_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], 'ms/step', d['ms_per_step'], 'launch', d['roofline']['avg_launch_ms'], 'frac', d['roofline']['frac'], 'parity', (d.get('parity') or {}).get('max_nrel_vs_oracle'))"
done
