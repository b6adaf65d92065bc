# Sweep of one experiment switch: $1 = variable name, $2 = space-separated
# values (first = control), $3 = pytest -k expression run under every non-empty
# value, remaining args = bench workloads timed under each value.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V="$1"; VALS="$2"; KX="$3"; shift 3
for val in $VALS; do
  if [ -n "$KX" ]; then
    env $V=$val timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "$KX" > gpurun_out/sw_pytest.log 2>&1; rc=$?
    echo "$V=$val pytest rc=$rc $(tail -1 gpurun_out/sw_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/sw_pytest.log | head; exit $rc; }
  fi
  for w in "$@"; do
    env $V=$val timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/sw.json 2> gpurun_out/sw.err; rc=$?
    [ $rc -eq 0 ] || { tail -20 gpurun_out/sw.err; exit $rc; }
    python -c "import json; d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('$w $V=$val', d['value'], 'ms', d['ms_per_step'], 'launch', d['roofline']['avg_launch_ms'])"
  done
done
