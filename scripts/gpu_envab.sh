# A/B of an experiment switch: $1 = env assignment for arm B (e.g. GDSP_COL_WG=512),
# $2 = pytest -k expression run under arm B, remaining args = bench workloads
# timed under both arms.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="$1"; KX="$2"; shift 2
env $B timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "$KX" > gpurun_out/ab_pytest.log 2>&1; rc=$?
echo "B pytest rc=$rc $(tail -1 gpurun_out/ab_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/ab_pytest.log | head; exit $rc; }
for w in "$@"; do
  for arm in A B; do
    if [ $arm = A ]; then E=""; else E="$B"; fi
    env $E timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || { tail -20 gpurun_out/ab.err; exit $rc; }
    python -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$w arm $arm', d['value'], 'launch', d['roofline']['avg_launch_ms'])"
  done
done
