set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "${K:-mixed or chirpz or plan_kinds or 3000}" > gpurun_out/quick_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/quick_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload bluestein3000 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/q1.json 2>&1; rc=$?; echo rc=$rc; [ $rc -eq 0 ] || exit $rc
GDSP_MIXED_GENERIC=1 timeout -k 10 300 python bench.py --workload bluestein3000 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/q2.json 2>&1; rc=$?; echo rc=$rc
python - <<'P'
import json
for f in ["gpurun_out/q1.json","gpurun_out/q2.json"]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"], d["parity"])
P
