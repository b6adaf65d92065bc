# Quick GPU iteration: selected parity tests (-k expression $1), then bench
# lines for the workloads in $2 (default bluestein3000 chirpz3000).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "${1:-mixed or chirpz or plan_kinds}" > gpurun_out/quick_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/quick_pytest.log
[ $rc -eq 0 ] || exit $rc
for w in ${2:-bluestein3000 chirpz3000}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/quick_$w.json 2> gpurun_out/quick_$w.err; rc=$?
  echo "== $w rc=$rc"; cat gpurun_out/quick_$w.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/quick_$w.err; exit $rc; }
done
