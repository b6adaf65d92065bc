# Pwelch partial-spectrum reduction with its loads in flight together:
# pytest -k pwelch, then kernel stats of the pwelch workload.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "pwelch or Pwelch" > gpurun_out/red_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/red_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_stats_round.sh pwelch
