set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "chirpz or bluestein or prime or 3000 or smoke or fullsize" > gpurun_out/kn_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/kn_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_BLU_NOKN=1" 3
