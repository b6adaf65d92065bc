# Twiddle powers by the three-term recurrence (default build, GDSP_TW_CHEB=1)
# against complex products (lib_dev built with -DGDSP_TW_CHEB=0): parity of the
# default build first, then alternating bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "chirpz or bluestein or fullsize or sizes" > gpurun_out/cheb_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/cheb_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_env.sh "chirpz3000" "GDSP_X=1" 3
