# Full GPU suite on the current build, then A/B of the chirp-z and Pwelch
# kernels against the previous commit's build (go-dsp_amd/lib_head).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r03_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh "chirpz3000 pwelch radix4096" "default go-dsp_amd/lib_head" 3 || exit 1
