set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_tw1/libgdspfft.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "pwelch" > gpurun_out/r03_pytest_tw1.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r03_pytest_tw1.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh pwelch "default go-dsp_amd/lib_tw1" 4 || exit 1
