# chirp-z: the next row touched into L2 by the block TA places later in
# dispatch order (GDSP_C6_TA), and the persistent form (GDSP_C6_PERSIST)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so GDSP_C6_PERSIST=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "chirpz6k" > gpurun_out/ab_pytest.log 2>&1; echo "persist pytest rc=$? $(tail -1 gpurun_out/ab_pytest.log)"
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_C6_TA=256 GDSP_C6_TA=512 GDSP_C6_TA=768 GDSP_C6_TA=1024 GDSP_C6_TA=2048 GDSP_C6_PERSIST=1" 2
timeout -k 10 400 python -u -m pytest tests/test_multi.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04_multi2.log 2>&1; echo "multi rc=$? $(tail -1 gpurun_out/r04_multi2.log)"
