# Occupancy variants: Pwelch without the register prefetch / with the
# half-size exchange buffer at 3 waves per SIMD, chirp-z with the half-size
# exchange buffer (dev build switches GDSP_PW_OCC, GDSP_BLU_HALFX).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh pwelch "GDSP_PW_OCC=1 GDSP_PW_OCC=2 GDSP_PW_OCC=3" 2 pwelch && \
GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so GDSP_BLU_HALFX=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k chirpz > gpurun_out/ab_pytest2.log 2>&1 && tail -1 gpurun_out/ab_pytest2.log && \
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_BLU_HALFX=1" 2
