# chirp-z M = 8192 with 16 points per thread (4 waves per SIMD) against the
# default 32 (dev build switches GDSP_BLU_E16, GDSP_BLU_E16KN), on the current kernels.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_BLU_E16=1 GDSP_BLU_E16=1,GDSP_BLU_E16KN=1" 2 chirpz
