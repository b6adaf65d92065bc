# FFT2 8192^2: the two column steps slab by slab (A then B per column slab,
# so B reads A's output from the Infinity Cache), optionally dealt over side
# streams (dev build switches GDSP_FFT2_SLAB, GDSP_FFT2_STREAMS).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh fft2_8192 "GDSP_FFT2_SLAB=512 GDSP_FFT2_SLAB=1024 GDSP_FFT2_SLAB=256 GDSP_FFT2_SLAB=512,GDSP_FFT2_STREAMS=2 GDSP_FFT2_SLAB=256,GDSP_FFT2_STREAMS=2 GDSP_FFT2_SLAB=256,GDSP_FFT2_STREAMS=4 GDSP_FFT2_SLAB=128,GDSP_FFT2_STREAMS=4" 2 fft2
