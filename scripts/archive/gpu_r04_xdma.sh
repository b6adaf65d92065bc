# Rehearsal (shim replay + gloo default bench N=2,4) then the chirp-z LDS-DMA
# prologue A/B (GDSP_C6_XDMA=1 on the dev build) with its parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_r04_rehearse.sh || exit $?
bash scripts/gpu_ab_env.sh "chirpz3000" "GDSP_C6_XDMA=1" 3 "bluestein or chirp or 3000 or real_batch"
