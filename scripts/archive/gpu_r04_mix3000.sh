# n = 3000 production kernel: alternative radix lists compiled by hipRTC
# (dev switch GDSP_JIT_RADICES) against the compiled 25*15*8 specialisation
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh bluestein3000 "GDSP_JIT_RADICES=25x15x8 GDSP_JIT_RADICES=10x15x20 GDSP_JIT_RADICES=20x15x10 GDSP_JIT_RADICES=12x10x25 GDSP_JIT_RADICES=8x15x25 GDSP_JIT_RADICES=24x5x25 GDSP_JIT_RADICES=6x20x25" 2
