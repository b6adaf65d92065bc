# n = 3000 production kernel: alternative radix lists compiled by hipRTC
# (dev switch GDSP_JIT_RADICES) against the compiled 25*15*8 specialisation
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh bluestein3000 "GDSP_JIT_RADICES=25,15,8 GDSP_JIT_RADICES=10,15,20 GDSP_JIT_RADICES=20,15,10 GDSP_JIT_RADICES=12,10,25 GDSP_JIT_RADICES=8,15,25 GDSP_JIT_RADICES=24,5,25 GDSP_JIT_RADICES=6,20,25" 2
