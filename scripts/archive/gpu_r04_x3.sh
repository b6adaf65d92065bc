# chirp-z ablations: 16 = x loads only replaced by constants, 32 = the
# premultiply chirp loads only, 1 = both (timing only, wrong results)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_C6_ABL=16 GDSP_C6_ABL=32 GDSP_C6_ABL=1" 2
