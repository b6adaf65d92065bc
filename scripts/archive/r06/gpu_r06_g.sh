# Round 6: SQ passes of the kind-8 / kind-7 kernels, then the rocprofv3
# traces and stats of every bench workload (one session, one stamp).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_r06_prof.sh sq && bash $R/scripts/gpu_r06_prof.sh stats
