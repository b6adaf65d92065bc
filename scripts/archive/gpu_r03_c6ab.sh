# chirp-z M = 6144 variants (A/B), then SQ counters of the default build
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab.sh chirpz3000 "$1" 2 && bash scripts/gpu_sq.sh chirpz3000
