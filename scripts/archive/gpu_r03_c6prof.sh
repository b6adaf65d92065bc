# Full GPU suite + smoke on the build with the M = 6144 chirp-z kernel, then
# its kernel stats (20 + 3 launches), HBM PMC passes and SQ counter passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite.sh && bash scripts/gpu_stats_round.sh chirpz3000 && \
  bash scripts/gpu_pmc_r03.sh chirpz3000 && bash scripts/gpu_sq.sh chirpz3000
