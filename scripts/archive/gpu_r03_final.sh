# Closing evidence of round 3: the full GPU suite + smoke, then rocprofv3
# kernel stats of the five bench workloads (20 timed + 3 warm-up launches).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite.sh && bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch
