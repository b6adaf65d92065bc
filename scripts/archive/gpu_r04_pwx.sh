# Round 4: Pwelch occupancy variants (dev build, GDSP_PW_ROWX, pwelch_rowx.hip)
# against the default row kernel, alternating, 2 rounds; parity of each
# variant from the bench line's oracle check (Hann window).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh pwelch "GDSP_PW_ROWX=1 GDSP_PW_ROWX=2 GDSP_PW_ROWX=5 GDSP_PW_ROWX=6 GDSP_PW_ROWX=7" 2
