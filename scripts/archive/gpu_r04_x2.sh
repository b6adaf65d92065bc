# Round 4: Pwelch two-buffer exchange with the Hann window in registers
# (GDSP_PW_ROWX=8) and chirp-z ablations (GDSP_C6_ABL: 1 no x/chirp loads,
# 2 no bhat loads, 4 no output chirp loads, 7 none of them, 8 no exchange
# barriers, 15 all; timing only, wrong results)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh pwelch "GDSP_PW_ROWX=8 GDSP_PW_ROWX=1" 2 && \
bash scripts/gpu_ab_env.sh chirpz3000 "GDSP_C6_ABL=1 GDSP_C6_ABL=2 GDSP_C6_ABL=4 GDSP_C6_ABL=7 GDSP_C6_ABL=8 GDSP_C6_ABL=15" 1
