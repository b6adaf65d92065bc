# n = 3000 mixed kernel at four waves per SIMD (VGPRs capped at 128) with the
# split exchange: one (GDSP_MIX_TPW=14) or two (=24) transforms per block
# (dev build), against the default kernel.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh bluestein3000 "GDSP_MIX_TPW=14 GDSP_MIX_TPW=24 GDSP_MIX_TPW=15" 3 "mixed or 3000"
