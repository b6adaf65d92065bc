# n = 3000 mixed-radix kernel: exchange as real / imaginary halves (24 KiB of
# LDS: six workgroups per CU instead of three) against the complex exchange
# (dev build switch GDSP_MIX_SPLIT).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_ab_env.sh "bluestein3000" "GDSP_MIX_SPLIT=1" 3 "mixed or 3000 or sizes"
