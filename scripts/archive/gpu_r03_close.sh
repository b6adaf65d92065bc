# Round-3 closing run at HEAD: the default bench line (as the driver runs it),
# then the full GPU suite + smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_bench_default.sh && bash scripts/gpu_suite.sh
