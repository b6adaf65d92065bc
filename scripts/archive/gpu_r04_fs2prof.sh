# rocprofv3 kernel stats of the two-pass four-steps (2^16 power of 2, 48000 =
# 375 x 128, 10^6 = 1000 x 1000 smooth rows, composed chirp-z 65537)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fs2 -o fs2 --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/scripts/bench_sizes_default.py 65536 48000 1000000 65537 > $GRAFT_REPO_ROOT/gpurun_out/prof_fs2.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof_fs2.log
find $GRAFT_REPO_ROOT/gpurun_out/prof_fs2 -name "*kernel_stats.csv" | head -3
