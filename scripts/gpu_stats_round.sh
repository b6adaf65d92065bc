# rocprofv3 --kernel-trace --stats of the bench workloads with the bench's own
# step counts (20 timed, 3 warm-up), so the kernel averages are over the same
# launches bench.py times (the cold first launch is 1 of 23).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for W in ${@:-radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 20 --warmup 3 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/prof_$W.log 2>&1; rc=$?
  echo "stats $W rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/prof_$W.log; exit $rc; }
done
