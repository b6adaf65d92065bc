# Round 3 profile set: rocprofv3 --kernel-trace --stats of the five bench
# workloads (20 timed + 3 warm-up launches, as bench.py), the HBM PMC passes
# of the two kernels rebuilt this round, and the SQ counter passes of all five.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_stats_round.sh radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for W in chirpz3000 pwelch; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${W}_$c -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/pmc_${W}_$c.log 2>&1; rc=$?
    echo "pmc $W $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${W}_$c.log; exit $rc; }
  done
done
cd $R && bash scripts/gpu_sq.sh radix4096 bluestein3000 chirpz3000 pwelch fft2_8192
