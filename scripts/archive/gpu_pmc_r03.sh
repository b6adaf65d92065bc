# HBM PMC passes (FETCH_SIZE, WRITE_SIZE: one counter set per run) of the
# given bench workloads' dominant kernels; summarised by tools/pmc_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for W in ${@:-radix4096 bluestein3000 fft2_8192}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${W}_$c -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/pmc_${W}_$c.log 2>&1; rc=$?
    echo "pmc $W $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${W}_$c.log; exit $rc; }
  done
done
