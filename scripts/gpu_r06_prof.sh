# Round 6, closing profile session at the current sources: the sources'
# stamp, then rocprofv3 --kernel-trace --stats of every bench workload
# (tools/trace_summary.py reads them), the HBM PMC passes of the headline,
# configs[4] and the new kind-8 line, and the SQ passes of the kind-7/8
# kernels. Usage: gpu_r06_prof.sh stats|pmc|sq [pmc workloads]
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
python3 $R/tools/source_stamp.py > $R/gpurun_out/source_stamp.json
cd /tmp && export TMPDIR=/tmp
case "$1" in
stats)
  for W in radix4096 bluestein3000 chirpz3000 prime3001 pfa3027 fft2_8192 pwelch pwelch_default; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 20 --warmup 3 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/prof_$W.log 2>&1; rc=$?
    echo "stats $W rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/prof_$W.log; exit $rc; }
  done ;;
pmc)
  for W in ${2:-radix4096 pwelch pfa3027 prime3001}; do
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${W}_$c -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/pmc_${W}_$c.log 2>&1; rc=$?
      echo "pmc $W $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${W}_$c.log; exit $rc; }
    done
  done ;;
sq)
  bash $R/scripts/gpu_sq.sh pfa3027 prime3001 ;;
esac
