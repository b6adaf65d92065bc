# Round 5, second evidence session: HBM PMC passes (FETCH_SIZE, WRITE_SIZE)
# of the two new bench lines, and the Pwelch NFFT cases of
# scripts/bench_pwelch.py under a rocprofv3 kernel trace (per-case kernel
# times; tools/trace_cases.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
for W in prime3001 pwelch_default; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -d $R/gpurun_out/pmc_${W}_$c -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/pmc_${W}_$c.log 2>&1; rc=$?
    echo "pmc $W $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${W}_$c.log; exit $rc; }
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_pw -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py > $R/gpurun_out/prof_pw.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -20 $R/gpurun_out/prof_pw.log; [ $rc -eq 0 ] || exit $rc
cd $R && python3 tools/trace_cases.py gpurun_out/prof_pw/run_kernel_trace.csv > gpurun_out/pw_cases.txt && cat gpurun_out/pw_cases.txt
