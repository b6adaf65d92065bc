# Round-2 baseline: smoke, bench lines of the five BASELINE workloads, and a
# rocprofv3 kernel-stats summary of the chirp-z and Pwelch workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/smoke.log; exit $rc; }
for w in radix4096 bluestein3000 chirpz3000 fft2_8192 pwelch; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/base_$w.json 2> gpurun_out/base_$w.err; rc=$?
  echo "== $w rc=$rc"; cat gpurun_out/base_$w.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/base_$w.err; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
for w in chirpz3000 pwelch; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 5 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$w.log 2>&1; rc=$?
  echo "prof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
