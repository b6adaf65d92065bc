# Parity tests, then every BASELINE workload through bench.py, each also
# under rocprofv3 --kernel-trace --stats. Stops at the first GPU failure.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in ${WORKLOADS:-radix4096 bluestein3000 chirpz3000 fft2_8192 fft2_dist pwelch fftn_512 wav_decode}; do
  cs=10
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds $cs > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err; rc=$?
  echo "== $w rc=$rc"; cat gpurun_out/bench_$w.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$w.err; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-radix4096 bluestein3000 chirpz3000 fft2_8192 fft2_dist pwelch fftn_512 wav_decode}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 5 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$w.log 2>&1; rc=$?
  echo "prof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
