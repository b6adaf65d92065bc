# Small-call latency: the host API polling its stream (default) against the
# runtime's blocking wait (development build, GDSP_SMALL_BLOCK=1).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for r in 1 2; do
  echo "== poll"; timeout -k 10 300 python scripts/bench_host_latency.py || exit 1
  echo "== block"; GDSP_LIB=$DEV GDSP_SMALL_BLOCK=1 timeout -k 10 300 python scripts/bench_host_latency.py || exit 1
done
timeout -k 10 300 python bench.py --workload fftreal1024 --steps 20 --warmup 3 --cpu-seconds 2 > gpurun_out/fftreal.json 2> gpurun_out/fftreal.err; rc=$?
[ $rc -eq 0 ] || { tail -20 gpurun_out/fftreal.err; exit $rc; }
cat gpurun_out/fftreal.json
