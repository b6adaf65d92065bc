# Pwelch worker counts on the development build (GDSP_PW_WORKERS), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for r in 1 2; do
  for w in 2048 1536 2560 3072 4096; do
    GDSP_PW_WORKERS=$w timeout -k 10 300 python bench.py --workload pwelch --steps 20 --warmup 3 --cpu-seconds 0 --check-rows 0 > gpurun_out/pw.json 2> gpurun_out/pw.err; rc=$?
    [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/pw.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/pw.json'));print('workers',$w,d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
