# N = 4096 LDS kernel with (default build) and without (lib_v1) the
# wave-priority pass, alternating; parity of the default build first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT/go-dsp_amd
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "4096 or batch or sizes or chirpz_plan" > gpurun_out/prio_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/prio_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for L in lib lib_v1; do
    GDSP_LIB=$R/$L/libgdspfft.so timeout -k 10 300 python bench.py --workload radix4096 --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('radix4096','$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],(d.get('parity') or {}).get('max_nrel_vs_oracle'))"
  done
done
