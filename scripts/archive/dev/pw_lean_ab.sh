# Register-lean Pwelch (GDSP_PW_LEAN=1, three waves per SIMD): parity with the
# switch on, then alternating timings against the default kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_PW_LEAN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pwelch" > gpurun_out/lean_pytest.log 2>&1; rc=$?
[ $rc -eq 0 ] && { GDSP_PW_LEAN=1 GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_leannc/libgdspfft.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pwelch" >> gpurun_out/lean_pytest.log 2>&1; rc=$?; }
echo "pytest rc=$rc"; tail -3 gpurun_out/lean_pytest.log; [ $rc -eq 0 ] || exit $rc
one() {  # label, env...
  env "${@:2}" timeout -k 10 300 python bench.py --workload pwelch --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "$1 failed"; tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$1',d['ms_per_step'],r['avg_launch_ms'])"
}
for r in 1 2 3; do
  one default GDSP_X=0
  one lean GDSP_PW_LEAN=1
  one lean_lin GDSP_PW_LEAN=1 GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_leanlin/libgdspfft.so
  one lean_nocarry GDSP_PW_LEAN=1 GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_leannc/libgdspfft.so
  one lean_nc_w3072 GDSP_PW_LEAN=1 GDSP_PW_WORKERS=3072 GDSP_LIB=$GRAFT_REPO_ROOT/go-dsp_amd/lib_leannc/libgdspfft.so
done
