# A/B of the default library against development-build switches: for each
# workload in $1, alternate "default" and each "VAR=value[,VAR=value]" spec in
# $2 (run on go-dsp_amd/lib_dev) for $3 rounds; pytest -k $4 first on the
# dev build with the first spec's switches (parity).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
if [ -n "$4" ]; then
  first=$(echo $2 | awk '{print $1}' | tr ',' ' ')
  env GDSP_LIB=$DEV $first timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$4" > gpurun_out/ab_pytest.log 2>&1; rc=$?
  echo "pytest ($first) rc=$rc"; tail -2 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${3:-2}); do
for w in $1; do
  for L in default $2; do
    if [ "$L" = default ]; then EV="GDSP_X=0"; else EV="GDSP_LIB=$DEV $(echo $L | tr ',' ' ')"; fi
    env $EV timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || { echo "$w $L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$w','$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],(d.get('parity') or {}).get('max_nrel_vs_oracle'))"
  done
done
done
