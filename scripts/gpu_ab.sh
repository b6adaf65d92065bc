# A/B bench of alternate library builds: for each workload in $1, alternate
# the builds in $2 (paths relative to the repo; "default" = go-dsp_amd/lib)
# for $3 rounds (default 2). Parity tests selected by $4 (-k) run first on the
# default build.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$4" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$4" > gpurun_out/ab_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${3:-2}); do
for w in $1; do
  for L in $2; do
    # "default", a library directory, or env:VAR=value (default library, one switch set)
    unset GDSP_LIB; EV=""
    case "$L" in default) ;; env:*) EV="${L#env:}" ;; *) export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so ;; esac
    env $EV timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || { echo "$w $L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$w','$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],(d.get('parity') or {}).get('max_nrel_vs_oracle'))"
  done
done
done
