# Kernel-trace profiles of bench_sizes_default.py for the given lengths under each
# column-pass variant ($VARIANTS: env assignments, ';'-separated).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-X=0}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  ( export $v; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_col$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_sizes_default.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_col$i.log 2>&1 ); rc=$?
  echo "variant $i ($v) rc=$rc"; grep '^{' $GRAFT_REPO_ROOT/gpurun_out/prof_col$i.log | grep '"chirpz": false' | cut -c1-110
  [ $rc -eq 0 ] || exit $rc
done
