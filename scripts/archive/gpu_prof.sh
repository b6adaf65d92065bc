# rocprofv3 --kernel-trace --stats of bench workloads ($@), 5 timed steps each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 5 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$w.log 2>&1; rc=$?
  echo "prof $w rc=$rc"; [ $rc -eq 0 ] || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_$w.log; exit $rc; }
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$GRAFT_REPO_ROOT/gpurun_out/prof_$w/run_kernel_stats.csv')))
for r in rows: print('  %-90s calls=%s avg_us=%.1f min_us=%.1f' % (r['Name'][:90], r['Calls'], float(r['AverageNs'])/1e3, float(r['MinNs'])/1e3))
"
done
