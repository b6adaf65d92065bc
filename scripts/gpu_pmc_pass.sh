# One rocprofv3 --pmc pass over one bench workload (experiments):
#   scripts/gpu_pmc_pass.sh <workload> <tag> "<counters>" [VAR=value ...]
# Output: gpurun_out/pmc_<tag>/run_counter_collection.csv. The extra
# VAR=value arguments are exported for the profiled run (A/B switches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
W=$1; TAG=$2; C=$3; shift 3
for kv in "$@"; do export "$kv"; done
timeout -s KILL 90 rocprofv3 --pmc $C -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log 2>&1; rc=$?
echo "pmc $W $TAG rc=$rc"; [ $rc -eq 0 ] || tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log
exit $rc
