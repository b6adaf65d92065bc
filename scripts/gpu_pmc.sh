# HBM traffic of the bench workloads from rocprofv3 PMC counters: FETCH_SIZE
# and WRITE_SIZE in separate passes (TCC slots), kernel-trace only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
for W in ${@:-radix4096}; do
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${W}_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/pmc_${W}_$c.log 2>&1; rc=$?
  echo "pmc $W $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
