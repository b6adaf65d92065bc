# Round 6: the host-pointer API's PCIe-inclusive rate, fresh and resident outputs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06q
cd $R
timeout -k 10 300 python3 scripts/bench_host_batch.py > gpurun_out/r06q/host_batch.json 2> gpurun_out/r06q/host.err; rc=$?
echo "host rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06q/host.err; exit $rc; }
cat gpurun_out/r06q/host_batch.json
