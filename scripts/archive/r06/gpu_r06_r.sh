# Round 6: host-pointer API with 8 host copy threads (go-dsp_amd/lib_exp)
# against 4 (the product library), alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06r
cd $R
for r in 1 2; do
  for L in lib lib_exp; do
    GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/bench_host_batch.py > gpurun_out/r06r/${L}_$r.json 2> gpurun_out/r06r/host.err; rc=$?
    echo "$L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06r/host.err; exit $rc; }
    cat gpurun_out/r06r/${L}_$r.json
  done
done
