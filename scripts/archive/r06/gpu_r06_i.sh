# Round 6: chirp-z pass-B register targets — the non-smooth sweep on the
# libraries named in $1 (directories under go-dsp_amd/, alternating, 2 rounds)
# for the lengths in $2. Output gpurun_out/r06i/<lib>_<round>.jsonl.
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06i
cd $R
for r in 1 2; do
  for L in $1; do
    GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/sweep_nonsmooth.py $2 > gpurun_out/r06i/${L}_$r.jsonl 2> gpurun_out/r06i/sweep.err; rc=$?
    echo "$L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06i/sweep.err; exit $rc; }
  done
done
