# Round 6: the fused chirp-z for 129 <= n <= 1024 (pass-B radices 2-8,
# several transforms per workgroup): parity, then the sweep on the product
# library, the previous one (go-dsp_amd/lib_base: powers of 2 there) and
# go-dsp_amd/lib_exp (RB 5 and 8 at 2 waves per SIMD, no spills).
set -o pipefail
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
mkdir -p $R/gpurun_out/r06n
cd $R
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chirpz6k or chirpz_plan" > gpurun_out/r06n/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r06n/pytest.log; [ $rc -eq 0 ] || exit $rc
N="131 227 251 257 311 383 389 509 521 523 607 631 641 709 761 769 787 887 907 983 1021"
for r in 1 2; do
  for L in lib_base lib lib_exp; do
    GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so timeout -k 10 300 python3 scripts/sweep_nonsmooth.py $N > gpurun_out/r06n/${L}_$r.jsonl 2> gpurun_out/r06n/sweep.err; rc=$?
    echo "$L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06n/sweep.err; exit $rc; }
  done
done
