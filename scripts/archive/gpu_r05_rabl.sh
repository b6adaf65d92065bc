# Round 5, late: where the Rader kernel's time goes (development ablations,
# results wrong by design): lib_a1 without the b-hat loads (C = A), lib_a2
# without the ginv loads (identity scatter), lib_a3 without the gpow loads
# (identity gather); bench.py prime3001 per library, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_a1 lib_a2 lib_a3; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_rader.py 3001 > $R/gpurun_out/r05/rabl_$L.$r.jsonl 2>&1; rc=$?
  echo "== $L $r rc=$rc $(grep '^{' $R/gpurun_out/r05/rabl_$L.$r.jsonl | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms"])')"
  [ $rc -eq 0 ] || exit $rc
done
done
