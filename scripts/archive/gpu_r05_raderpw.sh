# Round 5, late: Rader's FFT_(n-1) on the fused Pwelch's own lists (lib_rp:
# 3000 -> 15 5 5 8, 4000 -> 10 10 10 4) against the FFT lists (25 15 8,
# 25 20 8): primes 3001 and 4001, two alternating rounds, plus the bench's
# prime3001 workload under a rocprofv3 kernel trace for each.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_rp; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_rader.py 3001 4001 > $R/gpurun_out/r05/rp_$L.$r.jsonl 2>&1; rc=$?
  echo "== rader $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/rp_$L.$r.jsonl; exit $rc; }
  grep '^{' $R/gpurun_out/r05/rp_$L.$r.jsonl
done
done
cd /tmp && export TMPDIR=/tmp
for L in default lib_rp; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05/prof_rp_$L -o run --output-format csv -- python3 $R/bench.py --workload prime3001 --steps 10 --warmup 3 > $R/gpurun_out/r05/rp_bench_$L.json 2> $R/gpurun_out/r05/rp_bench_$L.err; rc=$?
  echo "== bench $L rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/rp_bench_$L.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/r05/rp_bench_$L.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline'])"
done
