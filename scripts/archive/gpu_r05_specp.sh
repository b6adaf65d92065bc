# Round 5, late: six more lists for 3000 / 2000 / 2400 / 1500 (lib_p1..p6,
# tools/spec_variants.py) against the default: fused Pwelch at half overlap
# (rocprofv3 kernel traces) and the batched FFT, two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_p1 lib_p2 lib_p3 lib_p4 lib_p5 lib_p6; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_sp_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 3000:1500 2000:1000 2400:1200 1500:750 > $R/gpurun_out/r05/sp_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/sp_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_sp_$L.$r/run_kernel_trace.csv
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py 3000 2000 2400 1500 > $R/gpurun_out/r05/sp_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $R/gpurun_out/r05/sp_fft_$L.$r.jsonl | python3 -c "import sys,json; print(' '.join(f\"{d['n']}:{d['ms']:.3f}\" for d in map(json.loads,sys.stdin)))"
done
done
