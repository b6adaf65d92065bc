# Round 5, late: the runtime-compiled lists chosen with the lane-cost model
# (mixed_jit.hip jit_radices, lib_jc) against the default chooser, on 43 of
# the 127 smooth lengths whose list it changes: batched FFT, fused Pwelch
# (half overlap, rocprofv3 kernel traces), and Rader on 12 primes whose
# n - 1 list changes; two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NS="36 75 252 420 522 550 576 684 792 828 975 1116 1425 1584 1725 1960 2088 2280 2340 2480 2736 3100 3276 3400 3675 3850 3978 4104 4200 4464 4760 5670 6075 6264 6600 6912 7056 7290 7425 7605 7830 7956 8160"
PW=""; for n in $NS; do [ $n -ge 64 ] && PW="$PW $n:$((n/2))"; done
PR="37 73 421 577 691 1117 1657 2017 2341 3457 4201 6481"
for r in 1 2; do
for L in default lib_jc; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 400 python3 $R/scripts/bench_sizes_default.py $NS > $R/gpurun_out/r05/jc_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/jc_fft_$L.$r.jsonl; exit $rc; }
  timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_jc_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/jc_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/jc_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_jc_$L.$r/run_kernel_trace.csv > $R/gpurun_out/r05/jc_pwk_$L.$r.txt
  timeout -k 10 300 python3 $R/scripts/bench_rader.py $PR > $R/gpurun_out/r05/jc_rader_$L.$r.jsonl 2>&1; rc=$?
  echo "== rader $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/jc_rader_$L.$r.jsonl; exit $rc; }
done
done
