# Round 5, late: radix lists of 26 compiled specialisations (tools/spec_candidates.py's
# two best-ranked lists, lib_v1 / lib_v2, built by tools/spec_variants.py) against the
# default: batched FFT, fused Pwelch (half overlap, rocprofv3 kernel traces) and Rader
# on the primes n + 1 that use these lists; two alternating rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
NS="100 160 300 360 400 600 640 720 750 768 1080 1125 1152 1200 1280 1470 1764 1875 2160 2205 2500 2940 3750 4000 5880 8000"
PW=""; for n in $NS; do PW="$PW $n:$((n/2))"; done
PR="101 401 601 641 751 769 1153 1201 1471 2161 4001 5881"
for r in 1 2; do
for L in default lib_v1 lib_v2; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py $NS > $R/gpurun_out/r05/sd_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/sd_fft_$L.$r.jsonl; exit $rc; }
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_sd_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/sd_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/sd_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_sd_$L.$r/run_kernel_trace.csv > $R/gpurun_out/r05/sd_pwk_$L.$r.txt
  timeout -k 10 300 python3 $R/scripts/bench_rader.py $PR > $R/gpurun_out/r05/sd_rader_$L.$r.jsonl 2>&1; rc=$?
  echo "== rader $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/sd_rader_$L.$r.jsonl; exit $rc; }
done
done
