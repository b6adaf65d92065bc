# Round 5, late: four-pass lists for the fused Pwelch (lib_q1..q3,
# tools/spec_variants.py) against the default, for 6000 / 4500 / 4000 / 800 /
# 2880 / 3200 / 1536 / 2400 at half overlap (rocprofv3 kernel traces), two
# alternating rounds; winners become Pwelch-only lists (specspw).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for r in 1 2; do
for L in default lib_q1 lib_q2 lib_q3; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_sq_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 6000:3000 4500:2250 4000:2000 800:400 2880:1440 3200:1600 1536:768 2400:1200 > $R/gpurun_out/r05/sq_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/sq_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_sq_$L.$r/run_kernel_trace.csv
done
done
