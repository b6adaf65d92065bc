# Round 5, late: (1) radix lists for the specialisations 2560 / 2880 / 3200 /
# 3840 / 4500 / 6000, two variant libraries against the default, fused Pwelch
# (rocprofv3 kernel traces) and the batched FFT, two alternating rounds;
# (2) SQ counters of the Pwelch kernels at the current sources (three --pmc
# passes); (3) kernel traces of the Noverlap 0 cases 64 / 128 / 512.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PW="2560:1280 2880:1440 3200:1600 3840:1920 4500:2250 6000:3000"
for r in 1 2; do
for L in default lib_s6a lib_s6b; do
  unset GDSP_LIB; [ $L = default ] || export GDSP_LIB=$R/go-dsp_amd/$L/libgdspfft.so
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_s6_$L.$r -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/s6_pw_$L.$r.log 2>&1; rc=$?
  echo "== pw $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/s6_pw_$L.$r.log; exit $rc; }
  python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_s6_$L.$r/run_kernel_trace.csv
  timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py 2560 2880 3200 3840 4500 6000 > $R/gpurun_out/r05/s6_fft_$L.$r.jsonl 2>&1; rc=$?
  echo "== fft $L $r rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/s6_fft_$L.$r.jsonl; exit $rc; }
done
done
unset GDSP_LIB
CASES="256:128 512:256 1024:512 2048:1024 4096:2048 8192:4096 16384:8192 256:0 1024:0 3000:1500 6000:3000"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F64"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $R/gpurun_out/sq_pwend_$i -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/sq_pwend_$i.log 2>&1; rc=$?
  echo "sq pass$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/sq_pwend_$i.log; exit $rc; }
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pw0 -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py 64:0 128:0 512:0 256:0 > $R/gpurun_out/r05/pw0.log 2>&1; rc=$?
echo "== pw0 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/pw0.log; exit $rc; }
python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pw0/run_kernel_trace.csv
cd $R && for f in gpurun_out/r05/s6_fft_*.jsonl; do echo "== $f"; cat $f; done
