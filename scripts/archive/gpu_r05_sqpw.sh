# Round 5: SQ counters of the Pwelch kernels per NFFT case (what binds the
# half-overlap wave kernels), three --pmc passes over scripts/bench_pwelch.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export GDSP_JIT_CACHE=$R/gpurun_out/jitcache
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F64"
CASES="256:128 512:256 1024:512 2048:1024 4096:0 4096:2048 1000:500 3000:1500"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $R/gpurun_out/sq_pwcases_$i -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $CASES > $R/gpurun_out/sq_pwcases_$i.log 2>&1; rc=$?
  echo "sq pass$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/sq_pwcases_$i.log; exit $rc; }
done
