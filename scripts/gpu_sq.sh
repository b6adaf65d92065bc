# SQ/LDS/VALU counters of the bench workloads (what binds the compute-heavy
# kernels): three --pmc passes per workload, kernel counters only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_SALU"
P3="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F64"
for W in ${@:-radix4096 bluestein3000 chirpz3000 pwelch fft2_8192}; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/gpurun_out/sq_${W}_$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 --check-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/sq_${W}_$i.log 2>&1; rc=$?
    echo "sq $W pass$i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/sq_${W}_$i.log; exit $rc; }
  done
done
