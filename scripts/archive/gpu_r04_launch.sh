# Round 4: bench.py's own multi-rank launcher on the 1-GPU box, and the
# multi-device tests (8 Pwelch shards on device 0, grouped RCCL reduce).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multi.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04_multi.log 2>&1; rc=$?
echo "multi rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04_multi.log | tail -20; [ $rc -eq 0 ] || exit $rc
# nccl with fewer GPUs than ranks must refuse (exit 2, no line)
timeout -k 10 120 python3 bench.py --gpus 2 > gpurun_out/r04_nccl2.json 2> gpurun_out/r04_nccl2.err; rc=$?
echo "nccl --gpus 2 rc=$rc (want 2): $(cat gpurun_out/r04_nccl2.err | tail -1)"; [ $rc -eq 2 ] || exit 1
# gloo rehearsal through the plain command (no torch.distributed.run)
for w in radix4096 pwelch; do
  GDSP_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --workload $w --batch 16384 --steps 5 --warmup 1 > gpurun_out/r04_gloo2_$w.json 2> gpurun_out/r04_gloo2_$w.err; rc=$?
  echo "gloo2 $w rc=$rc"; cat gpurun_out/r04_gloo2_$w.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04_gloo2_$w.err; exit $rc; }
done
