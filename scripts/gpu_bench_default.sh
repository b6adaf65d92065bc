# The driver's default bench line (N=1, nested configs), then a 2-rank gloo
# rehearsal of the N>1 path on the box's one GPU (strong + weak + configs).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_default.err; exit $rc; }
if [ "${1:-}" = rehearse ]; then
  GDSP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 1 --cpu-seconds 0 --batch 16384 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err; rc=$?
  echo "rehearse rc=$rc"; cat gpurun_out/rehearse2.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearse2.err; exit $rc; }
fi
