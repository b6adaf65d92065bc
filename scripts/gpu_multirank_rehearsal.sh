# N>1 rehearsal on a 1-GPU box: 2 ranks share cuda:0 over gloo (RCCL needs one
# GPU per rank). Exercises sharding, barriers, max-over-ranks timing and the
# Pwelch all-reduce of bench.py / go-dsp_amd/distributed.py.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for w in radix4096 pwelch fft2_dist; do
  GDSP_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --workload $w --steps 5 --warmup 1 --batch 16384 > gpurun_out/rehearse_$w.json 2> gpurun_out/rehearse_$w.err; rc=$?
  echo "== $w rc=$rc"; cat gpurun_out/rehearse_$w.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/rehearse_$w.err; exit $rc; }
done
