# The driver's multi-GPU command shape (torch.distributed.run, one rank per
# GPU) rehearsed with gloo on the box's one GPU: default bench line at N = 2.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
GDSP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/torchrun_default_2.json 2> gpurun_out/torchrun_default_2.err; rc=$?
echo "torchrun N=2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/torchrun_default_2.err; exit $rc; }
python3 -c "import sys; l=open('gpurun_out/torchrun_default_2.json').read().splitlines(); assert len(l) == 1, l[:3]; print('stdout: one line')" && cat gpurun_out/torchrun_default_2.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['n_gpus'],d['value'],d['ms_per_step'],d['scaling'],d['config']['parallelism'],{k:v['value'] for k,v in d['configs'].items()})"
# N = 1, the driver's single-GPU command: stdout must be the one JSON line
timeout -k 10 300 python bench.py --workload radix4096 --steps 3 --warmup 1 --cpu-seconds 0 \
  > gpurun_out/n1_radix4096.json 2> gpurun_out/n1_radix4096.err; rc=$?
echo "N=1 rc=$rc"; [ $rc -eq 0 ] || { tail -30 gpurun_out/n1_radix4096.err; exit $rc; }
python3 -c "import json; l=open('gpurun_out/n1_radix4096.json').read().splitlines(); assert len(l) == 1, l[:3]; d=json.loads(l[0]); print('N=1 stdout: one line', d['n_gpus'], d['value'], d['ms_per_step'])"
