#!/bin/bash
# The 1/2/4/8-GPU curve of the BASELINE metric on one node: `bench.py --gpus N`
# (it starts the N rank processes itself, one per GPU, RCCL) for every N the
# node has GPUs for, each step under its own time limit, stopping at the first
# failure. Lines go to gpurun_out/scale/bench_gpus<N>.json, and the
# multi-device parity tests (tests/test_multi.py: the in-library RCCL clique
# and the torch-nccl world of N ranks, against the oracle) run first.
# Usage: scripts/gpu_scale.sh [steps] [warmup]
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
STEPS=${1:-20}
WARM=${2:-3}
OUT=gpurun_out/scale
mkdir -p "$OUT"
NDEV=$(python3 -c "import importlib.util as u, sys; s=u.spec_from_file_location('b','bench.py'); b=u.module_from_spec(s); s.loader.exec_module(b); print(b._device_count())")
echo "GPUs: $NDEV" | tee "$OUT/ndev.txt"
timeout -k 10 900 python3 -u -m pytest tests/test_multi.py -m gpu -x -v --timeout 600 \
    --timeout-method thread > "$OUT/pytest_multi.log" 2>&1 || { echo "multi tests failed"; exit 1; }
for N in 1 2 4 8; do
  [ "$N" -le "$NDEV" ] || break
  timeout -k 10 900 python3 bench.py --gpus "$N" --steps "$STEPS" --warmup "$WARM" \
      > "$OUT/bench_gpus$N.json" 2> "$OUT/bench_gpus$N.err" || { echo "N=$N failed"; exit 1; }
  cat "$OUT/bench_gpus$N.json"
done
