# forced chirp-z throughput over a list of lengths for alternate library
# builds ($1: space-separated library dirs or "default"), $2 rounds, rest = n
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
LIBS=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for L in $LIBS; do
    unset GDSP_LIB; [ "$L" = default ] || export GDSP_LIB=$GRAFT_REPO_ROOT/$L/libgdspfft.so
    timeout -k 10 300 python scripts/bench_sizes.py "$@" > gpurun_out/cz_sizes.json 2> gpurun_out/cz_sizes.err || { tail -5 gpurun_out/cz_sizes.err; exit 1; }
    python3 -c "
import json,sys
rows=[json.loads(l) for l in open('gpurun_out/cz_sizes.json') if l.strip()]
print('$L', ' '.join(f\"{r['n']}:{r['ms']}\" for r in rows if r['chirpz']))"
  done
done
