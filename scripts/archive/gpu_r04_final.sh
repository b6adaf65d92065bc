# Round-4 final: smoke + full GPU suite, then the default bench line (the
# driver's N = 1 command) with its one-line stdout check.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_r04_suite.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_final.err; exit $rc; }
python3 -c "
import json
l = open('gpurun_out/bench_final.json').read().splitlines()
assert len(l) == 1, l[:3]
d = json.loads(l[0])
print('stdout: one line;', d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['value'], v['ms_per_step']) for k, v in d['configs'].items()})
"
