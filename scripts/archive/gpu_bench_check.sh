set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench_default.json'))
print('head',d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])
for k,v in d['configs'].items(): print(k,v['ms_per_step'],v['roofline']['avg_launch_ms'],v['roofline']['frac'],v['cpu_baseline']['value'])"
for w in pwelch fft2_8192; do timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/s.json || exit 1; python -c "
import json;d=json.load(open('gpurun_out/s.json'));print('$w alone',d['ms_per_step'],d['roofline']['avg_launch_ms'])"; done
