# Round 5, after the radix-list changes: the whole GPU suite, then the batched
# FFT over every compiled specialisation's length and the smooth-NFFT Pwelch
# cases (rocprofv3 kernel traces).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_verify2.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify2.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
NS=$(python3 -c "
import re,glob
ns=[]
for f in sorted(glob.glob('$R/go-dsp_amd/csrc/fft_specs*.hip')):
    for m in re.finditer(r'Spec<([\d, ]+)>', open(f).read()):
        n=1
        for r in m.group(1).split(','): n*=int(r)
        ns.append(n)
print(' '.join(map(str,sorted(set(ns)))))")
timeout -k 10 300 python3 $R/scripts/bench_sizes_default.py $NS > $R/gpurun_out/r05/sizes_specs.jsonl 2>&1; rc=$?
echo "sizes rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
PW="480:240 800:400 1000:500 1200:600 1500:700 1536:768 2000:1000 2205:1102 2400:1200 2880:1440 3000:1500 3840:1920 4500:2250 6000:3000 8000:4000"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r05/prof_pwsmooth -o run --output-format csv -- python3 $R/scripts/bench_pwelch.py $PW > $R/gpurun_out/r05/pwsmooth.log 2>&1; rc=$?
echo "pw rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/r05/pwsmooth.log; exit $rc; }
python3 $R/tools/trace_cases.py $R/gpurun_out/r05/prof_pwsmooth/run_kernel_trace.csv
