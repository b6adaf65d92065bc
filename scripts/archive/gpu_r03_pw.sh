# Round 3: Pwelch row kernel parity + A/B against the round-2 kernel, then
# the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "pwelch or multi or smoke" > gpurun_out/r03_pytest_pw.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r03_pytest_pw.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh pwelch "default go-dsp_amd/lib_pwold go-dsp_amd/lib_pwl0" 3 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_default.err; exit $rc; }
