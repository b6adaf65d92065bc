# Round 6: a Pwelch step's time beyond its kernel (scripts/bench_pwelch_step.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r06l
cd $R
for o in "--nfft 4096 --noverlap 2048" "--nfft 256 --noverlap 0"; do
  timeout -k 10 300 python3 scripts/bench_pwelch_step.py $o >> gpurun_out/r06l/step.jsonl 2> gpurun_out/r06l/step.err; rc=$?
  echo "step $o rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06l/step.err; exit $rc; }
done
cat gpurun_out/r06l/step.jsonl
