# Pwelch NFFT 8192 (half overlap): the row kernel against pwelch_half_kernel<13>
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "pwelch" > gpurun_out/pw13_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc $(tail -1 gpurun_out/pw13_pytest.log)"; [ $rc -eq 0 ] || { grep -E "^FAILED|assert" gpurun_out/pw13_pytest.log | head; exit $rc; }
DEV=$GRAFT_REPO_ROOT/go-dsp_amd/lib_dev/libgdspfft.so
for r in 1 2; do
  timeout -k 10 120 python scripts/bench_pwelch.py 8192:4096 4096:2048 | sed "s/^/row /"
  GDSP_LIB=$DEV GDSP_PW13_HALF=1 timeout -k 10 120 python scripts/bench_pwelch.py 8192:4096 | sed "s/^/half /"
done
