# Round 5, after the runtime-compiled radix chooser's lane-cost rule: the whole
# GPU suite; every smooth length whose list the rule changed (127) forward,
# inverse and real input against the oracle (scripts/jit_sweep.py --lengths);
# the batched FFT and fused Pwelch of the DESIGN.md JIT-table lengths it moved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r05
export GDSP_JIT_CACHE=$GRAFT_REPO_ROOT/gpurun_out/jitcache
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/pytest_verify3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r05/pytest_verify3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u scripts/jit_sweep.py --lengths 36 50 72 75 80 144 252 280 288 420 450 510 522 525 540 550 558 570 576 650 675 684 690 700 792 810 825 828 855 864 975 1035 1044 1116 1275 1300 1425 1550 1575 1584 1638 1656 1725 1728 1872 1960 2016 2040 2088 2100 2232 2280 2304 2320 2340 2394 2448 2480 2610 2700 2736 2790 2808 3100 3150 3240 3276 3312 3375 3400 3420 3456 3675 3680 3800 3850 3906 3960 3978 4032 4080 4104 4140 4176 4200 4275 4284 4464 4560 4608 4760 4830 5100 5670 5850 6050 6075 6174 6210 6264 6480 6552 6600 6624 6696 6912 7020 7038 7056 7245 7254 7290 7308 7344 7425 7488 7600 7605 7700 7812 7830 7866 7920 7956 8064 8120 8160 > gpurun_out/r05/jit_sweep_changed.jsonl 2>&1; rc=$?
echo "sweep rc=$rc"; tail -1 gpurun_out/r05/jit_sweep_changed.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_sizes_default.py 810 7290 7600 > gpurun_out/r05/jit_table_sizes.jsonl 2>&1; rc=$?
echo "sizes rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat gpurun_out/r05/jit_table_sizes.jsonl
