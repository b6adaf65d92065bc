# Round 6 closing profile session, one stamp: SQ passes, rocprofv3 traces and
# stats, and the HBM PMC passes of all eight bench workloads.
set -o pipefail
R=$GRAFT_REPO_ROOT
W="radix4096 bluestein3000 chirpz3000 prime3001 pfa3027 fft2_8192 pwelch pwelch_default"
python3 $R/tools/source_stamp.py > $R/gpurun_out/source_stamp.json || exit 1
GDSP_JIT_CACHE=$R/gpurun_out/jitcache bash $R/scripts/gpu_sq.sh $W || exit 1
bash $R/scripts/gpu_r06_prof.sh stats || exit 1
bash $R/scripts/gpu_r06_prof.sh pmc "$W" || exit 1
# and the random sample of non-smooth lengths at the same sources
mkdir -p $R/gpurun_out/r06p
cd $R && GDSP_JIT_CACHE=$R/gpurun_out/jitcache timeout -k 10 500 python3 scripts/sweep_nonsmooth.py --no-chirpz --samples 67108864 $(cat scripts/nonsmooth_sample.txt) > gpurun_out/r06p/sample.jsonl 2> gpurun_out/r06p/sweep.err || exit 1
echo "sample sweep rc=0"
