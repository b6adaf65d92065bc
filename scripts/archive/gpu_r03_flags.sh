# Compiler-flag variants of the whole library (go-dsp_amd/lib_vN, built with
# HIPCC="hipcc -mllvm <flag>") against the default build, alternating over
# the five bench workloads. Args: the variant directories (default lib_v1 lib_v2).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT/go-dsp_amd
LIBS="lib ${@:-lib_v1 lib_v2}"
for r in 1 2; do
for w in radix4096 bluestein3000 chirpz3000 pwelch fft2_8192; do
  for L in $LIBS; do
    GDSP_LIB=$R/$L/libgdspfft.so timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/ab.json 2> gpurun_out/ab.err; rc=$?
    [ $rc -eq 0 ] || { echo "$w $L rc=$rc"; tail -20 gpurun_out/ab.err; exit $rc; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));r=d['roofline'];print('$w','$L',d['ms_per_step'],r['avg_launch_ms'],r['frac'],(d.get('parity') or {}).get('max_nrel_vs_oracle'))"
  done
done
done
