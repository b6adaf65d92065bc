# rocprofv3 kernel stats of fft2_8192 under env settings given as arguments
# ("default" or VAR=value[,VAR=value])
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for V in "$@"; do
  EV=""; [ "$V" = default ] || EV="${V//,/ }"
  N=$(echo "$V" | tr -c 'A-Za-z0-9\n' '_')
  env $EV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/f2_$N -o run --output-format csv -- python3 $R/bench.py --workload fft2_8192 --steps 20 --warmup 3 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/f2_$N.log 2>&1 || exit 1
  python3 - $R/gpurun_out/f2_$N <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if int(r["Calls"]) > 2:
        print(sys.argv[1].split("/")[-1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
