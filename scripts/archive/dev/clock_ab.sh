# Shader clock under load (GRBM_GUI_ACTIVE cycles / kernel duration) of one
# workload for the default library and alternates ($2...): is a variant's
# speed-up its clock?
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; W=$1; shift
for L in default "$@"; do
  unset GDSP_LIB; [ "$L" = default ] || export GDSP_LIB=$R/$L/libgdspfft.so
  N=$(basename $L)
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/clk_$N -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 5 --warmup 1 --cpu-seconds 0 --check-rows 0 > $R/gpurun_out/clk_$N.log 2>&1 || { tail -5 $R/gpurun_out/clk_$N.log; exit 1; }
  python3 - $R/gpurun_out/clk_$N <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cc = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
vals = collections.defaultdict(dict)
for r in csv.DictReader(open(cc)):
    vals[(r["Kernel_Name"][:40], r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for (k, i), m in sorted(vals.items(), key=lambda x: int(x[0][1])):
    if "fill" in k: continue
    g = m.get("GRBM_GUI_ACTIVE", 0); c = m.get("GRBM_COUNT", 0)
    print(d.split("/")[-1], k, i, "GUI_ACTIVE", int(g), "COUNT", int(c))
PY
done
