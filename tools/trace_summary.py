#!/usr/bin/env python3
"""Per-launch kernel durations of a rocprofv3 --kernel-trace run of bench.py
(gpurun_out/prof_<w>/run_kernel_trace.csv, scripts/gpu_stats_round.sh) ->
profiles/<tag>/<w>_kernel_trace.json: every kernel launched at least `min`
times, durations in ns in launch order, and "timed_last" = the bench's --steps
(the launches bench.py times are the last ones; the earlier are warm-up).

usage: tools/trace_summary.py <tag> <steps> <workload>...
"""
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def session_stamp():
    """The sources the profiled session ran on: gpurun_out/source_stamp.json,
    written on the GPU box by the session script (tools/source_stamp.py)."""
    p = os.path.join(REPO, "gpurun_out", "source_stamp.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def main(tag, steps, workloads):
    for w in workloads:
        path = os.path.join(REPO, "gpurun_out", f"prof_{w}", "run_kernel_trace.csv")
        rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
        d = defaultdict(list)
        for r in rows:
            d[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out = {"workload": w, "timed_last": steps,
               "source": f"rocprofv3 --kernel-trace of bench.py --workload {w} --steps {steps}",
               "stamp": session_stamp(),
               "kernels": {k: v for k, v in d.items() if len(v) >= steps}}
        dst = os.path.join(REPO, "profiles", tag, f"{w}_kernel_trace.json")
        with open(dst, "w") as f:
            json.dump(out, f)
        for k, v in out["kernels"].items():
            t = v[-steps:]
            print(f"{w}: {k[:60]} launches {len(v)}, last {steps} avg {sum(t) / len(t) / 1e6:.4f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3:])
