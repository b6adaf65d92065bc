#!/usr/bin/env python3
"""Per-kernel average durations from a rocprofv3 kernel-trace CSV, in
dispatch order, grouping consecutive dispatches of one kernel name (so the
cases of a sweep script that reuse a kernel template show up separately).
Helper kernels (fills, torch elementwise, copies, the Pwelch partial-sum
reduce) are dropped before grouping, so a case's repeated calls stay one
group."""
import csv
import sys

HELPERS = ("fill_uniform", "elementwise", "copyBuffer", "reduce_partials")


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    groups = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:70]
        if any(h in name for h in HELPERS):
            continue
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if groups and groups[-1][0] == name:
            groups[-1][1].append(dur)
        else:
            groups.append((name, [dur]))
    for name, d in groups:
        warm = d[1:] if len(d) > 1 else d
        print(f"{name:72s} n={len(d):3d} avg_us={sum(warm) / len(warm):9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
