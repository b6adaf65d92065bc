#!/usr/bin/env python3
"""Median per-launch counter values of gpurun_out/pmc_<tag>/ runs, per kernel
(experiments; scripts/gpu_pmc_pass.sh). usage: tools/pmc_print.py tag [...]"""
import csv, glob, os, statistics, sys
from collections import defaultdict
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for tag in sys.argv[1:]:
    vals = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(REPO, "gpurun_out", "pmc_" + tag, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0]
            if "fill_uniform" in k or "rocclr" in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", tag)
    for k, d in vals.items():
        print("  ", k[:70])
        for c, v in sorted(d.items()):
            print("      %-32s %.4g" % (c, statistics.median(v)))
