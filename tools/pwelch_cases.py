#!/usr/bin/env python3
"""Per-case Pwelch kernel times from rocprofv3 kernel traces of
scripts/bench_pwelch.py (gpurun_out/r05/prof_pwcases.<round>/, one warm-up and
five timed calls per case, helper kernels dropped) -> one JSON line per case:
the accumulation kernel, its per-round averages over the timed calls, and
2^28 x 8 B over the average against 8 TB/s. "before" = the round's start
(profiles/r05/pwelch_nfft_cases_start.json, where that case was measured).

usage: tools/pwelch_cases.py <out.jsonl> <cases...> (cases as nfft:noverlap)
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPERS = ("fill_uniform", "elementwise", "copyBuffer", "reduce_partials")


def per_case(path, ncases):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"].split("(")[0].replace("void ", ""),
           (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
          for r in rows if not any(h in r["Kernel_Name"] for h in HELPERS)]
    assert len(ks) == 6 * ncases, (path, len(ks))
    return [(ks[6 * i][0], sum(d for _, d in ks[6 * i + 1:6 * i + 6]) / 5) for i in range(ncases)]


def main(out, cases):
    paths = sorted(glob.glob(os.path.join(REPO, "gpurun_out", "r05", "prof_pwcases.*",
                                          "run_kernel_trace.csv")))
    runs = [per_case(p, len(cases)) for p in paths]
    start = {}
    sp = os.path.join(REPO, "profiles", "r05", "pwelch_nfft_cases_start.json")
    if os.path.exists(sp):
        start = json.load(open(sp))
    with open(out, "w") as f:
        for i, c in enumerate(cases):
            nfft, nov = map(int, c.split(":"))
            us = [r[i][1] for r in runs]
            avg = sum(us) / len(us)
            line = {"nfft": nfft, "noverlap": nov, "samples": 1 << 28, "kernel": runs[0][i][0],
                    "kernel_us": [round(u, 1) for u in us],
                    "hbm_frac_8tbs": round((8 << 28) / (avg * 1e-6) / 8e12, 3)}
            if c in start:
                line["round_start"] = start[c]
            f.write(json.dumps(line) + "\n")
            print(f"{c:>11s} {line['kernel'][:48]:48s} {line['kernel_us']} {line['hbm_frac_8tbs']}"
                  f" start={start.get(c, {}).get('us')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
