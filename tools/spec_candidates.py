#!/usr/bin/env python3
"""Candidate radix lists for the compiled mixed-radix specialisations
(fft_specs*.hip), ranked by a lane-occupancy cost model, for an A/B on the
GPU (scripts/archive/gpu_r05_specd.sh).

A pass of radix R over n points has n/R butterflies; FixedGeo gives every
transform T1 = max over passes of ceil((n/R) / jm) threads (jm = 16/R
butterflies per thread for R <= 16), so a pass with fewer butterflies than
T1 leaves lanes idle. The model charges each pass its DFT cost per point
(F64 instructions of dft_any<R>, counted by hand from mixed_core.hpp) plus
the twiddle chain (passes after the first), divided by the pass's lane use.
It is only a ranking for what to measure: round 5's measurements (2880,
3200, 3840, 4500 faster by 10-38 %) motivated it, and 6000 (model 0.76x,
Pwelch measured 1.0x) shows its limits.

usage: tools/spec_candidates.py [k]   -> for each spec, the current list and
the k best other lists with as many passes.
"""
import itertools
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
RADICES = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 20, 25]
DFT = {2: 2.0, 3: 4.7, 4: 4.0, 5: 7.2, 6: 8.0, 7: 9.4, 8: 6.5, 9: 11.1, 10: 10.8, 11: 13.6,
       12: 10.7, 13: 15.7, 15: 14.0, 16: 9.4, 20: 13.6, 25: 17.0}


def need(n, r):
    nb = n // r
    jm = 1 if r > 16 else 16 // r
    return -(-nb // jm), -(-nb // jm) * 0 + nb, jm


def cost(n, rad):
    needs = []
    for r in rad:
        nb = n // r
        jm = 1 if r > 16 else 16 // r
        needs.append((nb, -(-nb // jm)))
    t1 = max(q for _, q in needs)
    if t1 > 512:
        return None
    c = 0.0
    for p, (r, (nb, q)) in enumerate(zip(rad, needs)):
        jj = -(-nb // t1)  # butterflies per thread (loop count)
        use = nb / (jj * t1)
        w = DFT[r] + (8.0 * (r - 1) / r if p > 0 else 0.0)
        c += w / use
    return c, t1


def lists(n, npass):
    def rec(m, k):
        if k == 0:
            if m == 1:
                yield []
            return
        for r in RADICES:
            if m % r == 0:
                for rest in rec(m // r, k - 1):
                    yield [r] + rest
    yield from rec(n, npass)


def specs():
    out = []
    for f in sorted((ROOT / "go-dsp_amd" / "csrc").glob("fft_specs*.hip")):
        for line in f.read_text().splitlines():
            m = re.search(r"Spec<([\d, ]+)>", line)
            if m:
                rad = [int(x) for x in m.group(1).split(",")]
                out.append((f.name, rad))
    return out


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    for fname, rad in specs():
        n = 1
        for r in rad:
            n *= r
        cur = cost(n, rad)
        alts = []
        for cand in lists(n, len(rad)):
            if cand == rad:
                continue
            c = cost(n, cand)
            if c:
                alts.append((c[0], c[1], cand))
        alts.sort(key=lambda a: (a[0], -a[2][-1] & (a[2][-1] - 1) == 0))
        best = ", ".join(f"{'.'.join(map(str, a[2]))} ({a[0]:.1f}, T1 {a[1]})" for a in alts[:k])
        print(f"{fname} {n}: {'.'.join(map(str, rad))} ({cur[0]:.1f}, T1 {cur[1]}) | {best}")


if __name__ == "__main__":
    main()
