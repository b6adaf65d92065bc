#!/usr/bin/env python3
"""Per-2^27-sample time of the two-pass smooth-row plan for each admissible
row length C (GDSP_MXROW_C, development build) of a few n: which C the rule
should pick. One JSON line per (n, C) plus the default plan's choice."""
import json
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = os.path.join(R, "go-dsp_amd", "lib_dev", "libgdspfft.so")


def smooth(m, primes=(2, 3, 5, 7, 11, 13)):
    for p in primes:
        while m % p == 0:
            m //= p
    return m == 1


def run(n, c=None):
    env = dict(os.environ)
    if c:
        env.update(GDSP_LIB=DEV, GDSP_MXROW_C=str(c))
    out = subprocess.run([sys.executable, os.path.join(R, "scripts", "bench_sizes_default.py"), str(n)],
                         env=env, capture_output=True, text=True, timeout=120)
    return json.loads(out.stdout.strip().splitlines()[-1])["ms"] if out.returncode == 0 else None


for n in [int(a) for a in sys.argv[1:]]:
    cs = [c for c in range(16, 1025) if n % c == 0 and c & (c - 1) and n // c >= 64 and smooth(c)]
    if len(cs) > 8:
        step = len(cs) / 8
        cs = sorted(set(cs[int(i * step)] for i in range(8)) | {max(cs)})
    print(json.dumps({"n": n, "C": "default", "ms": run(n)}), flush=True)
    for c in cs:
        print(json.dumps({"n": n, "C": c, "L": n // c, "ms": run(n, c)}), flush=True)
