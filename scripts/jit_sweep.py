#!/usr/bin/env python3
"""Every 13-smooth length in [2, 8192] that is not a power of 2: plan kind,
plan-build time (runtime compilation included) and the forward / inverse /
real-input error against the oracle, one JSON line per length, plus a
summary line. A sweep of the runtime-compiled specialisations' radix
chooser and kernels beyond the parity suite's samples."""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")


# SWEEP23=1: the lengths whose largest prime factor is 17..31 instead
BIG = (17, 19, 23, 29, 31)
PRIMES = (2, 3, 5, 7, 11, 13) + (BIG if os.environ.get("SWEEP23") else ())


def smooth(n):
    for p in PRIMES:
        while n % p == 0:
            n //= p
    return n == 1


def nrel(y, r):
    return max(float(np.linalg.norm(a - b) / np.linalg.norm(b)) for a, b in zip(y, r))


if __name__ == "__main__":
    # "--lengths n ...": exactly those lengths (e.g. the ones whose radix list
    # a chooser change moved); else [lo, hi] (default 2 .. 8192)
    listed = [int(a) for a in sys.argv[2:]] if sys.argv[1:2] == ["--lengths"] else None
    lo, hi = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 and not listed else (2, 8192)
    rng = np.random.default_rng(1)
    worst, count, kinds, t_build = 0.0, 0, {}, 0.0
    for n in listed or range(lo, hi + 1):
        if not listed and (not smooth(n) or n & (n - 1) == 0 or (os.environ.get("SWEEP23") and all(
                n % p for p in BIG))):
            continue
        t0 = time.perf_counter()
        k = D.plan(n).kind
        dt = time.perf_counter() - t0
        t_build += dt
        x = rng.uniform(-1, 1, (2, n)) + 1j * rng.uniform(-1, 1, (2, n))
        e = max(nrel(g.fft.FFTBatch(x), oracle.fft_rows(x)),
                nrel(g.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)),
                nrel(g.fft.FFTRealBatch(x.real.copy()), oracle.fft_rows(x.real.astype(complex))))
        worst = max(worst, e)
        count += 1
        kinds[k] = kinds.get(k, 0) + 1
        print(json.dumps({"n": n, "kind": k, "plan_s": round(dt, 3), "err": e}), flush=True)
    print(json.dumps({"summary": True, "lengths": count, "kinds": kinds, "worst_err": worst,
                      "plan_build_s_total": round(t_build, 1)}), flush=True)
    sys.exit(0 if worst < 1e-9 else 1)
