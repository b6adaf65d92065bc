#!/usr/bin/env python3
"""Prime-factor Rader (plan kind 8) against the chirp-z plan it replaces, on a
stratified sample of the composites it takes: for each cofactor M = 2 ... 32
with an in-register DFT, up to --per lengths n = M * P <= 8192 (P > 31 prime,
gcd(M, P) = 1, P - 1 25-smooth), spread over P. One JSON line per n: the
Rader list of P - 1, kind-8 and chirp-z kernel times (HIP events, ~2^26
complex128 samples per batch), fractions of 8 TB/s. The data behind the
kind-8 cost rule (gdsp_api.hip pfa_rader_try).

usage: sweep_pfa_calib.py [--per 5] [--samples 2^26] [n ...]"""
import argparse
import importlib
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
D = importlib.import_module("go-dsp_amd.device")
F = importlib.import_module("go-dsp_amd.fft")


def factor(n):
    f, d = [], 2
    while d * d <= n:
        while n % d == 0:
            f.append(d)
            n //= d
        d += 1
    if n > 1:
        f.append(n)
    return f


def smooth(n, b):
    return n == 1 or max(factor(n)) <= b


def candidates(per):
    nat = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 17, 19, 20, 23, 25, 29, 31, 32}
    def ok_m(m):
        if m in nat:
            return True
        return any(m % r == 0 and r in nat and (m // r) in nat and gcd(r, m // r) == 1
                   for r in range(2, m))
    from math import gcd
    out = []
    for M in range(2, 33):
        if not ok_m(M):
            continue
        ps = [p for p in range(37, 8192 // M + 1) if factor(p) == [p] and smooth(p - 1, 25)
              and M % p and max(factor(M)) < p]
        if not ps:
            continue
        k = min(per, len(ps))
        out += [M * ps[round(i * (len(ps) - 1) / max(1, k - 1))] for i in range(k)]
    return sorted(set(out))


def timed(x, y, chirpz, reps):
    s = torch.cuda.Stream()
    for _ in range(2):
        D.fft_batch(x, y, stream=s, chirpz=chirpz)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        D.fft_batch(x, y, stream=s, chirpz=chirpz)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per", type=int, default=5)
    ap.add_argument("--samples", type=int, default=1 << 26)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-race", action="store_true",
                    help="the kind-8 kernel itself (GDSP_ALGO_NO_RACE), not the race's choice")
    ap.add_argument("sizes", nargs="*", type=int)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    if a.no_race:
        F.SetAlgorithm(F.ALGO_NO_RACE)
    for n in a.sizes or candidates(a.per):
        batch = max(1, a.samples // n)
        x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
        D.fill_uniform(x, 0x5EED + n)
        y = torch.empty_like(x)
        p = D.plan(n)
        rec = {"n": n, "kind": p.kind, "m1": p.n1, "p": p.n2, "radices": list(p.radices)}
        ms = timed(x, y, False, a.reps)
        cz = timed(x, y, True, a.reps)
        gb = 32 * batch * n / 1e6
        rec.update({"ms": round(ms, 4), "frac": round(gb / ms / 8000, 4),
                    "chirpz_ms": round(cz, 4), "chirpz_frac": round(gb / cz / 8000, 4),
                    "chirpz_m": D.plan(n, True).m, "speedup": round(cz / ms, 3)})
        print(json.dumps(rec), flush=True)
        del x, y


if __name__ == "__main__":
    main()
