#!/usr/bin/env python3
"""Batched fft.FFT over lengths that are not 31-smooth (the reference sends
every non-power-of-2 n to Bluestein, fft/fft.go:82-86 -> fft/bluestein.go:
68-94): ~2^27 complex128 samples per batch, device-resident, HIP events on one
stream. For each n, the production plan (kind, ms, Gsamples/s, fraction of
8 TB/s at 32 B per sample) and the forced chirp-z plan (gdsp_plan_create_chirpz,
the reference's algorithm) on the same batch, plus the production output's
oracle error on sampled rows (forward) and the round trip. One JSON line per n.

usage: sweep_nonsmooth.py [--samples 2^27] [n ...]   (default: the list below)
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
D = importlib.import_module("go-dsp_amd.device")

# composites with a prime factor > 31 (P - 1 smooth and not), primes whose
# p - 1 is not smooth, and primes Rader already takes (for reference)
DEFAULT = [74, 111, 222, 370, 481, 518, 606, 742, 1111, 1202, 1261, 1406, 1507, 1622, 1833,
           2062, 2167, 2222, 2419, 2626, 2798, 3027, 3131, 3334, 3502, 3737, 3894, 4058, 4097,
           4402, 4981, 5402, 6011, 6122, 6666, 7006, 7474, 8006, 8186,
           1031, 2039, 3299, 4099, 6143, 7919, 3001, 1201]


def timed(n, x, y, chirpz, reps):
    s = torch.cuda.Stream()
    D.fft_batch(x, y, stream=s, chirpz=chirpz)
    torch.cuda.synchronize()
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
    ap.add_argument("--samples", type=int, default=1 << 27)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-chirpz", action="store_true")
    ap.add_argument("sizes", nargs="*", type=int)
    a = ap.parse_args()
    import oracle
    torch.cuda.set_device(0)
    for n in a.sizes or DEFAULT:
        batch = max(1, a.samples // n)
        x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
        D.fill_uniform(x, 0x5EED + n)
        y = torch.empty_like(x)
        p = D.plan(n)
        ms = timed(n, x, y, False, a.reps)
        rows = np.linspace(0, batch - 1, 4).astype(int)
        ref = oracle.fft_rows(x[rows].cpu().numpy())
        got = y[rows].cpu().numpy()
        nrel = max(float(np.linalg.norm(g - r) / np.linalg.norm(r)) for g, r in zip(got, ref))
        z = D.fft_batch(y, inverse=True)
        rt = float((torch.linalg.vector_norm(z - x, dim=1) /
                    torch.linalg.vector_norm(x, dim=1)).max())
        del z
        rec = {"n": n, "batch": batch, "plan_kind": p.kind, "m": p.m, "n1": p.n1, "n2": p.n2,
               "ms": round(ms, 4), "gsamples_s": round(batch * n / ms / 1e6, 2),
               "frac": round(32 * batch * n / ms / 1e6 / 8000.0, 4),
               "nrel_vs_oracle": nrel, "roundtrip_nrel": rt}
        if not a.no_chirpz:
            cz = timed(n, x, y, True, a.reps)
            rec.update({"chirpz_ms": round(cz, 4),
                        "chirpz_frac": round(32 * batch * n / cz / 1e6 / 8000.0, 4),
                        "speedup_vs_chirpz": round(cz / ms, 3)})
        print(json.dumps(rec), flush=True)
        del x, y


if __name__ == "__main__":
    main()
