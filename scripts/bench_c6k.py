#!/usr/bin/env python3
"""Forced chirp-z per 2^27 samples on the M = 3 * 2^k kernel (chirpz6k.hip,
default) against the reference's power-of-2 M (GDSP_ALGO_CHIRPZ_POW2), for
the lengths given (default: both ranges' ends and primes). One JSON line per
length: ms per 2^27 samples for each, alternating three times."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = importlib.import_module("go-dsp_amd.device")
F = importlib.import_module("go-dsp_amd.fft")


def once(x, y, s, reps=10):
    D.fft_batch(x, y, stream=s, chirpz=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        D.fft_batch(x, y, stream=s, chirpz=True)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    torch.cuda.set_device(0)
    sizes = [int(a) for a in sys.argv[1:]] or [1025, 1201, 1531, 2053, 2503, 3001]
    s = torch.cuda.Stream()
    for n in sizes:
        batch = (1 << 27) // n
        x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
        D.fill_uniform(x, 0x5EED)
        y = torch.empty_like(x)
        res = {"n": n, "batch": batch, "m": [], "ms_c6": [], "ms_pow2": []}
        for _ in range(3):
            for flags, key in ((0, "ms_c6"), (F.ALGO_CHIRPZ_POW2, "ms_pow2")):
                F.SetAlgorithm(flags)
                try:
                    res[key].append(round(once(x, y, s), 4))
                    if len(res["m"]) < 2:
                        res["m"].append(D.plan(n, chirpz=True).m)
                finally:
                    F.SetAlgorithm(0)
        print(json.dumps(res), flush=True)
        del x, y
        torch.cuda.empty_cache()
