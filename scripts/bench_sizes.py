#!/usr/bin/env python3
"""Throughput of fft.FFT on device-resident batches for a list of lengths,
default plan vs the forced chirp-z (reference algorithm) plan. HIP events on
one stream; ~2^28 complex samples per batch (capped). Prints one JSON line
per (n, plan)."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = importlib.import_module("go-dsp_amd.device")


def run(n, chirpz, samples=1 << 27, reps=10):
    batch = max(1, samples // n)
    x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
    D.fill_uniform(x, 0x5EED)
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    D.fft_batch(x, y, stream=s, chirpz=chirpz)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        D.fft_batch(x, y, stream=s, chirpz=chirpz)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"n": n, "batch": batch, "plan_kind": D.plan(n, chirpz).kind, "chirpz": chirpz,
            "ms": round(ms, 4), "gsamples_s": round(batch * n / ms / 1e6, 2),
            "alg_tb_s": round(32 * batch * n / ms / 1e9, 3)}


if __name__ == "__main__":
    torch.cuda.set_device(0)
    sizes = [int(a) for a in sys.argv[1:]] or [1000, 3000, 4096, 5000, 10000, 44100, 48000,
                                               65536, 1 << 20, 1000000]
    for n in sizes:
        for cz in (False, True):
            if cz and n & (n - 1) == 0:
                continue
            print(json.dumps(run(n, cz)), flush=True)
