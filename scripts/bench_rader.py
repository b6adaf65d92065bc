#!/usr/bin/env python3
"""Primes through Rader's algorithm (plan kind 7) against the chirp-z plan
the same prime takes with GDSP_ALGO_NO_RADER (kind 3: the fused chirp-z, M =
6144 / 3072 where it applies, else NextPowerOf2(2n - 1)). Device-resident
batches of ~2^27 samples, HIP events on one stream, ms per batch after
warm-up. One JSON line per prime."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = importlib.import_module("go-dsp_amd.device")
F = importlib.import_module("go-dsp_amd.fft")


def timed(n, x, y, s, reps=10):
    for _ in range(3):
        D.fft_batch(x, y, stream=s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        D.fft_batch(x, y, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def run(n, samples=1 << 27):
    batch = max(1, samples // n)
    x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
    D.fill_uniform(x, 0x5EED)
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    out = {"n": n, "batch": batch, "kind": D.plan(n).kind}
    ms = timed(n, x, y, s)
    yr = y[:4].clone()
    out.update(ms=round(ms, 4), alg_tb_s=round(32 * batch * n / ms / 1e9, 3))
    F.SetAlgorithm(F.ALGO_NO_RADER)
    try:
        out["kind_chirpz"] = D.plan(n).kind
        out["m_chirpz"] = D.plan(n).m
        mc = timed(n, x, y, s)
    finally:
        F.SetAlgorithm(0)
    out.update(ms_chirpz=round(mc, 4), alg_tb_s_chirpz=round(32 * batch * n / mc / 1e9, 3),
               speedup=round(mc / ms, 3))
    out["max_rel_diff"] = float(((yr - y[:4]).abs().max() / y[:4].abs().max()).item())
    return out


if __name__ == "__main__":
    torch.cuda.set_device(0)
    primes = [int(a) for a in sys.argv[1:]] or [
        17, 37, 97, 101, 257, 641, 1009, 1201, 1531, 2053, 2311, 2729, 3001, 4001, 4801, 6007,
        7681, 8009, 8191]
    for n in primes:
        print(json.dumps(run(n)), flush=True)
