#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer API (the cgo boundary) on the
BASELINE shapes: fft.FFTBatch on a host complex128 array (65 536 x 4096 and
65 536 x 3000: H2D through the library's pinned staging, the kernel, D2H),
and spectral.Pwelch on a host 2^30-sample float64 stream (H2D only). Never
the bench's `value`, which is HBM-resident."""
import importlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
g = importlib.import_module("go-dsp_amd")


def timed(f, reps):
    f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return (time.perf_counter() - t0) / reps


out = {}
for n in (4096, 3000):
    x = (np.random.default_rng(n).standard_normal((65536, n))
         + 1j * np.random.default_rng(n + 1).standard_normal((65536, n)))
    s = timed(lambda: g.fft.FFTBatch(x), 3)
    out[f"fft_batch_65536x{n}"] = {"s": round(s, 4), "gsamples_s": round(65536 * n / s / 1e9, 3),
                                   "bytes_over_pcie": 2 * x.nbytes,
                                   "pcie_gb_s": round(2 * x.nbytes / s / 1e9, 2)}
    # the same C-ABI call into an output the host has already touched (a Go
    # slice from make() is zeroed, so its pages are resident): without the
    # first-touch page faults of a fresh numpy array
    y = np.zeros_like(x)
    F = importlib.import_module("go-dsp_amd.fft")
    s = timed(lambda: F.check(F.lib().gdsp_fft_batch(F._p(x), F._p(y), n, 65536, 0), "fft_batch"), 3)
    out[f"fft_batch_65536x{n}_resident_out"] = {"s": round(s, 4),
                                                "gsamples_s": round(65536 * n / s / 1e9, 3),
                                                "pcie_gb_s": round(2 * x.nbytes / s / 1e9, 2)}
    del x, y
x = np.random.default_rng(7).uniform(-1, 1, 1 << 30)
o = g.spectral.PwelchOptions(NFFT=4096, Noverlap=2048)
s = timed(lambda: g.spectral.Pwelch(x, 1.0, o), 3)
out["pwelch_2p30_nfft4096"] = {"s": round(s, 4), "gsamples_s": round((1 << 30) / s / 1e9, 3),
                               "bytes_over_pcie": x.nbytes, "pcie_gb_s": round(x.nbytes / s / 1e9, 2)}
print(json.dumps(out))
