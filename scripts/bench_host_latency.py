#!/usr/bin/env python3
"""Latency of the synchronous host-pointer API (the cgo path): one fft.FFT
call on a host vector, H2D + kernel + D2H, for a few lengths; and the
reference restatement on one host thread for scale."""
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

for n in (8, 1024, 4096, 3000, 65536, 1 << 20):
    x = np.random.default_rng(n).standard_normal(n) + 0j
    g.fft.FFT(x)
    reps = 200 if n <= 65536 else 20
    t0 = time.perf_counter()
    for _ in range(reps):
        g.fft.FFT(x)
    dt = (time.perf_counter() - t0) / reps
    t1 = time.perf_counter()
    for _ in range(max(1, reps // 10)):
        oracle.fft(x)
    dc = (time.perf_counter() - t1) / max(1, reps // 10)
    print(json.dumps({"n": n, "gpu_call_us": round(dt * 1e6, 1),
                      "cpu_restatement_us": round(dc * 1e6, 1)}), flush=True)
