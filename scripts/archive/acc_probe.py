#!/usr/bin/env python3
"""Accuracy of the production plans against numpy's FFT (an exact DFT to
~1e-15) for the given lengths: normwise relative error per length, forward
and inverse. Diagnostic only (not a parity test: those use the oracle)."""
import importlib
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
for n in [int(a) for a in sys.argv[1:]]:
    rng = np.random.default_rng(n)
    b = max(1, 2000000 // n)
    x = rng.uniform(-1, 1, (b, n)) + 1j * rng.uniform(-1, 1, (b, n))
    ex = np.fft.fft(x, axis=1)
    y = g.fft.FFTBatch(x)
    yi = g.fft.FFTBatch(x, inverse=True)
    exi = np.fft.ifft(x, axis=1)
    e = float(np.max(np.linalg.norm(y - ex, axis=1) / np.linalg.norm(ex, axis=1)))
    ei = float(np.max(np.linalg.norm(yi - exi, axis=1) / np.linalg.norm(exi, axis=1)))
    print(json.dumps({"n": n, "batch": b, "kind": D.plan(n).kind, "fwd": e, "inv": ei}), flush=True)
