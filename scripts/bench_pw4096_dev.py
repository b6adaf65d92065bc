#!/usr/bin/env python3
"""NFFT 4096 / 50 % Pwelch accumulation of a 2^30-sample HBM stream (BASELINE
configs[4]) on the product row kernel and on the development build's
rejected kernels (pwelch_row3.hip: three workgroups per CU; pwelch_shfl.hip),
each run 8 times. Meant to run under rocprofv3 --kernel-trace with GDSP_LIB
pointing at the development build (tools/trace_cases.py summarises the
kernels); also prints the event time per call and the oracle check on the
first 2^22 samples."""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
L = g._lib.lib()
assert g._lib.is_dev_build(), "run with GDSP_LIB=go-dsp_amd/lib_dev/libgdspfft.so"
P = lambda t: ctypes.c_void_p(t.data_ptr())

torch.cuda.set_device(0)
n = 1 << 30
x = torch.empty(n, dtype=torch.float64, device="cuda")
D.fill_uniform(x, 0x5EED)
w = torch.tensor(np.asarray(g.window.Hann(4096), np.float64), device="cuda")
S = g.spectral.segment_count(n, 4096, 2048)
acc = torch.zeros(4096, dtype=torch.float64, device="cuda")


def product():
    D.pwelch_accumulate(x, 4096, 4096, 2048, 0, S, w, acc)


def dev(name):
    fn = getattr(L, name)
    return lambda: fn(P(x), n, 0, S, P(w), P(acc), None)


for label, f in (("product", product), ("row3", dev("gdsp_dev_pwelch4096_row3_accumulate")),
                 ("shfl", dev("gdsp_dev_pwelch4096_shfl_accumulate"))):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(8):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"kernel": label, "ms_per_call": round(e0.elapsed_time(e1) / 8, 4)}), flush=True)
