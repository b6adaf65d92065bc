"""Diagnose the NFFT 4096 half-overlap Pwelch accumulator against a numpy
reference of the packed-pair sums (experiments; GPU)."""
import importlib, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
D = importlib.import_module("go-dsp_amd.device")
g = importlib.import_module("go-dsp_amd")
F = 4096
for nseg in (2, 3, 8):
    n = (nseg - 1) * 2048 + F
    rng = np.random.default_rng(nseg)
    x = rng.standard_normal(n)
    w = np.array(g.window.Hann(F))
    acc = torch.zeros(F, dtype=torch.float64, device="cuda")
    D.pwelch_accumulate(torch.from_numpy(x).cuda(), F, F, 2048, 0, nseg, torch.from_numpy(w).cuda(), acc)
    a = acc.cpu().numpy()
    ref = np.zeros(F)
    for p in range(0, nseg, 2):
        s0 = x[p * 2048:p * 2048 + F] * w
        s1 = x[(p + 1) * 2048:(p + 1) * 2048 + F] * w if p + 1 < nseg else np.zeros(F)
        ref += np.abs(np.fft.fft(s0 + 1j * s1)) ** 2
    err = np.abs(a - ref) / np.abs(ref).max()
    bad = np.nonzero(err > 1e-10)[0]
    print(nseg, "maxerr", err.max(), "nbad", len(bad), "first bad", bad[:12])
    if len(bad):
        # is a[k] some permutation of ref?
        idx = [int(np.argmin(np.abs(ref - a[k]))) for k in bad[:12]]
        print("   matches ref bins", idx)
