"""Experiment: production chirp-z primes in (2048, 3072] on the wave kernel
with M = 6144 (GDSP_BLU_WAVE=1 GDSP_BLU_M6144=1) against the oracle, and
timing at 2^27 samples (GPU)."""
import importlib, os, sys
import numpy as np, torch
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "oracle"))
import oracle
D = importlib.import_module("go-dsp_amd.device")
for n in (2053, 2741, 3001, 3067):
    p = D.plan(n)
    x = np.random.default_rng(n).standard_normal((3, n)) + 1j * np.random.default_rng(n + 1).standard_normal((3, n))
    y = D.fft_batch(torch.from_numpy(x).cuda()).cpu().numpy()
    ref = oracle.fft_rows(x)
    err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
    batch = (1 << 27) // n
    xt = torch.empty((batch, n), dtype=torch.complex128, device="cuda"); D.fill_uniform(xt, 1)
    yt = torch.empty_like(xt)
    s = torch.cuda.Stream(); D.fft_batch(xt, yt, stream=s); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10): D.fft_batch(xt, yt, stream=s)
    e1.record(s); torch.cuda.synchronize()
    print(n, "m", p.m, "q", p.wave_q, "err %.2e" % err, "ms %.3f" % (e0.elapsed_time(e1) / 10), flush=True)
