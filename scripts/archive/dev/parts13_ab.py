"""GDSP_BLU_PARTS13 experiment: lengths in (4096, 5461] whose chirp-z runs on
M = 16384, as one convolution of 16384 or two parts on M = 8192. Parity of
the current process's plans against the oracle, then ms per 2^27 samples."""
import importlib, json, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import oracle
D = importlib.import_module("go-dsp_amd.device")
from bench_sizes import run
torch.cuda.set_device(0)
rng = np.random.default_rng(5)
for n in [int(a) for a in sys.argv[1:]]:
    p = D.plan(n)
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    xt = torch.from_numpy(x).cuda()
    err = 0.0
    for inv in (False, True):
        y = D.fft_batch(xt, inverse=inv).cpu().numpy()
        ref = oracle.ifft_rows(x) if inv else oracle.fft_rows(x)
        err = max(err, max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref)))
    assert err < 1e-9, (n, err)
    r = run(n, False)
    r.update(m=p.m, parts=p.parts, err=err)
    print(json.dumps(r), flush=True)
