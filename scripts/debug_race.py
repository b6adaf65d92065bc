import importlib, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
if os.environ.get("TORCH_FIRST"):
    import torch; torch.cuda.init()
sys.path.insert(0, "oracle"); import oracle
g = importlib.import_module("go-dsp_amd")
for n in [256, 1024, 4096, 16384, 3000]:
    errs = []
    for rep in range(6):
        rng = np.random.default_rng(n + rep)
        x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
        y = g.fft.FFTBatch(x)
        ref = oracle.fft_rows(x)
        errs.append([round(float(np.linalg.norm(a - b) / np.linalg.norm(b)), 3) for a, b in zip(y, ref)])
    print(os.environ.get("GDSP_DEBUG_COPY", "0"), os.environ.get("TORCH_FIRST", ""), n, errs, flush=True)
