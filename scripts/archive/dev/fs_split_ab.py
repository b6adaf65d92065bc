#!/usr/bin/env python3
"""Four-step row length vs batch for power-of-2 n > 16384: time fft.FFT on a
device-resident (batch, n) for the row length set by GDSP_FS_LC (read per
call by exec_fourstep), alternating settings, HIP events on one stream.
Usage: fs_split_ab.py log2n:batch[,...]  (prints one JSON line per case)."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
D = importlib.import_module("go-dsp_amd.device")


def timed(x, y, s, reps):
    D.fft_batch(x, y, stream=s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        D.fft_batch(x, y, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    for case in sys.argv[1:]:
        ln, batch = (int(v) for v in case.split(":"))
        n = 1 << ln
        x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
        D.fill_uniform(x, 0x5EED)
        y = torch.empty_like(x)
        lcs = [lc for lc in range(8, 14) if 4 <= ln - lc <= 9]
        ref = None
        res = {lc: [] for lc in lcs}
        for rnd in range(3):
            for lc in lcs:
                os.environ["GDSP_FS_LC"] = str(lc)
                res[lc].append(timed(x, y, s, 50 if batch * n <= 1 << 22 else 10))
                os.environ.pop("GDSP_FS_LC")
                y0 = y.clone()
                if ref is None:
                    ref = y0
                err = ((y0 - ref).abs().max() / ref.abs().max()).item()
                assert err < 1e-12, (ln, lc, err)
        print(json.dumps({"log2n": ln, "batch": batch,
                          "ms": {lc: [round(v, 4) for v in res[lc]] for lc in lcs}}), flush=True)
