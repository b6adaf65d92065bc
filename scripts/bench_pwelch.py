#!/usr/bin/env python3
"""Device Pwelch throughput for a list of (NFFT, Noverlap) on a 2^28-sample
HBM-resident stream (gdsp_pwelch_accumulate_device + finalize through
distributed.pwelch at world size 1). One JSON line per case."""
import importlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
gdsp = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
Dd = importlib.import_module("go-dsp_amd.distributed")

CASES = [(64, 32), (128, 0), (256, 0), (256, 128), (512, 256), (1024, 0), (1024, 512), (2048, 0),
         (2048, 1024), (4096, 0), (4096, 2048), (4096, 1024), (8192, 4096), (16384, 8192),
         (1000, 500), (3000, 1500)]

if __name__ == "__main__":
    torch.cuda.set_device(0)
    total = 1 << 28
    x = torch.empty(total, dtype=torch.float64, device="cuda")
    D.fill_uniform(x, 0x5EED)
    s = torch.cuda.Stream()
    cases = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or CASES  # "nfft:nov"
    for nfft, nov in cases:
        o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov)
        sh = Dd.plan_pwelch(total, 1, 0, nfft, 0, nov)
        Dd.pwelch(x, 1.0, o, sh, stream=s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            Dd.pwelch(x, 1.0, o, sh, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(json.dumps({"nfft": nfft, "noverlap": nov, "segments": sh.nsegs_total,
                          "ms": round(ms, 3), "gsamples_s": round(total / ms / 1e6, 1),
                          "hbm_tb_s": round(8 * total / ms / 1e9, 3)}), flush=True)
