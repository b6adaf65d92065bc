#!/usr/bin/env python3
"""Where a Pwelch step's time goes beyond its kernel (bench.py's pwelch and
pwelch_default lines): per-step wall time and HIP-event time of (a) the
library accumulation alone, (b) + zeroing the accumulators, (c) + the host
copy, (d) the whole distributed.pwelch step, on 2^30 device-resident samples.

usage: bench_pwelch_step.py [--steps 20] [--nfft 4096 --noverlap 2048]
"""
import argparse
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--nfft", type=int, default=4096)
    ap.add_argument("--noverlap", type=int, default=2048)
    a = ap.parse_args()
    import torch
    g = importlib.import_module("go-dsp_amd")
    D = importlib.import_module("go-dsp_amd.device")
    Dd = importlib.import_module("go-dsp_amd.distributed")
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    total = 1 << 30
    sh = Dd.plan_pwelch(total, 1, 0, a.nfft, 0, a.noverlap)
    x = torch.empty(sh.sample_hi - sh.sample_lo, dtype=torch.float64, device="cuda")
    D.fill_uniform(x, 7, stream=s)
    opts = g.spectral.PwelchOptions(NFFT=a.nfft, Noverlap=a.noverlap)
    nfft, pad, nov, wf, _ = g.spectral.resolve_options(opts)
    win = Dd._device_window(wf, sh.flen, x.device, torch)
    acc = torch.zeros(sh.flen, dtype=torch.float64, device="cuda")

    def acc_only():
        D.pwelch_accumulate(x, sh.nfft, sh.pad, sh.noverlap, 0, sh.seg_hi - sh.seg_lo, win, acc,
                            stream=s)

    def zero_acc():
        with torch.cuda.stream(s):
            acc.zero_()
        acc_only()

    def zero_acc_copy():
        zero_acc()
        with torch.cuda.stream(s):
            acc.cpu()

    def full():
        Dd.pwelch(x, 1.0, opts, sh, stream=s)

    out = {"nfft": a.nfft, "noverlap": a.noverlap}
    for name, f in (("accumulate", acc_only), ("zero+accumulate", zero_acc),
                    ("zero+accumulate+copy", zero_acc_copy), ("distributed.pwelch", full)):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.steps)]
        t0 = time.perf_counter()
        for e0, e1 in ev:
            e0.record(s)
            f()
            e1.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps * 1e3
        evm = sum(e0.elapsed_time(e1) for e0, e1 in ev) / a.steps
        out[name] = {"wall_ms": round(wall, 4), "event_ms": round(evm, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
