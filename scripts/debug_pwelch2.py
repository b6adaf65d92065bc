import importlib, os, sys
sys.path.insert(0, os.getcwd())
import torch
torch.cuda.set_device(0)
dev = importlib.import_module("go-dsp_amd.device")
gdsp = importlib.import_module("go-dsp_amd")
Dd = importlib.import_module("go-dsp_amd.distributed")
print("current stream", torch.cuda.current_stream(), torch.cuda.current_stream().cuda_stream, flush=True)
total, nfft, nov = 1 << 30, 4096, 2048
x = torch.empty(total, dtype=torch.float64, device="cuda")
dev.fill_uniform(x, 0x5EED)
win = torch.tensor(gdsp.window.Hann(nfft), dtype=torch.float64, device="cuda")
S = Dd.plan_pwelch(total, 1, 0, nfft, 0, nov).nsegs_total
for mode in ["nosync", "sync", "nosync", "sidestream"]:
    s = torch.cuda.Stream() if mode == "sidestream" else None
    ctx = torch.cuda.stream(s) if s is not None else torch.cuda.stream(torch.cuda.current_stream())
    with ctx:
        one = torch.zeros(nfft, dtype=torch.float64, device="cuda")
        dev.pwelch_accumulate(x, nfft, nfft, nov, 0, S, win, one)
        if mode == "sync": torch.cuda.synchronize()
        two = torch.zeros_like(one)
        if mode == "sync": torch.cuda.synchronize()
        for r in range(2):
            s2 = Dd.plan_pwelch(total, 2, r, nfft, 0, nov)
            dev.pwelch_accumulate(x[s2.sample_lo:s2.sample_hi], nfft, nfft, nov, 0, s2.seg_hi - s2.seg_lo, win, two)
            if mode == "sync": torch.cuda.synchronize()
    torch.cuda.synchronize()
    print(mode, float(one.sum()), float(two.sum()), flush=True)
