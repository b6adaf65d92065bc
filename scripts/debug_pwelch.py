import importlib, os, sys
sys.path.insert(0, os.getcwd())
import torch
torch.cuda.set_device(0)
dev = importlib.import_module("go-dsp_amd.device")
gdsp = importlib.import_module("go-dsp_amd")
Dd = importlib.import_module("go-dsp_amd.distributed")
for total in [1 << 20, 1 << 26, 1 << 30]:
    nfft, nov = 4096, 2048
    x = torch.empty(total, dtype=torch.float64, device="cuda")
    dev.fill_uniform(x, 0x5EED)
    win = torch.tensor(gdsp.window.Hann(nfft), dtype=torch.float64, device="cuda")
    S = Dd.plan_pwelch(total, 1, 0, nfft, 0, nov).nsegs_total
    one = torch.zeros(nfft, dtype=torch.float64, device="cuda")
    dev.pwelch_accumulate(x, nfft, nfft, nov, 0, S, win, one)
    parts = []
    for r in range(2):
        s2 = Dd.plan_pwelch(total, 2, r, nfft, 0, nov)
        acc = torch.zeros(nfft, dtype=torch.float64, device="cuda")
        dev.pwelch_accumulate(x[s2.sample_lo:s2.sample_hi], nfft, nfft, nov, 0, s2.seg_hi - s2.seg_lo, win, acc)
        parts.append(acc)
        print(total, r, s2, float(acc.sum()), flush=True)
    torch.cuda.synchronize()
    print(total, "one", float(one.sum()), "sum parts", float(parts[0].sum() + parts[1].sum()), flush=True)
