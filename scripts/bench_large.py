# BenchmarkFFT's size (fft/fft_test.go:262-280): one N=2^20 transform, and a
# batch of 64, through the device API (four-step path).
import importlib, os, sys, time
sys.path.insert(0, os.getcwd())
import torch
torch.cuda.set_device(0)
D = importlib.import_module("go-dsp_amd.device")
for n, batch in [(1 << 20, 1), (1 << 20, 64), (1 << 17, 256), (1 << 24, 4)]:
    x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
    D.fill_uniform(x, 1)
    y = torch.empty_like(x)
    for _ in range(3):
        D.fft_batch(x, y)
    torch.cuda.synchronize()
    t = time.perf_counter(); reps = 20
    for _ in range(reps):
        D.fft_batch(x, y)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(f"n=2^{n.bit_length()-1} batch={batch}: {dt*1e3:.3f} ms  {32*n*batch/dt/1e9:.0f} GB/s alg", flush=True)
