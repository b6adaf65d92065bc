#!/usr/bin/env python3
"""Production-plan throughput of fft.FFT over a spread of lengths (powers of
2, compiled mixed-radix specialisations, runtime-radix lengths, primes and
large-prime-factor lengths that go through chirp-z, four-step lengths), one
JSON line per length: the map of where the dispatch is fast and where not."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_sizes  # noqa: E402

SIZES = [8, 64, 256, 1024, 2048, 4096, 8192, 16384, 1 << 16, 1 << 20,
         480, 1000, 1536, 3000, 3072,              # compiled specialisations
         100, 360, 800, 1001, 2187, 2500, 4000,    # runtime radices
         4095, 6000, 7919, 1009, 2053, 3001, 4099, 8191,  # chirp-z (primes / large factors)
         10000, 44100, 48000, 100000, 1000000]

if __name__ == "__main__":
    import torch
    torch.cuda.set_device(0)
    for n in [int(a) for a in sys.argv[1:]] or SIZES:
        print(json.dumps(bench_sizes.run(n, False)), flush=True)
