#!/usr/bin/env python3
"""Benchmark of the go-dsp hot path on MI355X (BASELINE.json metric:
"Gsamples/s + % HBM roofline, batched N=4096 complex128 FFT at 1/2/4/8 GPUs").

A step = one batched transform over one HBM-resident batch of synthetic
input (configs[1]: N = 4096 complex128 x 65536 rows). Multi-GPU: one process
per GPU, started either by torch.distributed.run (WORLD_SIZE must then equal
--gpus) or, for a plain `python bench.py --gpus N`, by this script itself (N
rank processes spawned before anything touches a GPU; with the nccl backend it
exits non-zero when the node has fewer than N GPUs, GDSP_DIST_BACKEND=gloo
rehearses N ranks on one GPU); the 65536 rows are split over the ranks
(strong scaling; no data-path collective: the rows are
independent). value = 2^28 samples / max-over-ranks wall time; at N > 1 a
weak-scaling figure (65536 rows per rank) is added as "weak_scaling".

The default run also times the other BASELINE configs and nests them under
"configs": bluestein3000, chirpz3000, prime3001 and pfa3027 (configs[2]; the prime
n = 3001 and the composite 3027 = 3 x 1009 through the production dispatch: Rader,
and the prime-factor Rader kernel, each with its chirp-z plan timed beside it),
fft2_8192 (configs[3];
rows sharded with two RCCL all-to-alls at N > 1) and pwelch (configs[4]; one
RCCL all-reduce of the PSD accumulators). --workload X runs one alone.
bluestein3000 is fft.FFT of N = 3000 through the production dispatch (the
compiled mixed-radix 25*15*8 kernel); chirpz3000 times the same workload through the
reference's algorithm (forced Bluestein plan, gdsp_plan_create_chirpz), whose
convolution runs on M = 6144 (chirpz6k.hip); the same line carries the time on the
reference's M = 8192 (GDSP_ALGO_CHIRPZ_POW2) as "reference_m8192".

roofline.achieved = algorithmic bytes of one launch (32 B/sample: 16 B read +
16 B written) / the launch's average duration, measured with
HIP events on the stream the kernel runs on. roofline.traffic = HBM bytes per
launch from the committed rocprofv3 PMC summary (profiles/), or null.
cpu_baseline = the reference algorithm's CPU restatement (oracle/, test
infrastructure) with the reference's worker-pool structure, timed on a bounded
row sample on rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: measured float4 copy rate (BASELINE.md:33)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector spec (tools/fp64peak.hip measures 67.3 FMA-only)
# kernels whose FP64 work is taken from the committed SQ counter passes
# (profiles/r02/sq_counters.json: 64 x (2 FMA + ADD + MUL) F64 instructions)
SQ_KERNELS = {"radix4096": ["fft_lds_kernel<12"], "bluestein3000": ["fft_mixed_fixed_kernel"],
              "prime3001": ["rader_fixed_kernel"], "pfa3027": ["rader_pfa_kernel"],
              "chirpz3000": ["chirpz6k_kernel"], "pwelch": ["pwelch_row_kernel<12"],
              "pwelch_default": ["pwelch_wave_kernel<8"],
              "fft2_8192": ["fft_lds_kernel<13", "colfft_tile_kernel<6", "colfft_tile_kernel<7"],
              "fft2_dist": ["fft_lds_kernel<13", "colfft_tile_kernel<6", "colfft_tile_kernel<7"]}
SQ_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # SQ counter passes quoted: the newest round that has the kernel
# rocprofv3 --kernel-trace --stats summaries quoted beside the event timing
# (profiles/<round>/<workload>_kernel_stats.csv, the closing session's runs of
# `bench.py --workload <w>`): the newest round that has the workload
STATS_ROUNDS = ("r06", "r05", "r04", "r03", "r02")
SEED = 0x5EED
WARM_S = 0.06  # untimed GPU work before the timed steps (steady clocks; measure())
# algorithmic bytes of one launch in the N=1 full-size configuration the
# committed PMC (profiles/pmc_*.json) and SQ (profiles/r02/sq_counters.json)
# summaries were measured on
PROFILED_ALG_BYTES = {"radix4096": 32 * 4096 * 65536, "bluestein3000": 32 * 3000 * 65536,
                      "chirpz3000": 32 * 3000 * 65536, "prime3001": 32 * 3001 * 65536,
                      "pfa3027": 32 * 3027 * 65536,
                      "fft2_8192": 4 * 16 * 8192 * 8192,
                      "fft2_dist": 4 * 16 * 8192 * 8192, "pwelch": 8 * (1 << 30),
                      "pwelch_default": 8 * (1 << 30),
                      "fftn_512": 3 * 2 * 16 * 512 ** 3, "wav_decode": 10 * (1 << 30),
                      "fft_2p20": 32 * (1 << 20)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="default",
                    choices=["default"] + WORKLOADS,
                    help="default: the headline radix4096 line with the other BASELINE "
                         "configs nested under 'configs'")
    ap.add_argument("--batch", type=int, default=0,
                    help="rows in total, split over the ranks (0 = config default 65536)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU seconds for the headline cpu_baseline sample (0 disables)")
    ap.add_argument("--config-cpu-seconds", type=float, default=5.0,
                    help="target CPU seconds for each nested config's cpu_baseline")
    ap.add_argument("--check-rows", type=int, default=8, help="rows checked against the oracle")
    return ap.parse_args()


WORKLOADS = ["radix4096", "bluestein3000", "chirpz3000", "prime3001", "pfa3027", "fft2_8192",
             "fft2_dist",
             "pwelch", "pwelch_default",
             "fftn_512", "wav_decode", "fft_2p20", "fftreal1024"]
# the BASELINE configs nested in the default line: configs[2] (production
# dispatch and the reference's chirp-z algorithm), configs[3], configs[4]
NESTED = ["bluestein3000", "chirpz3000", "prime3001", "pfa3027", "fft2_8192", "pwelch",
          "pwelch_default", "fftreal1024"]
HEADLINE_METRIC = "Gsamples/s + % HBM roofline, batched N=4096 complex128 FFT at 1/2/4/8 GPUs"


class Ctx:
    """Process-wide run context: ranks, device, stream, modules."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.args = torch, dist, args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # GDSP_DIST_BACKEND=gloo rehearses the N>1 path with several ranks on
        # one GPU (RCCL refuses two ranks per device); production runs use nccl=RCCL
        self.backend = os.environ.get("GDSP_DIST_BACKEND", "nccl")
        if self.world > 1:
            ndev = torch.cuda.device_count()
            err = rank_device_check(ndev, local, self.backend, dict(os.environ), self.world)
            if err:
                raise SystemExit(f"bench.py: {err}")
            torch.cuda.set_device(local % ndev)
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local % ndev))
            else:
                dist.init_process_group(self.backend)
        else:
            torch.cuda.set_device(0)
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.gdsp = importlib.import_module("go-dsp_amd")
        self.D = importlib.import_module("go-dsp_amd.device")
        self.Dd = importlib.import_module("go-dsp_amd.distributed")
        self.stream = torch.cuda.Stream(self.dev)
        # the sources this run executes (tools/source_stamp.py), printed in the
        # line and compared with the stamps of the profiles it quotes
        sys.path.insert(0, os.path.join(REPO, "tools"))
        import source_stamp
        self.stamp = source_stamp.stamp()

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()


def setup(w: str, c: Ctx, weak: bool = False) -> dict:
    """Inputs in HBM and the step of workload w. Batched FFTs are strong
    scaling: the 65536 rows are split over the ranks (the
    reference's own benchmark is fixed-work, fft/fft_test.go:262-280);
    weak=True gives every rank the full 65536 rows instead."""
    torch, D, Dd, dev, stream, rank, world = c.torch, c.D, c.Dd, c.dev, c.stream, c.rank, c.world
    if w in ("radix4096", "bluestein3000", "chirpz3000", "prime3001", "pfa3027"):
        n = {"radix4096": 4096, "prime3001": 3001, "pfa3027": 3027}.get(w, 3000)
        chirpz = w == "chirpz3000"
        total = c.args.batch or 65536
        if weak:
            lo, hi, total = rank * total, (rank + 1) * total, total * world
        else:
            lo, hi = Dd.shard_range(total, world, rank)
        x = torch.empty((hi - lo, n), dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        D.fill_uniform(x, SEED, offset=lo * n * 2, stream=stream)
        p = D.plan(n, chirpz)
        kind = p.kind

        def step():
            D.fft_batch(x, y, stream=stream, chirpz=chirpz)

        algo = {1: "Stockham radix-16 (one kernel)", 3: "Bluestein chirp-z (fused, M=8192)",
                5: "mixed-radix Stockham 25*15*8 (one compiled kernel)",
                7: f"Rader (cyclic convolution of length {n - 1} = 25*15*8, two FFTs in one "
                   "runtime-compiled kernel; the reference: Bluestein, M=8192)",
                8: f"prime-factor Rader ({n} = {p.n1} x {p.n2}: DFT_{p.n1} per column, {p.n1} "
                   f"Rader transforms of {p.n2} on a {p.n2 - 1}-point convolution "
                   f"({'*'.join(map(str, p.radices))}), one runtime-compiled kernel; the "
                   "reference: Bluestein, M=8192)"}.get(kind, str(kind))
        kernel = {1: "fft_lds_kernel<12>", 3: "bluestein_kernel<13>",
                  5: "fft_mixed_fixed_kernel<25,15,8>",
                  7: "rader_fixed_kernel", 8: "rader_pfa_kernel"}.get(kind, str(kind))
        if kind == 3 and p.m == 6144:
            # 2817 <= n <= 3072: the convolution on M = 6144 (chirpz6k.hip);
            # bluestein.go:70 pads to 8192 (GDSP_ALGO_CHIRPZ_POW2 keeps it)
            algo = "Bluestein chirp-z (fused, M=6144=16*24*16; the reference pads to 8192)"
            kernel = "chirpz6k_kernel"
        return dict(step=step, x=x, y=y, total_samples=total * n, rank_samples=(hi - lo) * n,
                    alg_bytes=32 * (hi - lo) * n, kernel=kernel, metric=HEADLINE_METRIC,
                    scaling="weak" if weak else "strong",
                    cfg={"workload": f"fft.FFT batched complex128 N={n} x {total} rows"
                                     + (" per GPU" if weak else ", split over the GPUs"),
                         "n": n, "batch_total": total, "batch_per_gpu": hi - lo,
                         "parallelism": f"rows{world}", "algorithm": algo})
    if w == "fft2_8192" and world == 1:
        rows = cols = 8192
        x = torch.empty((rows, cols), dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        work = torch.empty_like(x)
        D.fill_uniform(x, SEED, stream=stream)

        def step():
            D.fft2(x, y, work=work, stream=stream)

        return dict(step=step, x=x, y=y, total_samples=rows * cols, rank_samples=rows * cols,
                    alg_bytes=2 * 2 * 16 * rows * cols, kernel="fft2 (all launches)",
                    metric="Gsamples/s, fft.FFT2 8192x8192 complex128", scaling="strong",
                    cfg={"workload": "fft.FFT2 complex128 8192x8192", "rows": rows,
                         "cols": cols, "parallelism": "rows1"})
    if w in ("fft2_8192", "fft2_dist"):
        # one 8192^2 FFT2 with its rows sharded over the ranks (strong)
        R = C = 8192
        lo, hi = Dd.shard_range(R, world, rank)
        x = torch.empty((hi - lo, C), dtype=torch.complex128, device=dev)
        D.fill_uniform(x, SEED, offset=lo * C * 2, stream=stream)
        result = {}

        def step():
            result["y"] = Dd.fft2_sharded(x, R, stream=stream)

        return dict(step=step, total_samples=R * C, rank_samples=x.numel(),
                    alg_bytes=2 * 2 * 16 * x.numel(),
                    kernel="fft2_sharded (all launches and both all-to-alls)",
                    metric="Gsamples/s, fft.FFT2 8192x8192 complex128", scaling="strong",
                    cfg={"workload": "fft.FFT2 complex128 8192x8192, rows sharded over the "
                                     "ranks (row FFTs, RCCL all-to-all, column FFTs, "
                                     "all-to-all back)",
                         "rows": R, "cols": C, "parallelism": f"rows{world}+alltoall"})
    if w == "fft_2p20":  # the reference's own BenchmarkFFT (fft/fft_test.go:262-280)
        n = 1 << 20
        c.gdsp.fft.EnsureRadix2Factors(n)  # as BenchmarkFFT does (fft_test.go:273)
        x = torch.empty((1, n), dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        D.fill_uniform(x, SEED, offset=rank * n * 2, stream=stream)

        def step():
            D.fft_batch(x, y, stream=stream)

        return dict(step=step, x=x, y=y, total_samples=n * world, rank_samples=n,
                    alg_bytes=32 * n, kernel="four-step (colfft tile, row FFTs, transpose)",
                    metric="Gsamples/s, fft.FFT N=2^20 (BenchmarkFFT)", scaling="weak",
                    cfg={"workload": "fft.FFT of one N=2^20 complex128 vector (BenchmarkFFT, "
                                     "fft/fft_test.go:262-280), device-resident", "n": n,
                         "batch": 1, "parallelism": f"replicas{world}",
                         "algorithm": "four-step (3 launches)"})
    if w == "fftn_512":  # fft.FFTN of a 512^3 complex128 Matrix
        dims = (512, 512, 512)
        x = torch.empty(dims, dtype=torch.complex128, device=dev)
        y = torch.empty_like(x)
        D.fill_uniform(x, SEED, offset=rank * x.numel() * 2, stream=stream)

        def step():
            D.fftn(x, y, stream=stream)

        return dict(step=step, total_samples=x.numel() * world, rank_samples=x.numel(),
                    alg_bytes=3 * 2 * 16 * x.numel(),  # each axis: one read + one write
                    kernel="fftn (all launches: rows, then two column-tile axes)",
                    metric="Gsamples/s, fft.FFTN 512^3 complex128", scaling="weak",
                    cfg={"workload": "fft.FFTN complex128 512x512x512 (computeFFTN, "
                                     "fft.go:157-192)", "dims": list(dims),
                         "parallelism": f"replicas{world}"})
    if w == "wav_decode":  # wav.ReadFloats -> float64 Pwelch input
        wav = importlib.import_module("go-dsp_amd.wav")
        count = 1 << 30
        raw = torch.empty(2 * count, dtype=torch.uint8, device=dev)
        # synthetic PCM16 little-endian samples: the bytes of a uniform stream
        u = torch.empty(count // 4, dtype=torch.float64, device=dev)
        D.fill_uniform(u, SEED, offset=rank * count, stream=stream)
        torch.cuda.synchronize()
        raw.view(torch.float64).copy_(u)
        del u
        y = torch.empty(count, dtype=torch.float64, device=dev)

        def step():
            wav.device_floats(raw, count, 1, 16, out=y, stream=stream)

        return dict(step=step, raw=raw, y=y, total_samples=count * world, rank_samples=count,
                    alg_bytes=10 * count,  # 2 B PCM16 in, 8 B float64 out
                    kernel="wav_decode_vec_kernel<16, f64>", dtype="pcm16 -> f64",
                    metric="Gsamples/s, wav.ReadFloats PCM16 2^30 samples", scaling="weak",
                    cfg={"workload": "wav.ReadFloats PCM16 -> float64 Pwelch input, 2^30 "
                                     "samples (wav.go:135-161)", "samples": count,
                         "format": "PCM16", "parallelism": f"replicas{world}"})
    # pwelch: 2^30 samples total, NFFT 4096, 50 % overlap, Hann (strong
    # scaling); pwelch_default: the same stream with the reference's
    # PwelchOptions{} defaults, NFFT 256, Noverlap 0, Pad = NFFT, Hann
    # (spectral/pwelch.go:85-95), what pwelch_test.go and every zero-valued
    # options caller get
    nfft, nov = (256, 0) if w == "pwelch_default" else (4096, 2048)
    total = 1 << 30
    sh = Dd.plan_pwelch(total, world, rank, nfft, 0, nov)
    x = torch.empty(sh.sample_hi - sh.sample_lo, dtype=torch.float64, device=dev)
    D.fill_uniform(x, SEED, offset=sh.sample_lo, stream=stream)
    opts = c.gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov)
    result = {}

    def step():
        result["pxx"], _ = Dd.pwelch(x, 1.0, opts, sh, stream=stream)

    if w == "pwelch_default":
        return dict(step=step, x=x, shard=sh, opts=opts, result=result, total_samples=total,
                    rank_samples=total // world,
                    alg_bytes=8 * x.numel(), kernel="pwelch_wave_kernel<8, false, false>",
                    metric="Gsamples/s, spectral.Pwelch 2^30 samples, PwelchOptions{} defaults "
                           "(NFFT 256, Noverlap 0)",
                    scaling="strong",
                    cfg={"workload": "spectral.Pwelch 2^30-sample stream, the reference's "
                                     "default options: Hann NFFT 256, Noverlap 0, Pad 256",
                         "segments_total": sh.nsegs_total,
                         "parallelism": f"segments{world}+allreduce"})
    return dict(step=step, x=x, shard=sh, opts=opts, result=result, total_samples=total,
                rank_samples=total // world,
                alg_bytes=8 * x.numel(), kernel="pwelch_row_kernel<12>",
                metric="Gsamples/s, spectral.Pwelch 2^30 samples NFFT 4096 50% overlap",
                scaling="strong",
                cfg={"workload": "spectral.Pwelch 2^30-sample stream, Hann NFFT 4096, 50% "
                                 "overlap", "segments_total": sh.nsegs_total,
                     "parallelism": f"segments{world}+allreduce"})


def measure(wl: dict, c: Ctx) -> dict:
    """W untimed warm-up steps, then exactly K timed steps between barrier +
    synchronize; wall time = max over ranks. Per-step HIP events on the
    stream the kernels run on give the average launch duration."""
    torch, args = c.torch, c.args
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        wl["step"]()
    torch.cuda.synchronize()
    # Steady state: the first launches of a run are up to 30 % slower while
    # the chip's clocks ramp (rocprofv3 per-launch traces, profiles/r04/
    # *_kernel_trace.json: chirp-z 2.64-3.00 ms for the first launches, 2.28-2.33
    # from the tenth on). After the W warm-up steps, further untimed steps run
    # until about WARM_S of GPU work has passed since the start (the same count
    # on every rank: collectives run inside some steps). Reported as
    # "warmup_steps_run".
    t1 = time.perf_counter()
    wl["step"]()
    torch.cuda.synchronize()
    est = max(time.perf_counter() - t1, 1e-6)
    extra = min(200, max(0, int(WARM_S / est) - args.warmup - 1))
    if c.world > 1:
        t = torch.tensor([extra], dtype=torch.int64, device=c.dev if c.backend == "nccl" else "cpu")
        c.dist.all_reduce(t, op=c.dist.ReduceOp.MAX)
        extra = int(t.item())
    for _ in range(extra):
        wl["step"]()
    torch.cuda.synchronize()
    wl["warmup_steps_run"] = args.warmup + 1 + extra
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    c.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        starts[i].record(c.stream)
        wl["step"]()
        ends[i].record(c.stream)
    torch.cuda.synchronize()
    # each rank's clock stops when its own GPU work is done; the closing
    # barrier's latency (an RCCL round trip at N > 1) is not step time, and
    # the max over ranks below is the slowest rank's finish
    elapsed = time.perf_counter() - t0
    c.barrier()
    if c.world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=c.dev if c.backend == "nccl" else "cpu")
        c.dist.all_reduce(t, op=c.dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ev_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    return {"elapsed": elapsed, "avg_launch_s": sum(ev_ms) / len(ev_ms) / 1e3}


def parity(w: str, wl: dict, c: Ctx):
    """Untimed spot check of this run's output against the oracle (rank 0)."""
    if c.rank != 0 or c.args.check_rows <= 0:
        return None
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle
    if w in ("radix4096", "bluestein3000", "chirpz3000", "prime3001", "pfa3027"):
        x, y = wl["x"], wl["y"]
        rows = np.linspace(0, y.shape[0] - 1, c.args.check_rows).astype(int)
        xs, ys = x[rows].cpu().numpy(), y[rows].cpu().numpy()
        ref = oracle.fft_rows(xs)
        err = max(float(np.linalg.norm(a - b) / np.linalg.norm(b)) for a, b in zip(ys, ref))
        return {"rows": len(rows), "max_nrel_vs_oracle": err}
    if w == "fft_2p20":
        ref = oracle.fft(wl["x"][0].cpu().numpy())
        got = wl["y"][0].cpu().numpy()
        return {"rows": 1, "max_nrel_vs_oracle": float(np.linalg.norm(got - ref) /
                                                         np.linalg.norm(ref))}
    if w == "wav_decode":
        m = 1 << 20
        ref = oracle.wav_floats(wl["raw"][:2 * m].cpu().numpy().tobytes(), m, 1, 16)
        got = wl["y"][:m].cpu().numpy()
        return {"samples": m, "bit_exact": bool(np.array_equal(got, ref.astype(np.float64)))}
    if w == "fft2_8192" and "y" in wl:
        return parity_fft2(wl, np, oracle)
    if w in ("pwelch", "pwelch_default"):
        return parity_pwelch(wl, c, np, oracle)
    return None


def parity_fft2(wl: dict, np, oracle) -> dict:
    """Whole output rows of this run's 8192^2 FFT2 against the oracle
    (fft/fft_test.go:148-162 pins the same transform at 2x3 / 3x5): output
    row k1 is FFT_C(sum_r x[r, :] e^{-2 pi i k1 r / R}) (computeFFT2,
    fft/fft.go:123-154, column DFT then row DFT), so the column sum is taken
    in float64 on the host and the row FFT by the oracle; plus five single
    bins as direct 2-D DFT sums, error / sqrt(R C)."""
    x, y = wl["x"], wl["y"]
    R, C = x.shape
    xr = x.cpu().numpy()
    r = np.arange(R)
    rows = [0, 1, 1234, R - 1]
    nrel = 0.0
    for k1 in rows:
        col = np.exp(-2j * np.pi * ((k1 * r) % R) / R) @ xr
        ref = oracle.fft(col)
        got = y[k1].cpu().numpy()
        nrel = max(nrel, float(np.linalg.norm(got - ref) / np.linalg.norm(ref)))
    c = np.arange(C)
    bins = [(0, 0), (1, 0), (0, 1), (1234, 4321), (8191, 17)]
    berr = 0.0
    for k1, k2 in bins:
        want = np.exp(-2j * np.pi * ((k1 * r) % R) / R) @ (
            xr @ np.exp(-2j * np.pi * ((k2 * c) % C) / C))
        berr = max(berr, abs(complex(y[k1, k2].item()) - want) / np.sqrt(R * C))
    return {"rows": len(rows), "max_nrel_vs_oracle": nrel, "bins": len(bins),
            "max_bin_err_over_sqrt_RC": float(berr),
            "check": "output rows 0, 1, 1234, 8191 = oracle.fft of the float64 column DFT; "
                     "5 bins as direct 2-D DFT sums"}


def parity_pwelch(wl: dict, c: Ctx, np, oracle) -> dict:
    """This run's Pwelch path against the oracle (spectral/pwelch_test.go:31-46
    pins the same function on 100 samples): the first 2^22 samples of the
    same HBM stream through the same device accumulate + finalize as the
    timed step and through the host C ABI (gdsp.spectral.Pwelch), each vs
    oracle.pwelch; plus the timed full-size Pxx itself (finite, 2049 bins,
    the white uniform[-1,1) stream's level 2/3 at Fs = 1)."""
    Dd, spectral = c.Dd, c.gdsp.spectral
    sh, opts = wl["shard"], wl["opts"]
    pre = 1 << 22
    x = wl["x"]
    if sh.sample_lo != 0 or x.numel() < pre:
        return None
    nfft, nov = sh.nfft, sh.noverlap
    xp = x[:pre]
    host = xp.cpu().numpy()
    ref, _ = oracle.pwelch(host, 1.0, nfft=nfft, noverlap=nov)
    sp = Dd.plan_pwelch(pre, 1, 0, nfft, 0, nov)
    win = c.torch.as_tensor(c.gdsp.window.Hann(sp.flen), dtype=c.torch.float64, device=x.device)
    acc = c.torch.zeros(sp.flen, dtype=c.torch.float64, device=x.device)
    Dd.gpu_accumulate(xp, sp, win, acc, stream=c.stream)
    c.torch.cuda.synchronize()
    dev_p, _ = spectral.finalize(acc.cpu().numpy(), sp.nsegs_total, nfft, nfft,
                                 np.asarray(c.gdsp.window.Hann(nfft)), 1.0, False)
    host_p, _ = spectral.Pwelch(host, 1.0, opts)
    e_dev = float(np.linalg.norm(dev_p - ref) / np.linalg.norm(ref))
    e_host = float(np.linalg.norm(host_p - ref) / np.linalg.norm(ref))
    full = wl["result"].get("pxx")
    level = float(np.median(full[1:-1])) if full is not None else None
    fs = {"bins": None if full is None else int(full.size),
          "finite": None if full is None else bool(np.all(np.isfinite(full))),
          "median_interior": level, "expected": 2.0 / 3.0}
    if full is not None and c.world == 1:
        # the timed full-size Pxx itself against the oracle over the whole
        # stream (every segment; oracle.pwelch_chunked on 16 host threads)
        t0 = time.perf_counter()
        xh = x.cpu().numpy()
        ref_full, _ = oracle.pwelch_chunked(xh, 1.0, nfft, nov,
                                            nthreads=max(1, min(16, os.cpu_count() or 1)))
        del xh
        fs.update({"samples": int(x.numel()), "segments": sh.nsegs_total,
                   "nrel_vs_oracle": float(np.linalg.norm(full - ref_full) /
                                           np.linalg.norm(ref_full)),
                   "oracle_s": round(time.perf_counter() - t0, 2),
                   "check": "the timed step's 2^30-sample Pxx vs oracle.pwelch_chunked over "
                            "every segment (pwelch.go:104-136)"})
    return {"samples": pre, "segments": sp.nsegs_total,
            "max_nrel_vs_oracle": max(e_dev, e_host), "nrel_device_path": e_dev,
            "nrel_host_api": e_host, "full_size": fs}


def run_fftreal1024(c: Ctx) -> dict:
    """BASELINE configs[0]: fft.FFTReal of one N = 1024 float64 vector
    (fft/fft.go:25-27), called the way the reference is called: a host slice
    in, a fresh complex128 slice out, through the host-pointer C ABI
    (gdsp_fft_real: mapped pinned buffers, one launch, one synchronisation).
    A step is one call; each timed step is the mean of 200 calls. The kernel's
    own duration (HIP events, device-resident row) is the roofline figure."""
    import numpy as np
    torch, D, args = c.torch, c.D, c.args
    n = 1024
    xd = torch.empty(n, dtype=torch.float64, device=c.dev)
    D.fill_uniform(xd, SEED, stream=c.stream)
    torch.cuda.synchronize()
    xh = xd.cpu().numpy()
    fr = c.gdsp.fft.FFTReal
    reps = 200
    for _ in range(args.warmup * reps):
        fr(xh)
    c.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps * reps):
        y = fr(xh)
    elapsed = time.perf_counter() - t0
    per_call = elapsed / (args.steps * reps)
    # the kernel alone: the same FFTReal on the device-resident float64 row
    # (gdsp_fft_real_batch_device: the LOAD_REAL kernel the host call runs)
    xr = xd.reshape(1, n)
    yc = torch.empty((1, n), dtype=torch.complex128, device=c.dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(10):
        D.fft_real_batch(xr, yc, stream=c.stream)
    ev[0].record(c.stream)
    for _ in range(reps):
        D.fft_real_batch(xr, yc, stream=c.stream)
    ev[1].record(c.stream)
    torch.cuda.synchronize()
    kern_s = ev[0].elapsed_time(ev[1]) / reps / 1e3
    alg = 8 * n + 16 * n  # float64 in, complex128 out
    check = None
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    if c.rank == 0 and args.check_rows > 0:
        ref = oracle.fft_real(xh)
        check = {"rows": 1, "max_nrel_vs_oracle": float(np.linalg.norm(y - ref) /
                                                          np.linalg.norm(ref)),
                 "nrel_vs_numpy": float(np.linalg.norm(y - np.fft.fft(xh)) /
                                        np.linalg.norm(ref))}
    crossover = None
    if c.rank == 0 and args.check_rows > 0:
        crossover = small_call_crossover(c, np, oracle)
    return {
        "metric": "Gsamples/s (us per call), fft.FFTReal N=1024 on a host vector",
        "value": round(n / per_call / 1e9, 6),
        "unit": "Gsamples/s",
        "small_n": crossover,
        "ms_per_step": round(per_call * 1e3, 5),
        "us_per_call": round(per_call * 1e6, 2),
        "scaling": "weak",
        "dtype": "f64 in, complex128 out",
        "config": {"workload": "fft.FFTReal of one N=1024 float64 host vector per call "
                               "(BASELINE configs[0]; host C ABI, PCIe-inclusive)",
                   "n": n, "batch": 1, "calls_timed": args.steps * reps,
                   "parallelism": f"replicas{c.world}"},
        "roofline": {"bound": "latency", "kernel": "fft_lds_kernel<10> (one float64 row, LOAD_REAL)",
                     "achieved": round(alg / kern_s / 1e9, 3), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / kern_s / 1e9 / HBM_PEAK_GBS, 6),
                     "frac_vs_copy": round(alg / kern_s / 1e9 / HBM_COPY_GBS, 6),
                     "avg_launch_ms": round(kern_s * 1e3, 5), "alg_bytes_per_launch": alg,
                     "traffic": None,
                     "note": "one 24 KiB transform: launch-latency bound, not HBM bound; "
                             "the call's cost is launch + synchronisation (us_per_call)"},
        "fp64": None,
        "cpu_baseline": None,
        "parity": check,
        "drop_in_policy": {
            "gpu_min_n": 0, "source": "go/fft/fft_gpu.go",
            "note": "every one-vector call of the drop-in goes to the C ABI (round 6: no reference "
                    "FFT code in the gdspgpu build); small_n.first_n_gpu_faster is where a "
                    "one-vector GPU call beats one host thread"},
    }


def small_call_crossover(c: Ctx, np, oracle) -> dict:
    """fft.FFTReal per-call time through the host C ABI against the
    reference algorithm's restatement on one host thread, by length: where
    a one-vector call starts to pay on the GPU (small-n
    policy)."""
    rows = []
    cross = None
    for n in (64, 256, 1024, 2048, 4096, 8192, 16384, 65536):
        x = oracle.fill_uniform(n, SEED)
        reps = 200 if n <= 16384 else 40
        c.gdsp.fft.FFTReal(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            c.gdsp.fft.FFTReal(x)
        g = (time.perf_counter() - t0) / reps
        oracle.fft_real(x)
        t0 = time.perf_counter()
        for _ in range(reps):
            oracle.fft_real(x)
        h = (time.perf_counter() - t0) / reps
        rows.append({"n": n, "gpu_call_us": round(g * 1e6, 2), "cpu_1thread_us": round(h * 1e6, 2)})
        if cross is None and g < h:
            cross = n
    return {"by_n": rows, "first_n_gpu_faster": cross}


def run(w: str, c: Ctx, weak: bool = False) -> dict:
    """One workload: setup, timed steps, its bench-line fields."""
    if w == "fftreal1024":
        return run_fftreal1024(c)
    wl = setup(w, c, weak=weak)
    m = measure(wl, c)
    check = parity(w, wl, c)
    elapsed, avg_launch_s, args, world = m["elapsed"], m["avg_launch_s"], c.args, c.world
    value = wl["total_samples"] * args.steps / elapsed / 1e9
    achieved = wl["alg_bytes"] / avg_launch_s / 1e9
    # the committed PMC / SQ summaries were taken at the N=1 full-size
    # configuration: scale them to this launch's share of that work (a rank's
    # shard at N>1, or a --batch override)
    share = wl["alg_bytes"] / PROFILED_ALG_BYTES[w]
    traffic = traffic_src = None
    pmc = os.path.join(REPO, "profiles", f"pmc_{w}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            pj = json.load(f)
        t = pj.get("hbm_bytes_per_launch")
        pk = pj.get("kernel")
        if isinstance(pk, str) and not wl["kernel"].startswith(pk):
            t = None  # profiled on another kernel than the one timed here
        traffic = None if t is None else int(round(t * share))
        traffic_src = {"file": f"profiles/pmc_{w}.json", "source": pj.get("source"),
                       "stamp": pj.get("stamp"),
                       "same_sources": stamp_matches(pj.get("stamp"), c.stamp)}
    out = {
        "metric": wl["metric"],
        "value": round(value, 3),
        "unit": "Gsamples/s",
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "warmup_steps_run": wl.get("warmup_steps_run"),
        "scaling": wl["scaling"],
        "dtype": wl.get("dtype", "f64 (complex128)"),
        "config": wl["cfg"],
        "roofline": {"bound": "hbm", "kernel": wl["kernel"],
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "frac_vs_copy": round(achieved / HBM_COPY_GBS, 4),
                     "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                     "alg_bytes_per_launch": wl["alg_bytes"], "traffic": traffic,
                     "traffic_source": traffic_src,
                     "rocprof": rocprof_info(w, wl["alg_bytes"], share, c.stamp)},
        "fp64": fp64_info(w, avg_launch_s, share),
        "cpu_baseline": None,  # filled in by main() after every GPU measurement
        "parity": check,
    }
    if w == "chirpz3000" and not weak and wl["kernel"] == "chirpz6k_kernel":
        # the same workload on the reference's convolution length M = 8192
        # (bluestein.go:70; GDSP_ALGO_CHIRPZ_POW2), timed the same way
        F = c.gdsp.fft
        del wl
        F.SetAlgorithm(F.ALGO_CHIRPZ_POW2)
        try:
            w8 = setup(w, c)
            m8 = measure(w8, c)
        finally:
            F.SetAlgorithm(F.ALGO_DEFAULT)
        out["reference_m8192"] = {
            "kernel": w8["kernel"], "algorithm": w8["cfg"]["algorithm"],
            "ms_per_step": round(m8["elapsed"] / args.steps * 1e3, 4),
            "avg_launch_ms": round(m8["avg_launch_s"] * 1e3, 4),
            "frac": round(w8["alg_bytes"] / m8["avg_launch_s"] / 1e9 / HBM_PEAK_GBS, 4)}
        del w8
        c.torch.cuda.empty_cache()
        return out
    if (w, wl["kernel"]) in (("prime3001", "rader_fixed_kernel"),
                             ("pfa3027", "rader_pfa_kernel")) and not weak:
        # the same prime on the chirp-z kernel it took before Rader
        # (GDSP_ALGO_NO_RADER: the fused chirp-z on M = 6144), timed the same way
        F = c.gdsp.fft
        del wl
        F.SetAlgorithm(F.ALGO_NO_RADER)
        try:
            wc = setup(w, c)
            mc = measure(wc, c)
        finally:
            F.SetAlgorithm(F.ALGO_DEFAULT)
        out["chirpz"] = {
            "kernel": wc["kernel"], "algorithm": wc["cfg"]["algorithm"],
            "ms_per_step": round(mc["elapsed"] / args.steps * 1e3, 4),
            "avg_launch_ms": round(mc["avg_launch_s"] * 1e3, 4),
            "frac": round(wc["alg_bytes"] / mc["avg_launch_s"] / 1e9 / HBM_PEAK_GBS, 4)}
        del wc
        c.torch.cuda.empty_cache()
        return out
    if c.rank == 0 and w == "fft_2p20":
        # fft.FFT on a host vector, the way BenchmarkFFT calls it: H2D +
        # transform + D2H through the C ABI's pinned staging (PCIe-inclusive;
        # reported beside value, never as value)
        xh = wl["x"][0].cpu().numpy()
        c.gdsp.fft.FFT(xh)
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            c.gdsp.fft.FFT(xh)
        dt = (time.perf_counter() - t0) / reps
        out["host_api"] = {"ms_per_call": round(dt * 1e3, 4),
                           "gsamples_s": round(xh.size / dt / 1e9, 4),
                           "note": "gdsp.fft.FFT on a host numpy vector (C ABI host-pointer "
                                   "path, PCIe-inclusive)"}
    del wl
    c.torch.cuda.empty_cache()
    return out


def launch_plan(gpus: int, env: dict, device_count) -> tuple:
    """What `bench.py --gpus N` does before anything touches a GPU.

    Returns ("run", None) when this process is a rank (WORLD_SIZE set by
    torch.distributed.run or by launch(), or N = 1), ("spawn", [env per rank])
    when it must start N rank processes itself, or ("error", message).
    device_count() is only called for a spawn with the nccl backend (RCCL
    needs one GPU per rank); the gloo rehearsal (GDSP_DIST_BACKEND=gloo) may
    put several ranks on one GPU."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    ws = env.get("WORLD_SIZE")
    backend = env.get("GDSP_DIST_BACKEND", "nccl")
    if ws is not None:
        if int(ws) != gpus:
            return "error", (f"WORLD_SIZE={ws} (set by the launcher) but --gpus {gpus}: "
                             "the two must agree")
        return "run", None
    if gpus == 1:
        return "run", None
    if backend == "nccl":
        have = device_count()
        if have < gpus:
            return "error", (f"--gpus {gpus} with the nccl (RCCL) backend needs {gpus} GPUs, "
                             f"this node has {have}; GDSP_DIST_BACKEND=gloo rehearses the "
                             "multi-rank path with ranks sharing a GPU")
    port = env.get("MASTER_PORT") or str(_free_port())
    ranks = []
    for r in range(gpus):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(gpus),
                  "LOCAL_WORLD_SIZE": str(gpus), "GROUP_RANK": "0",
                  "MASTER_ADDR": env.get("MASTER_ADDR", "127.0.0.1"), "MASTER_PORT": port})
        ranks.append(e)
    return "spawn", ranks


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(cmd: list, ranks: list, poll_s: float = 0.2) -> int:
    """Start one child per rank (cmd with that rank's environment) and wait.
    Only rank 0's JSON line reaches stdout: every other line a child prints on
    stdout (e.g. gloo's "[Gloo] Rank 1 is connected to ..." banner) goes to
    stderr, so the result stays one parseable line. The first child to fail
    ends the others (their exact PIDs), and its exit status is returned. This
    process makes no GPU call."""
    import subprocess
    import threading
    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE, text=True) for e in ranks]

    def pump(rank: int, stream):
        for raw in stream:
            line = raw.rstrip("\n")
            if rank == 0 and line.startswith("{"):
                print(line, flush=True)
            elif line:
                print(line, file=sys.stderr, flush=True)

    pumps = [threading.Thread(target=pump, args=(i, p.stdout), daemon=True)
             for i, p in enumerate(procs)]
    for t in pumps:
        t.start()
    rc = 0
    try:
        while procs:
            for p in list(procs):
                r = p.poll()
                if r is None:
                    continue
                procs.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in procs:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for t in pumps:
            t.join(timeout=5)
    return rc if rc >= 0 else 128 - rc  # a signalled child: 128 + signal number


def rank_device_check(ndev: int, local: int, backend: str, env: dict, world: int):
    """A rank's own check before it binds a GPU (None: fine, else the reason).
    RCCL needs one GPU per rank of this node, so the ranks on this node
    (LOCAL_WORLD_SIZE, set by torch.distributed.run and by launch(); WORLD_SIZE
    only when neither set it) are compared with the GPUs this rank sees. A
    launcher that hands each rank its own GPU through a visibility variable
    leaves every rank one device, which is fine. Multi-node jobs pass, since
    only the node's own ranks count."""
    if backend != "nccl":
        return None  # the gloo rehearsal may share one GPU
    local_world = int(env.get("LOCAL_WORLD_SIZE", str(world)))
    if ndev >= local_world and local < ndev:
        return None
    if ndev == 1 and _visible_limit(env) == 1:
        return None
    return (f"{local_world} ranks on this node over nccl (RCCL) need {local_world} GPUs, "
            f"rank {local} sees {ndev}")


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _visible_limit(env: dict):
    """How many devices the visibility variables leave (None: no limit). The
    HIP runtime honours ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES on top of it; each is a comma list of indices or
    UUIDs, so the count is its number of entries (an empty value hides all)."""
    lim = None
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v is None:
            continue
        n = len([p for p in v.split(",") if p.strip()])
        lim = n if lim is None else min(lim, n)
    return lim


def kfd_gpu_count(root: str = None, env: dict = None):
    """GPUs in the KFD topology (sysfs): nodes with a nonzero gpu_id and SIMDs.
    Reading sysfs loads no HIP/HSA runtime, so the launcher parent stays free
    of any GPU state before it starts the ranks. None when the topology is not
    readable (no amdgpu driver, or a sandbox without /sys)."""
    env = os.environ if env is None else env
    root = KFD_NODES if root is None else root
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(root, d, "gpu_id")) as f:
                gid = int(f.read().strip() or "0")
            simd = 0
            with open(os.path.join(root, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count":
                        simd = int(v)
        except (OSError, ValueError):
            continue
        if gid != 0 and simd > 0:
            n += 1
    lim = _visible_limit(env)
    return n if lim is None else min(n, lim)


def _device_count() -> int:
    """GPUs visible to the ranks, counted without initialising HIP in this
    (launcher) process: the KFD topology in sysfs, or else a short-lived
    child process that asks torch (its runtime dies with it)."""
    n = kfd_gpu_count()
    if n is not None:
        return n
    import subprocess
    p = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(p.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def main():
    args = parse()
    what, info = launch_plan(args.gpus, dict(os.environ), _device_count)
    if what == "error":
        print(f"bench.py: {info}", file=sys.stderr, flush=True)
        sys.exit(2)
    if what == "spawn":
        sys.exit(launch([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], info))
    # stdout carries the one JSON line and nothing else: whatever the
    # libraries below write to file descriptor 1 (gloo's "[Gloo] Rank 1 is
    # connected to ..." banner from every rank, runtime notices) goes to stderr
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    c = Ctx(args)
    w = "radix4096" if args.workload == "default" else args.workload
    head = run(w, c)
    line = {"metric": head["metric"], "value": head["value"], "unit": "Gsamples/s",
            "n_gpus": c.world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "warmup_steps_run": head.get("warmup_steps_run"),
            "scaling": head["scaling"], "vs_baseline": None, "dtype": head["dtype"],
            "data": "synthetic (splitmix64 uniform[-1,1), generated in HBM)",
            "sources": c.stamp}
    line.update({k: head[k] for k in ("config", "roofline", "fp64", "cpu_baseline", "parity")})
    if "host_api" in head:
        line["host_api"] = head["host_api"]
    if c.world > 1 and w == "radix4096":
        # secondary: every rank with its own 65536 rows (weak scaling)
        weak = run(w, c, weak=True)
        line["weak_scaling"] = {k: weak[k] for k in ("value", "ms_per_step", "config")}
    if args.workload == "default":
        line["configs"] = {}
        for cw in NESTED:
            r = run(cw, c)
            r.pop("metric")
            line["configs"][cw] = r
    # CPU baselines last, so that no GPU measurement follows seconds of an
    # idle GPU (rank 0 at N=1 only)
    if c.rank == 0 and c.world == 1:
        if args.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
        for cw, r in line.get("configs", {}).items():
            if args.config_cpu_seconds > 0:
                r["cpu_baseline"] = cpu_baseline(cw, args.config_cpu_seconds)
    if c.rank == 0:
        print(json.dumps(line), file=result_out, flush=True)
    if c.world > 1:
        c.dist.destroy_process_group()


def fp64_info(workload: str, launch_s: float, share: float = 1.0):
    """FP64 work of one launch (from the committed SQ counters of the newest
    round that profiled this workload's kernels, FFT2 summed over its
    kernels, times this launch's share of the profiled work) against the FP64
    vector peak — the second roofline of the compute-heavy paths (chirp-z,
    Pwelch)."""
    w = "fft2_8192" if workload == "fft2_dist" else workload
    ks = SQ_KERNELS.get(w)
    if not ks:
        return None
    for rnd in SQ_ROUNDS:
        path = os.path.join(REPO, "profiles", rnd, "sq_counters.json")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            sq = json.load(f).get(w, {})
        flop, found = 0.0, True
        for k in ks:
            hit = [v for name, v in sq.items() if k in name]
            if not hit:
                found = False
                break
            flop += hit[0]["f64_flop"]
        if not found:
            continue
        flop *= share
        tf = flop / launch_s / 1e12
        return {"flop_per_launch": flop, "achieved_tflops": round(tf, 2),
                "peak_tflops": FP64_PEAK_TFLOPS, "frac": round(tf / FP64_PEAK_TFLOPS, 4),
                "source": f"profiles/{rnd}/sq_counters.json (SQ_INSTS_VALU_{{FMA,ADD,MUL}}_F64)"}
    return None


def stamp_matches(profiled, now):
    """Whether a committed profile was taken on the sources this run executes
    (tools/source_stamp.py: the kernel sources' sha256); None if unstamped."""
    if not profiled or not now:
        return None
    return profiled.get("source_sha") == now.get("source_sha")


def rocprof_info(workload: str, alg_bytes: int, share: float = 1.0, stamp=None):
    """The dominant kernel's duration from the committed rocprofv3
    --kernel-trace --stats summary of this workload (newest round; FFT2: its
    launches summed), and roofline.frac recomputed from that average: the
    profiler's figure quoted beside the HIP-event one. The summary was taken
    at the N=1 full-size configuration; share scales it to this launch."""
    w = "fft2_8192" if workload == "fft2_dist" else workload
    ks = SQ_KERNELS.get(w)
    if not ks:
        return None
    import csv
    for rnd in STATS_ROUNDS:
        # per-launch trace: the average over the launches that run timed
        # (the last timed_last; the earlier ones are the run's warm-up)
        tpath = os.path.join(REPO, "profiles", rnd, f"{w}_kernel_trace.json")
        if os.path.exists(tpath):
            with open(tpath) as f:
                tr = json.load(f)
            last = tr["timed_last"]
            avg = mn = 0.0
            calls = []
            for k in ks:
                hit = [v for name, v in tr["kernels"].items() if k in name]
                if not hit:
                    break
                d = max(hit, key=len)[-last:]
                avg += sum(d) / len(d)
                mn += min(d)
                calls.append(len(d))
            else:
                avg_s = avg * 1e-9 * share
                ach = alg_bytes / avg_s / 1e9
                return {"avg_launch_ms": round(avg_s * 1e3, 4),
                        "min_launch_ms": round(mn * 1e-6 * share, 4), "calls": calls,
                        "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                        "over": "the timed launches of the profiled run (its last "
                                f"{last}; warm-up excluded)",
                        "source": f"profiles/{rnd}/{w}_kernel_trace.json",
                        "stamp": tr.get("stamp"),
                        "same_sources": stamp_matches(tr.get("stamp"), stamp)}
        path = os.path.join(REPO, "profiles", rnd, f"{w}_kernel_stats.csv")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            rows = list(csv.DictReader(f))
        avg = mn = 0.0
        calls = []
        for k in ks:
            hit = [r for r in rows if k in r["Name"]]
            if not hit:
                break
            r = max(hit, key=lambda r: int(r["Calls"]))  # the timed template
            avg += float(r["AverageNs"])
            mn += float(r["MinNs"])
            calls.append(int(r["Calls"]))
        else:
            avg_s = avg * 1e-9 * share
            ach = alg_bytes / avg_s / 1e9
            return {"avg_launch_ms": round(avg_s * 1e3, 4), "min_launch_ms": round(mn * 1e-6 * share, 4),
                    "calls": calls, "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                    "source": f"profiles/{rnd}/{w}_kernel_stats.csv"}
    return None


def cpu_baseline(workload: str, seconds: float):
    """The reference algorithm on the host (oracle/: C restatement of
    fft/radix2.go, fft/bluestein.go, spectral/pwelch.go) with the reference's
    worker pool of min(nproc, 16) threads inside every radix-2 transform
    (radix2.go:89-151), on a bounded sample of the same synthetic workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle
    cores = min(os.cpu_count() or 1, 16)  # the GPU box's CPU share is 16
    pool = f"reference worker pool of {cores} threads per radix-2 transform (radix2.go:89-151)"
    out = _cpu_baseline(workload, seconds, cores, pool, np, oracle)
    out["cpu_model"] = cpu_model()
    return out


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_baseline(workload: str, seconds: float, cores: int, pool: str, np, oracle) -> dict:
    if workload == "fftreal1024":
        # fft.FFTReal(N=1024) restated: ToComplex + radix2FFT, one call at a
        # time on one thread (the reference's pool of goroutines is not
        # restated here: OS threads per call would overstate its overhead)
        x = oracle.fill_uniform(1024, SEED)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for _ in range(100):
                oracle.fft_real(x)
            done += 100
        dt = time.perf_counter() - t0
        return {"value": round(done * 1024 / dt / 1e9, 6), "unit": "Gsamples/s", "cores": 1,
                "kind": "port", "us_per_call": round(dt / done * 1e6, 2),
                "sample": f"{done} fft.FFTReal calls of N=1024 ({dt:.1f} s), one thread, "
                          f"called from Python (ctypes) like the GPU line"}
    if workload in ("pwelch", "pwelch_default"):
        nfft, nov = (256, 0) if workload == "pwelch_default" else (4096, 2048)
        n = 1 << 20
        t0 = time.perf_counter()
        while True:
            x = oracle.fill_uniform(n, SEED)
            t1 = time.perf_counter()
            oracle.pwelch_threaded(x, 1.0, nfft, nov, cores)
            dt = time.perf_counter() - t1
            if dt > seconds / 3 or time.perf_counter() - t0 > seconds:
                break
            n *= 2
        return {"value": round(n / dt / 1e9, 6), "unit": "Gsamples/s", "cores": cores,
                "kind": "port",
                "sample": f"spectral.Pwelch on a {n}-sample prefix of the stream "
                          f"(NFFT {nfft}, Noverlap {nov}, {dt:.1f} s), {pool}"}
    if workload == "wav_decode":
        # wav.ReadFloats's conversion restated (oracle/oracle.c), one thread
        raw = oracle.fill_uniform(1 << 21, SEED).view(np.uint8)
        count = raw.size // 2
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.wav_floats(raw, count, 1, 16)
            done += count
        dt = time.perf_counter() - t0
        return {"value": round(done / dt / 1e9, 6), "unit": "Gsamples/s", "cores": 1,
                "kind": "port",
                "sample": f"{done} PCM16 samples ({dt:.1f} s) through the ReadFloats "
                          f"restatement (wav/wav.go:135-161), float32 out as the reference"}
    if workload == "fft_2p20":
        # BenchmarkFFT restated: one N=2^20 fft.FFT with the reference's worker
        # pool (GOMAXPROCS = NumCPU, capped at the box's 16-core share)
        x = oracle.fill_uniform(2 * (1 << 20), SEED).view(np.complex128).reshape(1, 1 << 20)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.fft_rows_threaded(x, cores)
            done += 1
        dt = time.perf_counter() - t0
        return {"value": round(done * (1 << 20) / dt / 1e9, 6), "unit": "Gsamples/s",
                "cores": cores, "kind": "port",
                "sample": f"{done} fft.FFT calls of N=2^20 ({dt:.1f} s), {pool}"}
    if workload == "fftn_512":
        # computeFFTN (fft.go:157-192): 3 x 512^2 line FFTs of 512; the
        # strided gather/scatter of axes 0 and 1 is not charged (favours the CPU)
        x = oracle.fill_uniform(2 * 512 * 256, SEED).view(np.complex128).reshape(256, 512)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.fft_rows_threaded(x, cores)
            done += 256
        dt = time.perf_counter() - t0
        t_fftn = 3 * 512 * 512 * dt / done
        return {"value": round(512 ** 3 / t_fftn / 1e9, 6), "unit": "Gsamples/s",
                "cores": cores, "kind": "port",
                "sample": f"{done} fft.FFT calls of N=512 ({dt:.1f} s) extrapolated to the "
                          f"786432 line FFTs of one 512^3 FFTN, {pool}"}
    if workload == "fft2_dist":
        workload = "fft2_8192"
    n = {"radix4096": 4096, "bluestein3000": 3000, "chirpz3000": 3000, "prime3001": 3001,
         "pfa3027": 3027, "fft2_8192": 8192}[workload]
    rows = 64 if n != 8192 else 16
    x = oracle.fill_uniform(2 * n * rows, SEED).view(np.complex128).reshape(rows, n)
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        oracle.fft_rows_threaded(x, cores)
        done += rows
    dt = time.perf_counter() - t0
    per_fft = dt / done
    if workload == "fft2_8192":
        # computeFFT2 = 8192 column FFTs + 8192 row FFTs of 8192 (fft.go:138-151);
        # the strided column gather/scatter is not charged (favours the CPU)
        t_fft2 = 2 * 8192 * per_fft
        return {"value": round(8192 * 8192 / t_fft2 / 1e9, 6), "unit": "Gsamples/s",
                "cores": cores, "kind": "port",
                "sample": f"{done} fft.FFT calls of N=8192 ({dt:.1f} s) extrapolated to the "
                          f"16384 calls of one 8192x8192 FFT2, {pool}"}
    return {"value": round(done * n / dt / 1e9, 6), "unit": "Gsamples/s",
            "cores": cores, "kind": "port",
            "sample": f"{done} rows x N={n} ({dt:.1f} s) of the bench's synthetic input, one "
                      f"fft.FFT call per row, {pool}"}


if __name__ == "__main__":
    main()
