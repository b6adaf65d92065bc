"""N>1 path on CPU: world_size 2 and 3 with the gloo backend. The GPU
accumulation is replaced by an oracle-based accumulator (tests may use the
oracle as the checker); everything else — segment sharding with halo, the
all-reduce of the PSD accumulators and the host finalisation — is the code the
GPU ranks run."""
import os
import socket

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _signal(n):
    t = np.arange(n)
    rng = np.random.default_rng(5)
    return np.sin(2 * np.pi * 0.1234 * t) + 0.5 * rng.standard_normal(n)


CASES = [
    dict(n=50000, nfft=4096, noverlap=2048, pad=0, fs=1.0),
    dict(n=30001, nfft=1000, noverlap=250, pad=2048, fs=3.0),
    dict(n=3000, nfft=256, noverlap=0, pad=0, fs=2.0),
    dict(n=100, nfft=0, noverlap=0, pad=0, fs=2.0),  # one zero-padded segment
]


def _worker(rank, world, port, outdir):
    import importlib
    import sys

    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    gdsp = importlib.import_module("go-dsp_amd")
    Dd = importlib.import_module("go-dsp_amd.distributed")
    results = []
    for c in CASES:
        x = _signal(c["n"])
        sh = Dd.plan_pwelch(x.size, world, rank, c["nfft"], c["pad"], c["noverlap"])
        xp = np.zeros(max(x.size, sh.nfft))
        xp[:x.size] = x
        x_local = torch.tensor(xp[sh.sample_lo:sh.sample_hi], dtype=torch.float64)

        def acc_fn(xl, shard, win, acc, stream):
            w = win.numpy()
            a = np.zeros(shard.flen)
            xl = xl.numpy()
            for s in range(shard.seg_hi - shard.seg_lo):
                seg = np.zeros(shard.flen)
                seg[:shard.nfft] = xl[s * shard.stride:s * shard.stride + shard.nfft]
                a += np.abs(oracle.fft_real(seg * w)) ** 2
            acc += torch.from_numpy(a)

        o = gdsp.spectral.PwelchOptions(NFFT=c["nfft"], Noverlap=c["noverlap"], Pad=c["pad"])
        p, f = Dd.pwelch(x_local, c["fs"], o, sh, accumulate=acc_fn)
        results.append((p, f, (sh.seg_lo, sh.seg_hi, sh.sample_lo, sh.sample_hi)))
    np.save(os.path.join(outdir, f"r{rank}.npy"),
            np.array([np.concatenate([p, f]) for p, f, _ in results], dtype=object),
            allow_pickle=True)
    np.save(os.path.join(outdir, f"s{rank}.npy"), np.array([r[2] for r in results]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pwelch_sharded_gloo(tmp_path, oracle, world):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    shards = [np.load(tmp_path / f"s{r}.npy") for r in range(world)]
    for ci, c in enumerate(CASES):
        pr, fr = oracle.pwelch(_signal(c["n"]), c["fs"], nfft=c["nfft"], pad=c["pad"],
                               noverlap=c["noverlap"])
        for r in range(world):
            got = np.load(tmp_path / f"r{r}.npy", allow_pickle=True)[ci]
            p, f = got[:pr.size], got[pr.size:]
            assert np.linalg.norm(p - pr) / np.linalg.norm(pr) < 1e-12
            assert np.array_equal(f, fr)
        # segment shards tile [0, S) exactly
        los = [int(shards[r][ci][0]) for r in range(world)]
        his = [int(shards[r][ci][1]) for r in range(world)]
        assert los[0] == 0 and all(his[r] == los[r + 1] for r in range(world - 1))


def test_shard_ranges(gdsp):
    Dd = __import__("importlib").import_module("go-dsp_amd.distributed")
    total = ((1 << 30) - 4096) // 2048 + 1
    for world in (1, 2, 4, 8):
        spans = [Dd.shard_range(total, world, r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == total
        assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1
    sh = Dd.plan_pwelch(1 << 30, 8, 3, 4096, 0, 2048)
    assert sh.sample_hi - sh.sample_lo == (sh.seg_hi - sh.seg_lo - 1) * 2048 + 4096


FFT2_SHAPES = [(16, 12), (17, 10), (9, 2), (64, 48)]


def _fft2_worker(rank, world, port, outdir):
    import importlib
    import sys

    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    Dd = importlib.import_module("go-dsp_amd.distributed")
    out = {}
    for R, C in FFT2_SHAPES:
        x = oracle.fill_uniform(2 * R * C, 0x5EED, R * 100 + C).view(np.complex128).reshape(R, C)
        lo, hi = Dd.shard_range(R, world, rank)
        for inv in (False, True):
            rf = (lambda a, inv=inv: torch.from_numpy(
                (oracle.ifft_rows if inv else oracle.fft_rows)(a.numpy())))
            cf = (lambda a, inv=inv: torch.from_numpy(np.ascontiguousarray(
                (oracle.ifft_rows if inv else oracle.fft_rows)(a.numpy().T.copy()).T))
                if a.numel() else a)
            y = Dd.fft2_sharded(torch.from_numpy(x[lo:hi].copy()), R, inverse=inv,
                                row_fft=rf, col_fft=cf)
            out[f"{R}x{C}_{int(inv)}"] = y.numpy()
    np.savez(os.path.join(outdir, f"fft2_r{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fft2_sharded_gloo(world, tmp_path, oracle):
    """Row-sharded FFT2 with the two all-to-alls (gloo): the gathered row
    shards equal the single-process FFT2 of the reference restatement."""
    import torch.multiprocessing as mp
    mp.spawn(_fft2_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    parts = [dict(np.load(tmp_path / f"fft2_r{r}.npz")) for r in range(world)]
    for R, C in FFT2_SHAPES:
        x = oracle.fill_uniform(2 * R * C, 0x5EED, R * 100 + C).view(np.complex128).reshape(R, C)
        for inv in (0, 1):
            got = np.concatenate([p[f"{R}x{C}_{inv}"] for p in parts], axis=0)
            ref = oracle.fft2(x, inverse=bool(inv))
            assert got.shape == (R, C)
            assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 1e-12, (R, C, inv)
