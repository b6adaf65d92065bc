"""Multi-GPU drivers for the go-dsp hot path: one process per GPU
(torch.distributed; backend "nccl" = RCCL over xGMI on ROCm).

- Batched FFT (fft.FFT over many rows): rows are independent, so each rank
  transforms a contiguous row shard; there is no data-path collective.
- FFT2 (fft/fft.go:123-154) of a matrix whose rows are sharded over the
  ranks: local row FFTs, one all-to-all that gives every rank all rows of its
  column block, local column FFTs (gdsp_fft_axis_device), and one all-to-all
  back to the row shards. Two RCCL all-to-alls of (W-1)/W of the shard each.
- Pwelch (spectral/pwelch.go:74-145): segments [S*r/W, S*(r+1)/W) go to rank
  r, which needs samples [lo*stride, (hi-1)*stride + nfft) — its slice plus an
  (nfft - stride)-sample halo. Each rank accumulates per-bin power sums on its
  GPU; one all-reduce (sum, float64, max(pad, nfft) values) combines them and
  every rank finalises Pxx on the host (gdsp_pwelch_finalize). The reordered
  summation changes Pxx only at roundoff (all terms are non-negative).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import spectral


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of `total` units for `rank` of `world`."""
    return total * rank // world, total * (rank + 1) // world


@dataclass
class PwelchShard:
    seg_lo: int      # first segment of this rank (global index)
    seg_hi: int      # one past the last segment
    sample_lo: int   # first sample this rank needs
    sample_hi: int   # one past the last sample it needs (halo included)
    nsegs_total: int
    nfft: int
    pad: int
    noverlap: int

    @property
    def stride(self) -> int:
        return self.nfft - self.noverlap

    @property
    def flen(self) -> int:
        return max(self.pad, self.nfft)


def plan_pwelch(n_samples: int, world: int, rank: int, nfft: int = 0, pad: int = 0,
                noverlap: int = 0) -> PwelchShard:
    """Segment/sample ranges of `rank` (defaults as pwelch.go:85-95; a signal
    shorter than nfft is zero-padded to nfft, pwelch.go:97-99)."""
    nfft = nfft or 256
    pad = pad or nfft
    lx = max(n_samples, nfft)
    nsegs = spectral.segment_count(lx, nfft, noverlap)
    lo, hi = shard_range(nsegs, world, rank)
    stride = nfft - noverlap
    if hi > lo:
        s_lo, s_hi = lo * stride, (hi - 1) * stride + nfft
    else:
        s_lo = s_hi = 0
    return PwelchShard(lo, hi, s_lo, s_hi, nsegs, nfft, pad, noverlap)


def gpu_accumulate(x_local, shard: PwelchShard, win_seg, acc, stream=None):
    """Per-bin power sums of the rank's segments on its GPU (fused kernel)."""
    from . import device
    device.pwelch_accumulate(x_local, shard.nfft, shard.pad, shard.noverlap, 0,
                             shard.seg_hi - shard.seg_lo, win_seg, acc, stream=stream)
    return acc


_win_dev: dict = {}


def _device_window(wf, flen: int, dev, torch):
    """wf(flen) as a float64 tensor on dev, uploaded once per (window, length,
    device): the window functions are pure, and a per-call pageable upload
    is a synchronous host copy inside every Pwelch step."""
    key = (wf, int(flen), str(dev))
    t = _win_dev.get(key)
    if t is None:
        if len(_win_dev) >= 32:  # e.g. a fresh lambda per call: keep it bounded
            _win_dev.clear()
        t = torch.as_tensor(np.ascontiguousarray(wf(flen)), dtype=torch.float64, device=dev)
        _win_dev[key] = t
    return t


def pwelch(x_local, Fs: float, o: spectral.PwelchOptions, shard: PwelchShard, group=None,
           accumulate: Optional[Callable] = None, stream=None):
    """Sharded spectral.Pwelch. x_local: this rank's samples
    [shard.sample_lo, shard.sample_hi) as a float64 tensor on its device
    (zero-padded to nfft if the whole signal is shorter). Returns (Pxx, freqs)
    as numpy arrays on every rank."""
    import torch
    import torch.distributed as dist

    nfft, pad, noverlap, wf, scaling = spectral.resolve_options(o)
    assert (nfft, pad, noverlap) == (shard.nfft, shard.pad, shard.noverlap)
    flen = shard.flen
    dev = x_local.device
    # every torch op below (window upload, zeroing, the host copy) is ordered
    # on the same stream as the library's kernels
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        win_seg = _device_window(wf, flen, dev, torch)
        acc = torch.zeros(flen, dtype=torch.float64, device=dev)
        if shard.seg_hi > shard.seg_lo:
            (accumulate or gpu_accumulate)(x_local, shard, win_seg, acc, stream)
        if dist.is_initialized():  # world size 1 included: the same RCCL path
            if acc.is_cuda and dist.get_backend(group) != "nccl":
                acc = acc.cpu()  # gloo (rehearsal of the N>1 path): reduce a host copy
            dist.all_reduce(acc, group=group)
        host = acc.cpu().numpy()
    return spectral.finalize(host, shard.nsegs_total, nfft, pad,
                             np.asarray(wf(nfft), np.float64), Fs, not scaling)


def _all_to_all_c128(send, recv, send_counts, recv_counts, group, dist, torch):
    """all_to_all_single of complex128 pieces (as float64 pairs). gloo (the
    CPU rehearsal of the N>1 path) exchanges host copies."""
    sv, rv = torch.view_as_real(send).reshape(-1), torch.view_as_real(recv).reshape(-1)
    host = sv.is_cuda and dist.get_backend(group) != "nccl"
    s_, r_ = (sv.cpu(), torch.empty(rv.shape, dtype=rv.dtype)) if host else (sv, rv)
    dist.all_to_all_single(r_, s_, [2 * c for c in recv_counts], [2 * c for c in send_counts],
                           group=group)
    if host:
        rv.copy_(r_)


def fft2_sharded(x_local, rows_total: int, inverse: bool = False, group=None, stream=None,
                 row_fft: Optional[Callable] = None, col_fft: Optional[Callable] = None):
    """Multi-GPU fft.FFT2 / IFFT2 (fft/fft.go:109-154). x_local: this rank's
    rows [shard_range(rows_total, W, r)) of the rows_total x C matrix, a
    (rows_r, C) complex128 tensor. Returns this rank's rows of the result.

    1. row FFTs of the local rows (independent rows: no exchange);
    2. all-to-all: the column block [C*q/W, C*(q+1)/W) of the local rows goes
       to rank q, so each rank holds every row of its column block;
    3. column FFTs of that rows_total x C_r block;
    4. all-to-all back to row shards.
    The reference transforms columns first (fft.go:138-147); the 2-D DFT is
    the same either way (separable), at roundoff level.
    row_fft / col_fft (tensor -> tensor, FFT along rows / along axis 0)
    replace the device kernels — the CPU tests pass oracle-backed ones."""
    import torch
    import torch.distributed as dist

    W = dist.get_world_size(group) if dist.is_initialized() else 1
    r = dist.get_rank(group) if dist.is_initialized() else 0
    rows_r, C = x_local.shape
    lo, hi = shard_range(rows_total, W, r)
    assert rows_r == hi - lo, "x_local is not this rank's row shard"
    if row_fft is None or col_fft is None:
        from . import device
    row_fft = row_fft or (lambda a: device.fft_batch(a, inverse=inverse, stream=stream))
    col_fft = col_fft or (lambda a: device.fft_axis(a, 0, inverse=inverse, stream=stream))
    ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
    with ctx:
        y = row_fft(x_local.contiguous())
        if not dist.is_initialized():
            return col_fft(y)
        rows = [shard_range(rows_total, W, q) for q in range(W)]
        cols = [shard_range(C, W, q) for q in range(W)]
        c_lo, c_hi = cols[r]
        even = C % W == 0
        if even:
            # the W column blocks of the local rows, block-major: one copy of
            # contiguous C/W-element runs (torch.cat of column slices took two)
            send = y.view(rows_r, W, C // W).transpose(0, 1).contiguous().view(-1)
        else:
            send = torch.cat([y[:, a:b].reshape(-1) for a, b in cols])
        blk = torch.empty((rows_total, c_hi - c_lo), dtype=y.dtype, device=y.device)
        _all_to_all_c128(send, blk, [rows_r * (b - a) for a, b in cols],
                         [(b - a) * (c_hi - c_lo) for a, b in rows], group, dist, torch)
        blk = col_fft(blk)
        back = torch.empty(rows_r * C, dtype=y.dtype, device=y.device)
        _all_to_all_c128(blk.reshape(-1), back, [(b - a) * (c_hi - c_lo) for a, b in rows],
                         [rows_r * (b - a) for a, b in cols], group, dist, torch)
        if even:
            return back.view(W, rows_r, C // W).transpose(0, 1).reshape(rows_r, C)
        pieces, off = [], 0
        for a, b in cols:
            pieces.append(back[off:off + rows_r * (b - a)].view(rows_r, b - a))
            off += rows_r * (b - a)
        return torch.cat(pieces, dim=1)


def fft_rows_sharded(x_shard, inverse: bool = False, out=None, stream=None):
    """Batched FFT of this rank's row shard (rows are independent: no
    collective). x_shard: (rows, n) complex128 tensor on the rank's GPU."""
    from . import device
    return device.fft_batch(x_shard, out=out, inverse=inverse, stream=stream)
