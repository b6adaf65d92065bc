"""Device-pointer entry points of libgdspfft for callers that hold HBM-resident
data in torch tensors (bench.py, distributed.py). torch provides device memory,
streams and torch.distributed only; the transforms are the library's HIP
kernels. Each call is stream-ordered on torch's current stream of the tensor's
device (or the given stream)."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check, lib


def _torch():
    import torch
    return torch


def _stream_ptr(stream, device):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


class Plan:
    """Cached device plan for transform length n on the current device
    (gdsp_plan_create). kind: 0 trivial, 1 LDS Stockham, 2 multi-pass
    Stockham, 3 fused Bluestein, 4 composed Bluestein, 5 mixed radix,
    6 mixed four-step, 7 Rader (a prime n <= 8193 whose n - 1 has a radix
    list; m = n - 1, the cyclic convolution's length), 8 prime-factor Rader
    (composite n = n1 * n2 <= 8192, n2 the prime; m = n2 - 1).
    chirpz=True forces the reference's Bluestein algorithm
    (gdsp_plan_create_chirpz) for a non-trivial length."""

    def __init__(self, n: int, chirpz: bool = False):
        self.n = int(n)
        self.chirpz = bool(chirpz)
        self.handle = ctypes.c_void_p()
        if self.chirpz:
            check(lib().gdsp_plan_create_chirpz(self.n, ctypes.byref(self.handle)),
                  "plan_create_chirpz")
        else:
            check(lib().gdsp_plan_create(self.n, ctypes.byref(self.handle)), "plan_create")
        self.kind = int(lib().gdsp_plan_kind(self.handle))
        v = [ctypes.c_int64() for _ in range(4)]
        rc = ctypes.c_int()
        check(lib().gdsp_plan_info(self.handle, *v, rc), "plan_info")
        # chirp-z convolution length; four-step split; runtime-compiled?
        self.m, self.n1, self.n2 = v[1].value, v[2].value, v[3].value
        self.runtime_compiled = bool(rc.value)
        # output parts of the chirp-z kernel (> 1: n in (8192, 14563] on M = 16384)
        self.parts = int(lib().gdsp_plan_parts(self.handle))
        # the mixed-radix passes (kind 5: the transform; 7 / 8: the Rader
        # convolution's), () for the other kinds
        r = (ctypes.c_int * 16)()
        k = int(lib().gdsp_plan_radices(self.handle, r, 16))
        self.radices = tuple(r[:min(k, 16)])


_plans: dict = {}


def plan(n: int, chirpz: bool = False) -> Plan:
    torch = _torch()
    # the library caches plans per (device, n, algorithm flags): so does this
    key = (torch.cuda.current_device(), int(n), bool(chirpz), int(lib().gdsp_get_algorithm()))
    if key not in _plans:
        _plans[key] = Plan(n, chirpz)
    return _plans[key]


def fft_batch(x, out=None, inverse: bool = False, stream=None, chirpz: bool = False):
    """Batched FFT/IFFT of the rows of a (batch, n) complex128 CUDA tensor
    (chirpz=True: through the forced-Bluestein plan)."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.complex128 and x.dim() == 2 and x.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    assert out.shape == x.shape and out.dtype == x.dtype and out.is_contiguous()
    with torch.cuda.device(x.device):
        p = plan(x.shape[1], chirpz)
        check(lib().gdsp_fft_batch_device(p.handle, _ptr(x), _ptr(out), x.shape[0], int(inverse),
                                          _stream_ptr(stream, x.device)), "fft_batch_device")
    return out


def fft_real_batch(x, out=None, inverse: bool = False, stream=None, chirpz: bool = False):
    """fft.FFTReal / IFFTReal of the rows of a (batch, n) float64 CUDA tensor
    into a complex128 tensor (gdsp_fft_real_batch_device: the kernels read the
    real rows themselves)."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.float64 and x.dim() == 2 and x.is_contiguous()
    if out is None:
        out = torch.empty(x.shape, dtype=torch.complex128, device=x.device)
    assert out.shape == x.shape and out.dtype == torch.complex128 and out.is_contiguous()
    with torch.cuda.device(x.device):
        p = plan(x.shape[1], chirpz)
        check(lib().gdsp_fft_real_batch_device(p.handle, _ptr(x), _ptr(out), x.shape[0],
                                               int(inverse), _stream_ptr(stream, x.device)),
              "fft_real_batch_device")
    return out


def fft2(x, out=None, inverse: bool = False, work=None, stream=None):
    """FFT2/IFFT2 of a (rows, cols) complex128 CUDA tensor."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.complex128 and x.dim() == 2 and x.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    with torch.cuda.device(x.device):
        wp = _ptr(work) if work is not None else ctypes.c_void_p()
        check(lib().gdsp_fft2_device(_ptr(x), _ptr(out), x.shape[0], x.shape[1], int(inverse), wp,
                                     _stream_ptr(stream, x.device)), "fft2_device")
    return out


def fftn(x, out=None, inverse: bool = False, stream=None):
    """FFTN/IFFTN (fft/fft.go:157-192) of a contiguous complex128 CUDA tensor
    of any rank: every axis in turn (gdsp_fftn_device)."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.complex128 and x.is_contiguous() and x.dim() >= 1
    if out is None:
        out = torch.empty_like(x)
    assert out.shape == x.shape and out.is_contiguous()
    if x.numel() == 0:
        return out
    dims = (ctypes.c_int64 * x.dim())(*x.shape)
    with torch.cuda.device(x.device):
        check(lib().gdsp_fftn_device(_ptr(x), _ptr(out), dims, x.dim(), int(inverse),
                                     _stream_ptr(stream, x.device)), "fftn_device")
    return out


def fft_axis(x, axis: int, out=None, inverse: bool = False, stream=None):
    """The 1-D FFT/IFFT along one axis of a contiguous complex128 CUDA tensor
    (gdsp_fft_axis_device; axis 0 of a matrix = computeFFT2's column pass)."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.complex128 and x.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    assert out.shape == x.shape and out.is_contiguous()
    if x.numel() == 0:
        return out
    dims = (ctypes.c_int64 * x.dim())(*x.shape)
    with torch.cuda.device(x.device):
        check(lib().gdsp_fft_axis_device(_ptr(x), _ptr(out), dims, x.dim(), axis % x.dim(),
                                         int(inverse), _stream_ptr(stream, x.device)),
              "fft_axis_device")
    return out


def fill_uniform(t, seed: int, offset: int = 0, stream=None):
    """Fill a float64 (or complex128, as interleaved pairs) CUDA tensor with the
    counter-based uniform[-1,1) generator."""
    torch = _torch()
    assert t.is_cuda and t.is_contiguous()
    count = t.numel() * (2 if t.dtype == torch.complex128 else 1)
    with torch.cuda.device(t.device):
        check(lib().gdsp_fill_uniform_device(_ptr(t), count, seed, offset,
                                             _stream_ptr(stream, t.device)), "fill_uniform")
    return t


def pwelch_accumulate(x, nfft: int, pad: int, noverlap: int, seg_begin: int, seg_end: int,
                      win_seg, acc, stream=None):
    """Adds the per-bin power sums of segments [seg_begin, seg_end) of the
    float64 CUDA signal x into acc (float64, max(pad, nfft) entries)."""
    torch = _torch()
    assert x.is_cuda and x.dtype == torch.float64 and acc.dtype == torch.float64
    with torch.cuda.device(x.device):
        check(lib().gdsp_pwelch_accumulate_device(
            _ptr(x), x.numel(), nfft, pad, noverlap, seg_begin, seg_end, _ptr(win_seg), _ptr(acc),
            _stream_ptr(stream, x.device)), "pwelch_accumulate")
    return acc
