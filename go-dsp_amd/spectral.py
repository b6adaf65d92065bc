"""Host mirror of go-dsp's `spectral` package (spectral/pwelch.go,
spectral/spectral.go). Pwelch runs the fused GPU kernel (window +
packed-pair FFT + |X|^2 accumulation) through gdsp_pwelch."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import _lib, window
from ._lib import Panic, check, lib


@dataclass
class PwelchOptions:
    """spectral/pwelch.go:28-65 (zero values select the defaults)."""
    NFFT: int = 0
    Window: Optional[Callable[[int], np.ndarray]] = None
    Pad: int = 0
    Noverlap: int = 0
    Scale_off: bool = False


def _p(a: np.ndarray):
    return a.ctypes.data_as(_lib._P)


def segment_count(lx: int, size: int, noverlap: int) -> int:
    """Segment count of spectral.Segment (spectral/spectral.go:22-33)."""
    c = _lib._I64(0)
    check(lib().gdsp_segment_count(lx, size, noverlap, c), "Segment")
    return int(c.value)


def Segment(x, size: int, noverlap: int):
    """spectral.Segment — spectral/spectral.go:22-47: copies of each segment
    (the GPU path never materialises them; this is the host API)."""
    x = np.asarray(x, dtype=np.float64)
    n = segment_count(x.size, size, noverlap)
    stride = size - noverlap
    return [x[i * stride:i * stride + size].copy() for i in range(n)]


def resolve_options(o: Optional[PwelchOptions]):
    """Defaults of spectral/pwelch.go:79-95; a nil options pointer panics."""
    if o is None:
        raise Panic(_lib.GDSP_ERR_INVALID,
                    "runtime error: invalid memory address or nil pointer dereference")
    nfft = o.NFFT or 256
    pad = o.Pad or nfft
    wf = o.Window or window.Hann
    return nfft, pad, o.Noverlap, wf, not o.Scale_off


def Pwelch(x, Fs: float, o: Optional[PwelchOptions]):
    """spectral.Pwelch — spectral/pwelch.go:74-145. Returns (Pxx, freqs)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if x.size == 0:
        return np.zeros(0), np.zeros(0)
    nfft, pad, noverlap, wf, scaling = resolve_options(o)
    flen = max(pad, nfft)
    win_seg = np.ascontiguousarray(wf(flen), dtype=np.float64)
    win_nfft = np.ascontiguousarray(wf(nfft), dtype=np.float64)
    lp = pad // 2 + 1
    pxx = np.empty(lp, np.float64)
    freqs = np.empty(lp, np.float64)
    lpo = _lib._I64(0)
    check(lib().gdsp_pwelch(_p(x), x.size, float(Fs), nfft, pad, noverlap, _p(win_seg),
                            _p(win_nfft), int(not scaling), _p(pxx), _p(freqs), lpo), "Pwelch")
    return pxx[:lpo.value], freqs[:lpo.value]


def finalize(acc: np.ndarray, nsegs: int, nfft: int, pad: int, win_nfft: np.ndarray, Fs: float,
             scale_off: bool):
    """Host finalisation (gdsp_pwelch_finalize, spectral/pwelch.go:113-142) of
    summed accumulators acc[0..flen)."""
    acc = np.ascontiguousarray(acc, dtype=np.float64)
    win_nfft = np.ascontiguousarray(win_nfft, dtype=np.float64)
    lp = pad // 2 + 1
    pxx = np.empty(lp, np.float64)
    freqs = np.empty(lp, np.float64)
    check(lib().gdsp_pwelch_finalize(_p(acc), acc.size, nsegs, nfft, pad, _p(win_nfft),
                                     float(Fs), int(scale_off), _p(pxx), _p(freqs)),
          "pwelch_finalize")
    return pxx, freqs


def PwelchMulti(x, Fs: float, o: Optional[PwelchOptions], devices=None):
    """spectral.Pwelch split over `devices` (None: the library's device set):
    segment shards with their halos, per-device accumulation and one
    in-process RCCL reduce of the per-bin sums (gdsp_pwelch_multi)."""
    from .fft import _dev_array
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
    if x.size == 0:
        return np.zeros(0), np.zeros(0)
    nfft, pad, noverlap, wf, scaling = resolve_options(o)
    flen = max(pad, nfft)
    win_seg = np.ascontiguousarray(wf(flen), dtype=np.float64)
    win_nfft = np.ascontiguousarray(wf(nfft), dtype=np.float64)
    lp = pad // 2 + 1
    pxx = np.empty(lp, np.float64)
    freqs = np.empty(lp, np.float64)
    lpo = _lib._I64(0)
    arr, n = _dev_array(devices)
    check(lib().gdsp_pwelch_multi(_p(x), x.size, float(Fs), nfft, pad, noverlap, _p(win_seg),
                                  _p(win_nfft), int(not scaling), _p(pxx), _p(freqs), lpo,
                                  arr, n), "PwelchMulti")
    return pxx[:lpo.value], freqs[:lpo.value]


def pwelch_shard(nsegs: int, nfft: int, noverlap: int, ndev: int, i: int):
    """(seg_lo, seg_hi, x_lo, x_hi) of device shard i (gdsp_pwelch_shard)."""
    v = [_lib._I64(0) for _ in range(4)]
    check(lib().gdsp_pwelch_shard(int(nsegs), int(nfft), int(noverlap), int(ndev), int(i), *v),
          "pwelch_shard")
    return tuple(a.value for a in v)
