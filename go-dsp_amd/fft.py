"""Host mirror of go-dsp's `fft` package (fft/fft.go, fft/radix2.go,
fft/bluestein.go) over the libgdspfft C ABI. Same names, argument meaning and
panics as the Go API; slices become numpy arrays. Every transform runs on the
GPU (gfx950 kernels); nothing here computes a transform on the CPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import Panic, check, lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(_lib._P)


def _as_c(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.complex128).reshape(-1))


def _as_f(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))


def FFT(x) -> np.ndarray:
    """fft.FFT — fft/fft.go:72-87. Returns a new array; x is not modified."""
    x = _as_c(x)
    out = np.empty_like(x)
    check(lib().gdsp_fft(_p(x), _p(out), x.size), "FFT")
    return out


def IFFT(x) -> np.ndarray:
    """fft.IFFT — fft/fft.go:35-52. Panics (index out of range) on len 0."""
    x = _as_c(x)
    if x.size == 0:
        raise Panic(_lib.GDSP_ERR_EMPTY, "runtime error: index out of range [0] with length 0")
    out = np.empty_like(x)
    check(lib().gdsp_ifft(_p(x), _p(out), x.size), "IFFT")
    return out


def FFTReal(x) -> np.ndarray:
    """fft.FFTReal — fft/fft.go:25-27 (full N-point complex spectrum)."""
    x = _as_f(x)
    out = np.empty(x.size, np.complex128)
    check(lib().gdsp_fft_real(_p(x), _p(out), x.size), "FFTReal")
    return out


def IFFTReal(x) -> np.ndarray:
    """fft.IFFTReal — fft/fft.go:30-32."""
    x = _as_f(x)
    if x.size == 0:
        raise Panic(_lib.GDSP_ERR_EMPTY, "runtime error: index out of range [0] with length 0")
    out = np.empty(x.size, np.complex128)
    check(lib().gdsp_ifft_real(_p(x), _p(out), x.size), "IFFTReal")
    return out


def Convolve(x, y) -> np.ndarray:
    """fft.Convolve — fft/fft.go:55-69."""
    x, y = _as_c(x), _as_c(y)
    if x.size != y.size:
        raise Panic(_lib.GDSP_ERR_UNEQUAL, "arrays not of equal size")
    out = np.empty_like(x)
    check(lib().gdsp_convolve(_p(x), _p(y), _p(out), x.size), "Convolve")
    return out


def FFTBatch(x, inverse: bool = False) -> np.ndarray:
    """Additive batched entry point: FFT (or IFFT) of every row
    of a (batch, n) complex array, in one GPU launch."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.complex128))
    if x.ndim != 2:
        raise ValueError("FFTBatch expects a 2-D (batch, n) array")
    out = np.empty_like(x)
    check(lib().gdsp_fft_batch(_p(x), _p(out), x.shape[1], x.shape[0], int(inverse)), "FFTBatch")
    return out


def FFTRealBatch(x) -> np.ndarray:
    """FFTReal of every row of a (batch, n) float64 array."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if x.ndim != 2:
        raise ValueError("FFTRealBatch expects a 2-D (batch, n) array")
    out = np.empty(x.shape, np.complex128)
    check(lib().gdsp_fft_real_batch(_p(x), _p(out), x.shape[1], x.shape[0]), "FFTRealBatch")
    return out


def _matrix(x, dtype) -> np.ndarray:
    """Flatten [][]T after the reference's checks (fft/fft.go:124-136)."""
    if isinstance(x, np.ndarray):
        if x.ndim != 2 or x.shape[0] == 0:
            if x.ndim == 2 or x.size == 0:
                raise Panic(_lib.GDSP_ERR_EMPTY, "empty input array")
            raise ValueError("expected a 2-D matrix")
        return np.ascontiguousarray(x, dtype=dtype)
    rows = list(x)
    if len(rows) == 0:
        raise Panic(_lib.GDSP_ERR_EMPTY, "empty input array")
    cols = len(rows[0])
    for r in rows:
        if len(r) != cols:
            raise Panic(_lib.GDSP_ERR_RAGGED, "ragged input array")
    return np.ascontiguousarray(np.asarray(rows, dtype=dtype).reshape(len(rows), cols))


def _fft2(x, real: bool, inverse: bool) -> np.ndarray:
    m = _matrix(x, np.float64 if real else np.complex128)
    out = np.empty(m.shape, np.complex128)
    fn = lib().gdsp_fft2_real if real else lib().gdsp_fft2
    check(fn(_p(m), _p(out), m.shape[0], m.shape[1], int(inverse)), "FFT2")
    return out


def FFT2(x) -> np.ndarray:
    """fft.FFT2 — fft/fft.go:109-111 (computeFFT2 :123-154)."""
    return _fft2(x, False, False)


def IFFT2(x) -> np.ndarray:
    """fft.IFFT2 — fft/fft.go:119-121."""
    return _fft2(x, False, True)


def FFT2Real(x) -> np.ndarray:
    """fft.FFT2Real — fft/fft.go:104-106."""
    return _fft2(x, True, False)


def IFFT2Real(x) -> np.ndarray:
    """fft.IFFT2Real — fft/fft.go:114-116."""
    return _fft2(x, True, True)


def _fftn(m, inverse: bool):
    from .dsputils import MakeMatrix
    x = np.ascontiguousarray(m.list, dtype=np.complex128)
    dims = np.ascontiguousarray(np.asarray(m.dims, dtype=np.int64))
    out = np.empty_like(x)
    check(lib().gdsp_fftn(_p(x), _p(out), _p(dims), dims.size, int(inverse)), "FFTN")
    return MakeMatrix(out, list(m.dims))


def FFTN(m):
    """fft.FFTN — fft/fft.go:157-159 (computeFFTN :166-192): N-D DFT of a
    dsputils.Matrix; returns a new Matrix."""
    return _fftn(m, False)


def IFFTN(m):
    """fft.IFFTN — fft/fft.go:162-164."""
    return _fftn(m, True)


def SetWorkerPoolSize(n: int) -> None:
    """fft.SetWorkerPoolSize — fft/fft.go:95-101 (recorded; the GPU path has no
    goroutine pool)."""
    lib().gdsp_set_worker_pool_size(int(n))


def EnsureRadix2Factors(input_len: int) -> None:
    """fft.EnsureRadix2Factors — fft/radix2.go:35-37: pre-build the device plan
    (twiddle table, and for non-powers of 2 the Bluestein tables)."""
    check(lib().gdsp_ensure_plan(int(input_len)), "EnsureRadix2Factors")


# ---- multi-device (include/gdsp_fft.h "multi-device") ---------------------
# The reference hides its parallelism inside each call (radix2.go:89-151);
# these select and use the GPUs of the node the same way.

def _dev_array(devices):
    import ctypes
    if devices is None:
        return None, 0
    ids = [int(d) for d in devices]
    return (ctypes.c_int * len(ids))(*ids), len(ids)


def SetDevices(devices=None) -> None:
    """Device set of the host-pointer calls (gdsp_set_devices): once set to
    more than one entry, large FFTBatch / FFTRealBatch / spectral.Pwelch calls
    split over it. A device may repeat (its shards then share it on separate
    streams). None or [] restores the default: the calling thread's current
    device (or GDSP_DEVICES), i.e. no automatic split."""
    arr, n = _dev_array(devices or [])
    check(lib().gdsp_set_devices(arr, n), "SetDevices")


def Devices() -> list[int]:
    """The current device set (gdsp_get_devices); [] without a GPU."""
    import ctypes
    n = int(lib().gdsp_get_devices(None, 0))
    arr = (ctypes.c_int * max(n, 1))()
    n = int(lib().gdsp_get_devices(arr, n))
    return list(arr[:n])


# algorithm selection (gdsp_set_algorithm, include/gdsp_fft.h)
ALGO_DEFAULT = 0
ALGO_GENERIC_MIXED = 1
ALGO_NO_CHIRPZ_PARTS = 2
ALGO_CHIRPZ_POW2 = 4
ALGO_CHIRPZ_UNFUSED = 8
ALGO_NO_RADER = 16
ALGO_NO_RACE = 32


def SetAlgorithm(flags: int = ALGO_DEFAULT) -> None:
    """Select alternative paths of the engine (same DFT) for plans built and
    Pwelch calls made after this call (gdsp_set_algorithm)."""
    check(lib().gdsp_set_algorithm(int(flags)), "SetAlgorithm")


def Algorithm() -> int:
    return int(lib().gdsp_get_algorithm())


def MultiStats() -> dict:
    """gdsp_multi_stats: calls split over a device set since process start,
    and how Pwelch accumulators were combined."""
    import ctypes
    v = [ctypes.c_int64() for _ in range(4)]
    check(lib().gdsp_multi_stats(*[ctypes.byref(a) for a in v]), "MultiStats")
    return dict(zip(("batch_calls", "pwelch_calls", "rccl_reduces", "host_reduces"),
                    (a.value for a in v)))


def FFTBatchMulti(x, inverse: bool = False, devices=None) -> np.ndarray:
    """FFTBatch split over `devices` (None: the device set): contiguous row
    shards, one per device, no collective (gdsp_fft_batch_multi)."""
    x = np.ascontiguousarray(np.asarray(x, dtype=np.complex128))
    if x.ndim != 2:
        raise ValueError("FFTBatchMulti expects a 2-D (batch, n) array")
    out = np.empty_like(x)
    arr, n = _dev_array(devices)
    check(lib().gdsp_fft_batch_multi(_p(x), _p(out), x.shape[1], x.shape[0], int(inverse),
                                     arr, n), "FFTBatchMulti")
    return out


def batch_shard(batch: int, ndev: int, i: int) -> tuple[int, int]:
    """Rows [lo, hi) of shard i of ndev (gdsp_batch_shard; host arithmetic)."""
    lo, hi = _lib._I64(0), _lib._I64(0)
    check(lib().gdsp_batch_shard(int(batch), int(ndev), int(i), lo, hi), "batch_shard")
    return lo.value, hi.value
