"""TEST INFRASTRUCTURE ONLY — ctypes view of the C restatement of the go-dsp
reference (oracle/oracle.c). Imported only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; the product package never imports it.

Each wrapper names the reference function it restates (file:line under
maddyblue/go-dsp).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

WINDOWS = {"hann": 0, "hamming": 1, "rectangular": 2, "bartlett": 3, "flattop": 4,
           "blackman": 5}


class OracleError(RuntimeError):
    pass


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        I64 = ctypes.c_int64
        for name, args in {
            "or_fft": [P, P, I64], "or_ifft": [P, P, I64], "or_fft_real": [P, P, I64],
            "or_ifft_real": [P, P, I64], "or_convolve": [P, P, P, I64],
            "or_fft2": [P, P, I64, I64, ctypes.c_int],
            "or_fft_threaded": [P, P, I64, ctypes.c_int],
            "or_fft_rows_threaded": [P, P, I64, I64, ctypes.c_int],
            "or_window": [ctypes.c_int, I64, P], "or_radix2_factors": [I64, P],
            "or_pwelch": [P, I64, ctypes.c_double, I64, I64, I64, ctypes.c_int,
                          ctypes.c_int, P, P, P],
        }.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ctypes.c_int
        L.or_pwelch_threaded.argtypes = [P, I64, ctypes.c_double, I64, I64, I64, ctypes.c_int,
                                         ctypes.c_int, P, P, P, ctypes.c_int]
        L.or_pwelch_threaded.restype = ctypes.c_int
        L.or_fftn.argtypes = [P, P, P, ctypes.c_int, ctypes.c_int]
        L.or_fftn.restype = ctypes.c_int
        L.or_segment_count.argtypes = [I64, I64, I64]
        L.or_segment_count.restype = I64
        L.or_reverse_bits.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_reverse_bits.restype = ctypes.c_uint64
        L.or_next_pow2.argtypes = [I64]
        L.or_next_pow2.restype = I64
        L.or_is_pow2.argtypes = [I64]
        L.or_is_pow2.restype = ctypes.c_int
        L.or_fill_uniform.argtypes = [P, I64, ctypes.c_uint64, ctypes.c_uint64]
        L.or_fill_uniform.restype = None
        L.or_wav_floats.argtypes = [P, I64, ctypes.c_int, ctypes.c_int, P]
        L.or_wav_floats.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(st: int, what: str):
    if st != 0:
        raise OracleError(f"{what}: status {st}")


def _c(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.complex128))


def _f(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


def fft(x) -> np.ndarray:
    """fft.FFT, fft/fft.go:72-87."""
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().or_fft(_p(x), _p(out), x.size), "fft")
    return out


def ifft(x) -> np.ndarray:
    """fft.IFFT, fft/fft.go:35-52."""
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().or_ifft(_p(x), _p(out), x.size), "ifft")
    return out


def fft_real(x) -> np.ndarray:
    """fft.FFTReal, fft/fft.go:25-27."""
    x = _f(x)
    out = np.empty(x.size, np.complex128)
    _check(lib().or_fft_real(_p(x), _p(out), x.size), "fft_real")
    return out


def ifft_real(x) -> np.ndarray:
    """fft.IFFTReal, fft/fft.go:30-32."""
    x = _f(x)
    out = np.empty(x.size, np.complex128)
    _check(lib().or_ifft_real(_p(x), _p(out), x.size), "ifft_real")
    return out


def convolve(x, y) -> np.ndarray:
    """fft.Convolve, fft/fft.go:55-69."""
    x, y = _c(x), _c(y)
    if x.size != y.size:
        raise OracleError("arrays not of equal size")
    out = np.empty_like(x)
    _check(lib().or_convolve(_p(x), _p(y), _p(out), x.size), "convolve")
    return out


def fft_rows(x) -> np.ndarray:
    """fft.FFT applied to every row of a 2-D array (one reference call per row)."""
    x = _c(x)
    out = np.empty_like(x)
    for i in range(x.shape[0]):
        _check(lib().or_fft(_p(x[i]), _p(out[i]), x.shape[1]), "fft")
    return out


def ifft_rows(x) -> np.ndarray:
    x = _c(x)
    out = np.empty_like(x)
    for i in range(x.shape[0]):
        _check(lib().or_ifft(_p(x[i]), _p(out[i]), x.shape[1]), "ifft")
    return out


def fft_rows_threaded(x, nworkers: int) -> np.ndarray:
    """Reference-threaded radix-2 per row (fft/radix2.go:89-151 structure)."""
    x = _c(x)
    out = np.empty_like(x)
    _check(lib().or_fft_rows_threaded(_p(x), _p(out), x.shape[1], x.shape[0], nworkers),
           "fft_rows_threaded")
    return out


def fft2(x, inverse: bool = False) -> np.ndarray:
    """fft.FFT2 / IFFT2, fft/fft.go:104-154 (column pass then row pass)."""
    x = _c(x)
    if x.ndim != 2 or x.shape[0] == 0:
        raise OracleError("empty input array")
    out = np.empty_like(x)
    _check(lib().or_fft2(_p(x), _p(out), x.shape[0], x.shape[1], int(inverse)), "fft2")
    return out


def fftn(x, dims, inverse: bool = False) -> np.ndarray:
    """fft.FFTN / IFFTN, fft/fft.go:157-192, on the flat row-major data of a
    Matrix of the given dims."""
    x = _c(x).ravel()
    d = np.ascontiguousarray(np.asarray(dims, dtype=np.int64))
    out = np.empty_like(x)
    _check(lib().or_fftn(_p(x), _p(out), _p(d), d.size, int(inverse)), "fftn")
    return out


def window(kind: str, L: int) -> np.ndarray:
    """window.{Hann,Hamming,Rectangular,Bartlett,FlatTop,Blackman}, window/window.go."""
    out = np.empty(max(L, 0), np.float64)
    _check(lib().or_window(WINDOWS[kind], L, _p(out)), "window")
    return out


def radix2_factors(n: int) -> np.ndarray:
    """getRadix2Factors, fft/radix2.go:39-69."""
    out = np.empty(n, np.complex128)
    _check(lib().or_radix2_factors(n, _p(out)), "radix2_factors")
    return out


def reverse_bits(v: int, s: int) -> int:
    """reverseBits, fft/radix2.go:184-199."""
    return int(lib().or_reverse_bits(v, s))


def next_pow2(x: int) -> int:
    """dsputils.NextPowerOf2, dsputils/dsputils.go:39-45."""
    return int(lib().or_next_pow2(x))


def segment_count(lx: int, size: int, noverlap: int) -> int:
    """Segment count of spectral.Segment, spectral/spectral.go:22-33."""
    return int(lib().or_segment_count(lx, size, noverlap))


def segment(x, size: int, noverlap: int):
    """spectral.Segment, spectral/spectral.go:22-47."""
    x = _f(x)
    n = segment_count(x.size, size, noverlap)
    if n < 0:
        raise OracleError("integer divide by zero")
    stride = size - noverlap
    return [x[i * stride:i * stride + size].copy() for i in range(n)]


def pwelch(x, fs: float, nfft: int = 0, pad: int = 0, noverlap: int = 0,
           window_kind: str = "hann", scale_off: bool = False):
    """spectral.Pwelch, spectral/pwelch.go:74-145."""
    x = _f(x)
    nf = nfft or 256
    pd = pad or nf
    lp = pd // 2 + 1
    pxx = np.empty(lp, np.float64)
    freqs = np.empty(lp, np.float64)
    lpo = ctypes.c_int64(0)
    _check(lib().or_pwelch(_p(x), x.size, float(fs), nfft, pad, noverlap,
                           WINDOWS[window_kind], int(scale_off), _p(pxx), _p(freqs),
                           ctypes.byref(lpo)), "pwelch")
    return pxx[:lpo.value].copy(), freqs[:lpo.value].copy()


def pwelch_threaded(x, fs: float, nfft: int, noverlap: int, nworkers: int):
    """spectral.Pwelch with the reference's worker pool in every FFT (CPU
    baseline only)."""
    x = _f(x)
    lp = (nfft or 256) // 2 + 1
    pxx = np.empty(lp, np.float64)
    freqs = np.empty(lp, np.float64)
    lpo = ctypes.c_int64(0)
    _check(lib().or_pwelch_threaded(_p(x), x.size, float(fs), nfft, 0, noverlap, 0, 0, _p(pxx),
                                    _p(freqs), ctypes.byref(lpo), nworkers), "pwelch_threaded")
    return pxx, freqs


def pwelch_chunked(x, fs: float, nfft: int, noverlap: int, nthreads: int = 16,
                   chunks: int = 64):
    """spectral.Pwelch (spectral/pwelch.go:74-145) of a long stream, for the
    full-size parity checks: the segments split into `chunks` contiguous
    ranges, each range's Pwelch by or_pwelch on its own sample span
    (segments s0 .. s1 - 1 need samples [s0 stride, (s1 - 1) stride + nfft)),
    run on `nthreads` host threads (ctypes releases the GIL), and the results
    combined as the segment-count-weighted mean. pwelch.go:126-136 finalises
    the per-bin power sum linearly (1 / nsegs, the window norm, the doubling of
    interior bins), so that mean is the whole stream's Pxx; only the order of
    the float64 additions differs from the reference's single pass. Pad = NFFT,
    Hann, scaling on."""
    from concurrent.futures import ThreadPoolExecutor
    x = _f(x)
    nf = nfft or 256
    nsegs = segment_count(x.size, nf, noverlap)
    stride = nf - noverlap
    if nsegs <= 0:
        return pwelch(x, fs, nfft=nfft, noverlap=noverlap)
    chunks = max(1, min(chunks, nsegs))
    bounds = [nsegs * i // chunks for i in range(chunks + 1)]

    def one(i):
        s0, s1 = bounds[i], bounds[i + 1]
        if s1 <= s0:
            return None
        p, f = pwelch(x[s0 * stride:(s1 - 1) * stride + nf], fs, nfft=nfft, noverlap=noverlap)
        return s1 - s0, p, f

    with ThreadPoolExecutor(max_workers=max(1, nthreads)) as ex:
        parts = [r for r in ex.map(one, range(chunks)) if r is not None]
    total = sum(k for k, _, _ in parts)
    pxx = sum(k * p for k, p, _ in parts) / total
    return pxx, parts[0][2]


def fill_uniform(count: int, seed: int, offset: int = 0) -> np.ndarray:
    """Synthetic inputs identical to the device generator."""
    out = np.empty(count, np.float64)
    lib().or_fill_uniform(_p(out), count, seed, offset)
    return out


def wav_floats(raw: bytes, count: int, audio_format: int, bits_per_sample: int) -> np.ndarray:
    """wav.ReadFloats's conversion (wav/wav.go:135-161) of `count` samples
    of little-endian bytes; float32 like the reference."""
    buf = np.frombuffer(bytes(raw), dtype=np.uint8)
    out = np.empty(count, np.float32)
    st = lib().or_wav_floats(_p(buf), count, audio_format, bits_per_sample, _p(out))
    if st != 0:
        raise ValueError("wav: unknown format")
    return out
