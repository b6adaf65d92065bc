"""Host mirror of go-dsp's `dsputils` helpers used on the FFT/Pwelch path
(dsputils/dsputils.go:25-83, dsputils/compare.go:24-96). Pure host utilities:
slice conversion, padding and the tolerance comparators."""
from __future__ import annotations

import math

import numpy as np

closeFactor = 1e-8  # dsputils/compare.go:24


def ToComplex(x) -> np.ndarray:
    """dsputils.go:25-31."""
    return np.asarray(x, dtype=np.float64).astype(np.complex128)


def ToComplex2(x):
    """dsputils.go:77-83."""
    return [ToComplex(r) for r in x]


def IsPowerOf2(x: int) -> bool:
    """dsputils.go:34-36 (true for 0, as in the reference)."""
    return x & (x - 1) == 0


def NextPowerOf2(x: int) -> int:
    """dsputils.go:39-45 (float Log2/Ceil/Pow, as in the reference)."""
    if IsPowerOf2(x):
        return x
    return int(math.pow(2, math.ceil(math.log2(float(x)))))


def ZeroPad(x, length: int) -> np.ndarray:
    """dsputils.go:49-57: x itself if already long enough."""
    x = np.asarray(x, dtype=np.complex128)
    if x.size >= length:
        return x
    r = np.zeros(length, np.complex128)
    r[:x.size] = x
    return r


def ZeroPadF(x, length: int) -> np.ndarray:
    """dsputils.go:61-69."""
    x = np.asarray(x, dtype=np.float64)
    if x.size >= length:
        return x
    r = np.zeros(length, np.float64)
    r[:x.size] = x
    return r


def ZeroPad2(x) -> np.ndarray:
    """dsputils.go:72-74."""
    return ZeroPad(x, NextPowerOf2(len(x)))


def Float64Equal(a: float, b: float) -> bool:
    """compare.go:94-96: |a-b| <= 1e-8 or |1-a/b| <= 1e-8."""
    if abs(a - b) <= closeFactor:
        return True
    with np.errstate(divide="ignore", invalid="ignore"):
        return bool(abs(1 - np.float64(a) / np.float64(b)) <= closeFactor)


def ComplexEqual(a: complex, b: complex) -> bool:
    """compare.go:84-91."""
    return Float64Equal(a.real, b.real) and Float64Equal(a.imag, b.imag)


def PrettyClose(a, b) -> bool:
    """compare.go:28-39."""
    return len(a) == len(b) and all(Float64Equal(float(c), float(d)) for c, d in zip(a, b))


def PrettyCloseC(a, b) -> bool:
    """compare.go:42-53."""
    return len(a) == len(b) and all(ComplexEqual(complex(c), complex(d)) for c, d in zip(a, b))


def PrettyClose2(a, b) -> bool:
    """compare.go:56-67."""
    return len(a) == len(b) and all(PrettyCloseC(c, d) for c, d in zip(a, b))


def PrettyClose2F(a, b) -> bool:
    """compare.go:70-81."""
    return len(a) == len(b) and all(PrettyClose(c, d) for c, d in zip(a, b))
