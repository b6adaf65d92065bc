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


def Segment(x, segs: int, noverlap: float):
    """dsputils.Segment — dsputils/dsputils.go:89-120: segs equal-length
    views into x with a fractional overlap noverlap (0 <= noverlap <= 1);
    the longest length that fits wins, trailing entries are dropped. Panics
    "too many segments" when none fits. Host index arithmetic (not on the
    GPU path); the results are numpy views, as the reference's are slices."""
    x = np.asarray(x)
    lx = len(x)
    length = lx
    step = 0
    while length > 0:
        overlap = int(float(length) * noverlap)  # Go int() truncates toward zero
        tot = segs * (length - overlap) + overlap
        if tot <= lx:
            step = length - overlap
            break
        length -= 1
    if length == 0:
        raise _panic("too many segments")
    return [x[n * step:n * step + length] for n in range(segs)]


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


class Matrix:
    """dsputils.Matrix — dsputils/matrix.go:21-216: an N-D row-major complex128
    array with whole-axis get/set (the container fft.FFTN transforms)."""

    def __init__(self, lst: np.ndarray, dims, offsets):
        self.list = lst
        self.dims = list(dims)
        self.offsets = list(offsets)

    def offset(self, dims) -> int:
        """matrix.go:93-107 (an index of -1 is used as is, like the reference)."""
        if len(dims) != len(self.dims):
            raise _panic("incorrect dimensions")
        i = 0
        for n, v in enumerate(dims):
            if v > self.dims[n]:
                raise _panic("incorrect dimensions")
            i += v * self.offsets[n]
        return i

    def indexes(self, dims):
        """matrix.go:110-142."""
        i = -1
        for n, v in enumerate(dims):
            if v == -1:
                if i >= 0:
                    raise _panic("only one dimension index allowed")
                i = n
            elif v >= self.dims[n]:
                raise _panic("dimension out of bounds")
        if i == -1:
            raise _panic("must specify one dimension index")
        x = sum(self.offsets[n] * v for n, v in enumerate(dims) if v >= 0)
        return x + self.offsets[i] * np.arange(self.dims[i])

    def Dimensions(self):
        """matrix.go:144-149."""
        return list(self.dims)

    def Dim(self, dims) -> np.ndarray:
        """matrix.go:156-164."""
        return self.list[self.indexes(dims)].copy()

    def SetDim(self, x, dims) -> None:
        """matrix.go:166-177."""
        inds = self.indexes(dims)
        x = np.asarray(x, np.complex128)
        if x.size != inds.size:
            raise _panic("incorrect array length")
        self.list[inds] = x

    def Value(self, dims) -> complex:
        """matrix.go:179-183."""
        return complex(self.list[self.offset(dims)])

    def SetValue(self, x, dims) -> None:
        """matrix.go:185-189."""
        self.list[self.offset(dims)] = x

    def To2D(self):
        """matrix.go:191-205."""
        if len(self.dims) != 2:
            raise _panic("can only convert 2-D Matrixes")
        return [self.list[i * self.dims[1]:(i + 1) * self.dims[1]].copy()
                for i in range(self.dims[0])]

    def Copy(self) -> "Matrix":
        """matrix.go:75-80."""
        return Matrix(self.list.copy(), self.dims, self.offsets)

    def PrettyClose(self, n: "Matrix") -> bool:
        """matrix.go:207-216."""
        if any(v != n.dims[i] for i, v in enumerate(self.dims)):
            return False
        return PrettyCloseC(self.list, n.list)


def _panic(msg: str):
    from ._lib import GDSP_ERR_INVALID, Panic
    return Panic(GDSP_ERR_INVALID, msg)


def MakeMatrix(x, dims) -> Matrix:
    """matrix.go:37-57 (x is used as the backing store, not copied)."""
    length = 1
    offsets = [0] * len(dims)
    for i in range(len(dims) - 1, -1, -1):
        if dims[i] < 1:
            raise _panic("invalid dimensions")
        offsets[i] = length
        length *= dims[i]
    x = np.asarray(x)
    if x.dtype != np.complex128:
        x = x.astype(np.complex128)
    x = x.reshape(-1)
    if x.size != length:
        raise _panic("incorrect dimensions")
    return Matrix(x, list(dims), offsets)


def MakeMatrix2(x) -> Matrix:
    """matrix.go:60-73."""
    dims = [len(x), len(x[0])]
    r = np.zeros(dims[0] * dims[1], np.complex128)
    for n, v in enumerate(x):
        if len(v) != dims[1]:
            raise _panic("ragged array")
        r[n * dims[1]:(n + 1) * dims[1]] = v
    return MakeMatrix(r, dims)


def MakeEmptyMatrix(dims) -> Matrix:
    """matrix.go:83-90."""
    return MakeMatrix(np.zeros(int(np.prod(dims)), np.complex128), dims)
