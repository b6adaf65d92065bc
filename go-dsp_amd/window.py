"""Host mirror of go-dsp's `window` package (window/window.go). The window
tables are generated on the host, once per call (the reference recomputes them
per segment, window.go:25-29); the GPU Pwelch kernel applies them."""
from __future__ import annotations

import ctypes
import functools
import math
from typing import Callable

import numpy as np

from . import _lib


def _cached(fn):
    """Window tables depend only on L: compute once (the reference recomputes
    them for every segment, window.go:25-29) and hand out copies."""
    table = functools.lru_cache(maxsize=64)(lambda L: fn(L))

    @functools.wraps(fn)
    def wrapper(L: int) -> np.ndarray:
        return table(int(L)).copy()
    return wrapper


def Apply(x: np.ndarray, windowFunction: Callable[[int], np.ndarray]) -> None:
    """window.go:25-29 — in place, the only mutating function of the path."""
    w = windowFunction(len(x))
    for i in range(len(w)):
        x[i] *= w[i]


@_cached
def Rectangular(L: int) -> np.ndarray:
    """window.go:32-40."""
    return np.ones(L, np.float64)


def _sym(L: int, f) -> np.ndarray:
    r = np.zeros(L, np.float64)
    if L == 1:
        r[0] = 1
    elif L > 1:
        N = L - 1
        for n in range(N + 1):
            r[n] = f(n, N)
    return r


@_cached
def Hamming(L: int) -> np.ndarray:
    """window.go:44-58."""
    return _sym(L, lambda n, N: 0.54 - 0.46 * math.cos(math.pi * 2 / float(N) * float(n)))


@_cached
def Hann(L: int) -> np.ndarray:
    """window.go:62-76 (the C ABI's host generator, gdsp_window_hann)."""
    out = np.empty(max(L, 0), np.float64)
    _lib.check(_lib.lib().gdsp_window_hann(L, out.ctypes.data_as(ctypes.c_void_p)), "Hann")
    return out


@_cached
def Bartlett(L: int) -> np.ndarray:
    """window.go:80-98."""
    r = np.zeros(L, np.float64)
    if L == 1:
        r[0] = 1
    elif L > 1:
        N = L - 1
        coef = 2 / float(N)
        n = 0
        while n <= N // 2:
            r[n] = coef * float(n)
            n += 1
        while n <= N:
            r[n] = 2 - coef * float(n)
            n += 1
    return r


@_cached
def FlatTop(L: int) -> np.ndarray:
    """window.go:102-135."""
    a0, a1, a2, a3, a4 = 0.21557895, 0.41663158, 0.277263158, 0.083578947, 0.006947368

    def f(n, N):
        fac = float(n) * (2 * math.pi / float(N))
        return (a0 - a1 * math.cos(fac) + a2 * math.cos(2 * fac) - a3 * math.cos(3 * fac)
                + a4 * math.cos(4 * fac))
    return _sym(L, f)


@_cached
def Blackman(L: int) -> np.ndarray:
    """window.go:138-152."""
    return _sym(L, lambda n, N: 0.42 + (-0.5 * math.cos(2 * math.pi * float(n) / float(N)))
                + 0.08 * math.cos(4 * math.pi * float(n) / float(N)))
