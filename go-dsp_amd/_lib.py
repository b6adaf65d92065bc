"""ctypes binding of libgdspfft (include/gdsp_fft.h).

The shared library is built in-tree by `make -C go-dsp_amd/csrc` (or
__graft_entry__.build()). Loading it does not touch the GPU; every compute
entry point runs on the GPU and returns GDSP_ERR_NO_DEVICE without one — there
is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# GDSP_LIB: an alternate build of the same library (A/B builds in experiments)
LIB_PATH = os.environ.get("GDSP_LIB") or os.path.join(_HERE, "lib", "libgdspfft.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gdsp_fft.h")
# queries only the development build (go-dsp_amd/lib_dev) exports
DEV_HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gdsp_fft_dev.h")

GDSP_OK = 0
GDSP_ERR_INVALID = 1
GDSP_ERR_UNEQUAL = 2
GDSP_ERR_EMPTY = 3
GDSP_ERR_RAGGED = 4
GDSP_ERR_DIVIDE_BY_ZERO = 5
GDSP_ERR_NO_DEVICE = 6
GDSP_ERR_HIP = 7
GDSP_ERR_NOMEM = 8
GDSP_ERR_UNSUPPORTED = 9

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_D = ctypes.c_double
_U64 = ctypes.c_uint64

# name -> (restype, argtypes); must cover every function in include/gdsp_fft.h
SIGNATURES = {
    "gdsp_status_string": (ctypes.c_char_p, [_I]),
    "gdsp_last_error": (ctypes.c_char_p, []),
    "gdsp_version": (ctypes.c_char_p, []),
    "gdsp_jit_stats": (_I, [ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                            ctypes.c_char_p, _I64]),
    "gdsp_device_count": (_I, []),
    "gdsp_fft": (_I, [_P, _P, _I64]),
    "gdsp_ifft": (_I, [_P, _P, _I64]),
    "gdsp_fft_real": (_I, [_P, _P, _I64]),
    "gdsp_ifft_real": (_I, [_P, _P, _I64]),
    "gdsp_convolve": (_I, [_P, _P, _P, _I64]),
    "gdsp_fft_batch": (_I, [_P, _P, _I64, _I64, _I]),
    "gdsp_fft_real_batch": (_I, [_P, _P, _I64, _I64]),
    "gdsp_fft2": (_I, [_P, _P, _I64, _I64, _I]),
    "gdsp_fft2_real": (_I, [_P, _P, _I64, _I64, _I]),
    "gdsp_ensure_plan": (_I, [_I64]),
    "gdsp_fftn": (_I, [_P, _P, _P, _I, _I]),
    "gdsp_fft_axis_device": (_I, [_P, _P, _P, _I, _I, _I, _P]),
    "gdsp_fftn_device": (_I, [_P, _P, _P, _I, _I, _P]),
    "gdsp_set_worker_pool_size": (None, [_I]),
    "gdsp_worker_pool_size": (_I, []),
    "gdsp_segment_count": (_I, [_I64, _I64, _I64, ctypes.POINTER(_I64)]),
    "gdsp_pwelch": (_I, [_P, _I64, _D, _I64, _I64, _I64, _P, _P, _I, _P, _P,
                         ctypes.POINTER(_I64)]),
    "gdsp_window_hann": (_I, [_I64, _P]),
    "gdsp_plan_create": (_I, [_I64, ctypes.POINTER(_P)]),
    "gdsp_plan_create_chirpz": (_I, [_I64, ctypes.POINTER(_P)]),
    "gdsp_plan_destroy": (_I, [_P]),
    "gdsp_plan_kind": (_I, [_P]),
    "gdsp_plan_parts": (_I, [_P]),
    "gdsp_plan_radices": (_I, [_P, ctypes.POINTER(_I), _I]),
    "gdsp_plan_info": (_I, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                            ctypes.POINTER(_I64), ctypes.POINTER(_I)]),
    "gdsp_fft_batch_device": (_I, [_P, _P, _P, _I64, _I, _P]),
    "gdsp_fft_real_batch_device": (_I, [_P, _P, _P, _I64, _I, _P]),
    "gdsp_fft2_device": (_I, [_P, _P, _I64, _I64, _I, _P, _P]),
    "gdsp_pwelch_accumulate_device": (_I, [_P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _P, _P]),
    "gdsp_pwelch_finalize": (_I, [_P, _I64, _I64, _I64, _I64, _P, _D, _I, _P, _P]),
    "gdsp_wav_read_floats": (_I, [_P, _I64, _I, _I, _P, _I]),
    "gdsp_wav_read_floats_device": (_I, [_P, _I64, _I, _I, _P, _I, _P]),
    "gdsp_fill_uniform_device": (_I, [_P, _I64, _U64, _U64, _P]),
    "gdsp_set_devices": (_I, [ctypes.POINTER(_I), _I]),
    "gdsp_get_devices": (_I, [ctypes.POINTER(_I), _I]),
    "gdsp_set_algorithm": (_I, [ctypes.c_uint]),
    "gdsp_get_algorithm": (ctypes.c_uint, []),
    "gdsp_multi_stats": (_I, [ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                              ctypes.POINTER(_I64)]),
    "gdsp_fft_batch_multi": (_I, [_P, _P, _I64, _I64, _I, ctypes.POINTER(_I), _I]),
    "gdsp_pwelch_multi": (_I, [_P, _I64, _D, _I64, _I64, _I64, _P, _P, _I, _P, _P,
                               ctypes.POINTER(_I64), ctypes.POINTER(_I), _I]),
    "gdsp_batch_shard": (_I, [_I64, _I, _I, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "gdsp_pwelch_shard": (_I, [_I64, _I64, _I64, _I, _I, ctypes.POINTER(_I64),
                               ctypes.POINTER(_I64), ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
}

# include/gdsp_fft_dev.h: bound only when the loaded library is the
# development build (the product library does not export them)
DEV_SIGNATURES = {
    "gdsp_dev_chirpz_wave_q": (_I, [_I64]),
    "gdsp_dev_fft_batch_chirpz_wave": (_I, [_I64, _P, _P, _I64, _I, _P]),
    "gdsp_dev_fft_batch_chirpz_shfl": (_I, [_I64, _P, _P, _I64, _I, _P]),
    "gdsp_dev_pwelch4096_shfl_accumulate": (_I, [_P, _I64, _I64, _I64, _P, _P, _P]),
    "gdsp_dev_pwelch4096_row3_accumulate": (_I, [_P, _I64, _I64, _I64, _P, _P, _P]),
}

_lib = None


class GDSPError(RuntimeError):
    """A libgdspfft status other than GDSP_OK."""

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class Panic(GDSPError):
    """Raised where the Go reference panics (same message)."""


_PANIC_STATUSES = {GDSP_ERR_UNEQUAL, GDSP_ERR_EMPTY, GDSP_ERR_RAGGED, GDSP_ERR_DIVIDE_BY_ZERO}


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Every function name declared in include/gdsp_fft.h (or another header)."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gdsp_[a-z0-9_]+)\s*\(", src)))


def _preload_torch_hip() -> None:
    """torch ships its own libamdhip64.so (same SONAME, libamdhip64.so.7). If
    libgdspfft.so were loaded first, /opt/rocm's runtime would be mapped and
    torch would then load a second HIP runtime into the process and fail to
    initialise. Loading torch first makes libgdspfft bind to the one runtime
    torch uses, so device pointers and streams are shared. Skipped when torch
    is absent (plain C-ABI users) or GDSP_NO_TORCH_PRELOAD is set."""
    if os.environ.get("GDSP_NO_TORCH_PRELOAD"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libgdspfft.so not built ({LIB_PATH}); run __graft_entry__.build() "
                "or make -C go-dsp_amd/csrc")
        _preload_torch_hip()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        for name, (res, args) in DEV_SIGNATURES.items():
            if hasattr(L, name):
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
        _lib = L
    return _lib


def check(status: int, what: str = "") -> None:
    if status == GDSP_OK:
        return
    L = lib()
    msg = L.gdsp_status_string(status).decode()
    detail = L.gdsp_last_error().decode()
    if status in _PANIC_STATUSES:
        raise Panic(status, msg)
    raise GDSPError(status, f"{what}: {msg} ({detail})")


def is_dev_build() -> bool:
    """True when the loaded library is the development build."""
    return hasattr(lib(), "gdsp_dev_chirpz_wave_q")


def device_count() -> int:
    return int(lib().gdsp_device_count())


def jit_stats() -> dict:
    """gdsp_jit_stats: runtime-compiled modules built / loaded from the cache /
    failed since process start, and the last failure."""
    b, c, f = _I64(0), _I64(0), _I64(0)
    msg = ctypes.create_string_buffer(4096)
    lib().gdsp_jit_stats(b, c, f, msg, len(msg))
    return {"built": b.value, "cached": c.value, "failed": f.value,
            "last_failure": msg.value.decode(errors="replace")}
