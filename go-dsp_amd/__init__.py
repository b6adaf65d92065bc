"""go-dsp_amd — MI355X (gfx950) engine for the go-dsp FFT / Pwelch hot path.

Host mirror of the reference's Go API (packages fft, spectral, window,
dsputils, wav) over the C ABI of libgdspfft (include/gdsp_fft.h). The directory
name is not a Python identifier; import it with
``importlib.import_module("go-dsp_amd")``.
"""
from . import _lib, dsputils, fft, spectral, wav, window  # noqa: F401
from ._lib import GDSPError, Panic, device_count  # noqa: F401

__all__ = ["fft", "spectral", "window", "dsputils", "wav", "GDSPError", "Panic",
           "device_count"]
