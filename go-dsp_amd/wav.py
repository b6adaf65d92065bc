"""Host mirror of go-dsp's `wav` package (wav/wav.go): the WAV reader that
feeds spectral.Pwelch.

Header parsing is byte-level host work (a few dozen bytes), exactly as
wav.New does it (wav.go:59-107). The sample conversion of ReadFloats
(wav.go:135-161) runs on the GPU through gdsp_wav_read_floats; the device
feeder `device_floats` decodes a data chunk straight into an HBM-resident
float64 Pwelch input (gdsp_wav_read_floats_device), so a long recording
never round-trips through host float conversion.

Go returns `error` values here (not panics); the mirror raises WavError
with the reference's message ("wav: missing RIFF", ..., and io's "EOF" /
"unexpected EOF" for short reads).
"""
from __future__ import annotations

import ctypes
import struct
from dataclasses import dataclass

import numpy as np

from . import _lib, spectral
from ._lib import check, lib

wavFormatPCM = 1
wavFormatIEEEFloat = 3


class WavError(Exception):
    """An error value the reference returns (message = Go's err.Error())."""


@dataclass
class Header:
    """wav.Header — the fmt chunk (wav.go:37-45)."""
    AudioFormat: int = 0
    NumChannels: int = 0
    SampleRate: int = 0
    ByteRate: int = 0
    BlockAlign: int = 0
    BitsPerSample: int = 0


def _read_full(r, n: int) -> bytes:
    """io.ReadFull: "EOF" if nothing was read, "unexpected EOF" if short."""
    b = r.read(n)
    if len(b) == 0 and n > 0:
        raise WavError("EOF")
    if len(b) < n:
        raise WavError("unexpected EOF")
    return b


class _LimitReader:
    """io.LimitReader over the data chunk (wav.go:103)."""

    def __init__(self, r, n: int):
        self.r, self.n = r, n

    def read(self, k: int) -> bytes:
        k = min(k, self.n)
        if k <= 0:
            return b""
        b = self.r.read(k)
        self.n -= len(b)
        return b


@dataclass
class Wav(Header):
    """wav.Wav (wav.go:48-56). Duration is a Go time.Duration (int64 ns)."""
    Samples: int = 0
    Duration: int = 0
    _r: object = None

    def _sample_type(self):
        if self.AudioFormat == wavFormatPCM:
            if self.BitsPerSample == 8:
                return np.uint8
            if self.BitsPerSample == 16:
                return np.int16
            raise WavError(f"wav: unknown bits per sample: {self.BitsPerSample}")
        if self.AudioFormat == wavFormatIEEEFloat:
            return np.float32
        raise WavError("wav: unknown audio format")

    def _read_raw(self, n: int):
        typ = np.dtype(self._sample_type()).newbyteorder("<")
        # binary.Read: io.ReadFull of the whole slice
        return _read_full(self._r, n * typ.itemsize), typ

    def ReadSamples(self, n: int) -> np.ndarray:
        """wav.go:110-131: n samples as uint8, int16 or float32."""
        raw, typ = self._read_raw(n)
        return np.frombuffer(raw, dtype=typ).astype(typ.newbyteorder("="))

    def ReadFloats(self, n: int) -> np.ndarray:
        """wav.go:135-161: n samples converted to float32 (on the GPU)."""
        raw, _ = self._read_raw(n)
        return read_floats(raw, n, self.AudioFormat, self.BitsPerSample)


def New(r) -> Wav:
    """wav.New — wav.go:59-107: reads the RIFF/WAVE header and the fmt chunk,
    skips other chunks, and stops at the data chunk. r: a binary file-like
    object (read(n))."""
    w = Wav()
    header = _read_full(r, 12)
    if header[0:4] != b"RIFF":
        raise WavError("wav: missing RIFF")
    if header[8:12] != b"WAVE":
        raise WavError("wav: missing WAVE")
    has_fmt = False
    while True:
        ch = _read_full(r, 8)
        sz = struct.unpack("<I", ch[4:8])[0]
        typ = ch[:4]
        if typ == b"fmt ":
            if sz < 16:
                raise WavError("wav: bad fmt size")
            f = _read_full(r, sz)
            (w.AudioFormat, w.NumChannels, w.SampleRate, w.ByteRate, w.BlockAlign,
             w.BitsPerSample) = struct.unpack("<HHIIHH", f[:16])
            if w.AudioFormat not in (wavFormatPCM, wavFormatIEEEFloat):
                raise WavError(f"wav: unknown audio format: {w.AudioFormat:02x}")
            has_fmt = True
        elif typ == b"data":
            if not has_fmt:
                raise WavError("wav: unexpected fmt chunk")
            if w.BitsPerSample == 0:
                raise WavError("runtime error: integer divide by zero")
            w.Samples = int(sz) // int(w.BitsPerSample) * 8
            if w.SampleRate == 0 or w.NumChannels == 0:
                raise WavError("runtime error: integer divide by zero")
            w.Duration = _go_div(_go_div(w.Samples * 1_000_000_000, w.SampleRate), w.NumChannels)
            w._r = _LimitReader(r, int(sz))
            return w
        else:
            r.read(sz)  # io.CopyN(ioutil.Discard, r, sz); its error is ignored


def _go_div(a: int, b: int) -> int:
    """Go integer division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _format_ok(audio_format: int, bits: int):
    if audio_format == wavFormatPCM and bits not in (8, 16):
        raise WavError(f"wav: unknown bits per sample: {bits}")
    if audio_format not in (wavFormatPCM, wavFormatIEEEFloat):
        raise WavError("wav: unknown audio format")


def read_floats(raw, count: int, audio_format: int, bits: int, f64: bool = False) -> np.ndarray:
    """ReadFloats's conversion of `count` little-endian samples in `raw`
    (bytes-like) on the GPU: float32, or float64 (the float32 values widened,
    a Pwelch input) with f64=True."""
    _format_ok(audio_format, bits)
    buf = np.frombuffer(bytes(raw), dtype=np.uint8)
    out = np.empty(count, np.float64 if f64 else np.float32)
    if count:
        check(lib().gdsp_wav_read_floats(buf.ctypes.data_as(_lib._P), count, audio_format, bits,
                                         out.ctypes.data_as(_lib._P), int(f64)),
              "wav.ReadFloats")
    return out


def device_floats(raw_dev, count: int, audio_format: int, bits: int, out=None, stream=None):
    """The GPU feeder: decode `count` samples from a uint8 CUDA tensor holding
    a data chunk into a float64 CUDA tensor (gdsp_wav_read_floats_device),
    ordered on `stream` — the HBM-resident input of device Pwelch."""
    import torch

    from . import device
    _format_ok(audio_format, bits)
    assert raw_dev.is_cuda and raw_dev.dtype == torch.uint8 and raw_dev.is_contiguous()
    if out is None:
        out = torch.empty(count, dtype=torch.float64, device=raw_dev.device)
    assert out.dtype == torch.float64 and out.numel() >= count
    with torch.cuda.device(raw_dev.device):
        check(lib().gdsp_wav_read_floats_device(
            ctypes.c_void_p(raw_dev.data_ptr()), count, audio_format, bits,
            ctypes.c_void_p(out.data_ptr()), 1, device._stream_ptr(stream, raw_dev.device)),
            "wav_read_floats_device")
    return out


def Pwelch(w: Wav, n: int, o, Fs: float = 0.0):
    """The feeder end to end: the next n samples of w, decoded on the GPU
    into float64 and run through the device Pwelch (no host float pass);
    Fs defaults to w.SampleRate. Equals spectral.Pwelch(float64(
    w.ReadFloats(n)), Fs, o) — the reference's pipeline (pwelch.go:74)."""
    import torch

    from . import distributed
    nfft, pad, nov, _, _ = spectral.resolve_options(o)
    raw, _ = w._read_raw(n)
    if n == 0:  # pwelch.go:75-77
        return np.zeros(0), np.zeros(0)
    fs = float(Fs or w.SampleRate)
    dev = torch.device("cuda", torch.cuda.current_device())
    rd = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    x = device_floats(rd, n, w.AudioFormat, w.BitsPerSample)
    if n < nfft:  # pwelch.go:97-99: zero-padded to nfft
        x = torch.cat([x, torch.zeros(nfft - n, dtype=torch.float64, device=dev)])
    sh = distributed.plan_pwelch(n, 1, 0, nfft, pad, nov)
    return distributed.pwelch(x, fs, o, sh)
