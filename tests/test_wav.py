"""wav package (the wav -> Pwelch feeder).

CPU: wav.New on the reference's own data files (tests/golden/wav/: small.wav
as shipped, float.wav's header plus the first 64 KiB of its data chunk)
against wav_test.go's header table (wav/wav_test.go:62-95), the reference's
error paths, and the oracle's ReadFloats restatement against numpy float32
arithmetic. GPU: ReadFloats / the device feeder bit-exact against the oracle
(integer-to-float conversion: bit-exact is the bar), and wav.Pwelch against
spectral.Pwelch / the oracle on the same samples (1e-9)."""
import io
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, nrel

WAVDIR = os.path.join(GOLDEN, "wav")
FILES = {"small.wav": "small.wav", "float.wav": "float_head.wav"}


def _open(name):
    return open(os.path.join(WAVDIR, FILES[name]), "rb")


def _wav_bytes(fmt, bits, data: bytes, rate=8000, ch=1, extra=b""):
    blk = ch * max(bits // 8, 1)
    fmt_chunk = struct.pack("<HHIIHH", fmt, ch, rate, rate * blk, blk, bits)
    body = b"WAVE" + extra + b"fmt " + struct.pack("<I", 16) + fmt_chunk + b"data" + \
        struct.pack("<I", len(data)) + data
    return b"RIFF" + struct.pack("<I", len(body)) + body


def test_TestWav_headers(gdsp, refvec):
    for name, want in refvec["wavTests"].items():
        with _open(name) as f:
            w = gdsp.wav.New(f)
        got = {k: getattr(w, k) for k in want}
        assert got == want, name


def test_wav_errors(gdsp):
    W = gdsp.wav
    with pytest.raises(W.WavError, match="missing RIFF"):
        W.New(io.BytesIO(b"RIFX" + b"\0" * 40))
    with pytest.raises(W.WavError, match="missing WAVE"):
        W.New(io.BytesIO(b"RIFF" + b"\0" * 40))
    with pytest.raises(W.WavError, match="^EOF$"):
        W.New(io.BytesIO(b""))
    with pytest.raises(W.WavError, match="unexpected EOF"):
        W.New(io.BytesIO(b"RIFF\0\0"))
    bad_fmt = b"RIFF\0\0\0\0WAVEfmt " + struct.pack("<I", 8) + b"\0" * 8
    with pytest.raises(W.WavError, match="bad fmt size"):
        W.New(io.BytesIO(bad_fmt))
    with pytest.raises(W.WavError, match="unknown audio format: 02"):
        W.New(io.BytesIO(_wav_bytes(2, 16, b"\0" * 8)))
    data_first = b"RIFF\0\0\0\0WAVEdata" + struct.pack("<I", 4) + b"\0" * 4
    with pytest.raises(W.WavError, match="unexpected fmt chunk"):
        W.New(io.BytesIO(data_first))
    # other chunks (JUNK, bext, ...) are skipped
    data = np.arange(1, 17, dtype="<i2").tobytes()
    w = W.New(io.BytesIO(_wav_bytes(1, 16, data, extra=b"JUNK" + struct.pack("<I", 4) + b"abcd")))
    assert w.Samples == 16 and list(w.ReadSamples(2)) == [1, 2]
    # the reference's Samples = size / BitsPerSample * 8 truncates first
    # (wav.go:100): a 4-byte 16-bit chunk reports 0 samples
    assert W.New(io.BytesIO(_wav_bytes(1, 16, b"\1\0\2\0"))).Samples == 0
    # reads past the data chunk: io.ReadFull errors
    w = W.New(io.BytesIO(_wav_bytes(1, 16, b"\1\0\2\0")))
    with pytest.raises(W.WavError, match="unexpected EOF"):
        w.ReadSamples(3)
    w = W.New(io.BytesIO(_wav_bytes(1, 24, b"\0" * 6)))
    with pytest.raises(W.WavError, match="unknown bits per sample: 24"):
        w.ReadSamples(1)


def test_read_samples_small_wav(gdsp):
    with _open("small.wav") as f:
        w = gdsp.wav.New(f)
        s = w.ReadSamples(1000)
    raw = open(os.path.join(WAVDIR, "small.wav"), "rb").read()[44:44 + 2000]
    assert s.dtype == np.int16 and np.array_equal(s, np.frombuffer(raw, "<i2"))


def _np_floats(raw, fmt, bits):
    """ReadFloats in numpy float32 arithmetic (IEEE, correctly rounded)."""
    if fmt == 3:
        return np.frombuffer(raw, "<f4").astype(np.float32)
    if bits == 8:
        return np.frombuffer(raw, np.uint8).astype(np.float32) / np.float32(255)
    v = np.frombuffer(raw, "<i2").astype(np.float32)
    return (v - np.float32(-32768)) / np.float32(65535)


def test_oracle_wav_floats(oracle):
    rng = np.random.default_rng(3)
    for fmt, bits, nbytes in [(1, 8, 1), (1, 16, 2), (3, 32, 4)]:
        raw = rng.integers(0, 256, 4000 * nbytes, dtype=np.uint8).tobytes()
        if fmt == 3:  # finite floats only
            raw = rng.standard_normal(4000).astype("<f4").tobytes()
        got = oracle.wav_floats(raw, 4000, fmt, bits)
        assert np.array_equal(got.view(np.uint32), _np_floats(raw, fmt, bits).view(np.uint32))
    # every int16 value once
    raw = np.arange(-32768, 32768, dtype="<i2").tobytes()
    assert np.array_equal(oracle.wav_floats(raw, 65536, 1, 16).view(np.uint32),
                          _np_floats(raw, 1, 16).view(np.uint32))


def test_wav_c_abi_without_gpu(gdsp):
    if gdsp.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(gdsp.GDSPError) as e:
        gdsp.wav.read_floats(b"\0\0\1\0", 2, 1, 16)
    assert e.value.status == gdsp._lib.GDSP_ERR_NO_DEVICE
    with pytest.raises(gdsp.wav.WavError, match="unknown bits per sample"):
        gdsp.wav.read_floats(b"\0" * 3, 1, 1, 24)


# ---- GPU -------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["small.wav", "float.wav"])
def test_read_floats_gpu_bit_exact(gdsp, oracle, name):
    with _open(name) as f:
        w = gdsp.wav.New(f)
        n = min(w.Samples, 65536 // (w.BitsPerSample // 8))
        got = w.ReadFloats(n)
    raw = open(os.path.join(WAVDIR, FILES[name]), "rb").read()[44:44 + n * w.BitsPerSample // 8]
    want = oracle.wav_floats(raw, n, w.AudioFormat, w.BitsPerSample)
    assert got.dtype == np.float32 and np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_device_feeder_formats(gdsp, oracle):
    import torch
    rng = np.random.default_rng(11)
    for fmt, bits, nb in [(1, 8, 1), (1, 16, 2), (3, 32, 4)]:
        count = 100003
        raw = rng.integers(0, 256, count * nb, dtype=np.uint8).tobytes()
        if fmt == 3:
            raw = rng.standard_normal(count).astype("<f4").tobytes()
        want = oracle.wav_floats(raw, count, fmt, bits)
        # aligned: the 16-B-per-lane kernel plus the byte-load tail (count is
        # not a multiple of the samples per load); odd offset: the data chunk
        # of a file uploaded whole is not aligned, byte loads throughout
        for off in (0, 1):
            dev = torch.frombuffer(bytearray(b"x" * off + raw), dtype=torch.uint8).cuda()[off:]
            got = gdsp.wav.device_floats(dev, count, fmt, bits).cpu().numpy()
            assert np.array_equal(got, want.astype(np.float64)), (fmt, off)
        host32 = gdsp.wav.read_floats(raw, count, fmt, bits)
        assert np.array_equal(host32.view(np.uint32), want.view(np.uint32))
        host64 = gdsp.wav.read_floats(raw, count, fmt, bits, f64=True)
        assert np.array_equal(host64, want.astype(np.float64))


@pytest.mark.gpu
@pytest.mark.parametrize("name,nfft,nov", [("small.wav", 1024, 512), ("small.wav", 256, 0),
                                           ("float.wav", 512, 256)])
def test_wav_pwelch_feeder(gdsp, oracle, name, nfft, nov):
    S = gdsp.spectral
    with _open(name) as f:
        w = gdsp.wav.New(f)
        n = min(w.Samples, 65536 // (w.BitsPerSample // 8))
        p, fr = gdsp.wav.Pwelch(w, n, S.PwelchOptions(NFFT=nfft, Noverlap=nov))
    raw = open(os.path.join(WAVDIR, FILES[name]), "rb").read()[44:44 + n * w.BitsPerSample // 8]
    x = oracle.wav_floats(raw, n, w.AudioFormat, w.BitsPerSample).astype(np.float64)
    pr, frr = oracle.pwelch(x, float(w.SampleRate), nfft=nfft, noverlap=nov)
    assert nrel(p, pr) < 1e-9 and np.array_equal(fr, frr)
    ps, _ = S.Pwelch(x, float(w.SampleRate), S.PwelchOptions(NFFT=nfft, Noverlap=nov))
    assert nrel(p, ps) < 1e-9
