#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run HERE (the build container), never on the GPU box: step 1 reads the
reference's test tables from /root/reference as data.

1. reference_vectors.json — the known-answer tables of the reference's own
   tests, transcribed mechanically (numbers only) from:
     fft/fft_test.go:38-141    fftTests      (FFTReal + IFFT round trip)
     fft/fft_test.go:148-162   fft2Tests     (FFT2Real + IFFT2 round trip)
     fft/fft_test.go:170-181   fftnTests     (FFTN; "next" row, kept as data)
     fft/fft_test.go:189-195   reverseBitsTests
     fft/fft_test.go:306-319   ExampleFFTReal output (magnitude/phase, 0.1)
     spectral/pwelch_test.go:31-46   pwelchTests
     spectral/spectral_test.go:31-56 segmentTests
     window/window_test.go:34-59     windowTests
     wav/wav_test.go:62-95           wavTests      (header fields per file)
     dsputils/dsputils_test.go:29-39 dsputilsSegmentTests
   and wav/small.wav (copied) + the first 64 KiB of wav/float.wav's data
   chunk (header intact) into tests/golden/wav/ — the data files the
   reference's wav test reads.
2. golden_fft.npz / golden_pwelch.npz — full-precision vectors (seeded inputs,
   outputs of the C restatement in oracle/, cross-checked here against numpy's
   pocketfft and scipy.signal.welch before they are written).
"""
from __future__ import annotations

import json
import math
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402


def _block(path: str, start: str) -> str:
    src = open(os.path.join(REF, path)).read()
    i = src.index(start)
    i = src.index("{", i + len(start) - 1)
    depth = 0
    for k in range(i, len(src)):
        if src[k] == "{":
            depth += 1
        elif src[k] == "}":
            depth -= 1
            if depth == 0:
                return src[i:k + 1]
    raise ValueError(start)


def _literal_to_json(text: str):
    t = re.sub(r"//[^\n]*", "", text)
    t = t.replace("&PwelchOptions{}", "null")
    t = re.sub(r"(\[\])+\w+", "", t)
    t = re.sub(r"complex\(([^,()]+),\s*([^()]+)\)", r"[\1, \2]", t)
    t = t.replace("sqrt2_2", repr(math.sqrt(2) / 2))
    t = re.sub(r"(?<![\w.])\.(\d)", r"0.\1", t)
    t = t.replace("{", "[").replace("}", "]")
    t = re.sub(r",\s*]", "]", t)
    return json.loads(t)


def reference_vectors() -> dict:
    out = {}
    out["fftTests"] = [
        {"in": e[0], "out": e[1]}
        for e in _literal_to_json(_block("fft/fft_test.go", "var fftTests = []fftTest{"))]
    out["fft2Tests"] = [
        {"in": e[0], "out": e[1]}
        for e in _literal_to_json(_block("fft/fft_test.go", "var fft2Tests = []fft2Test{"))]
    out["fftnTests"] = [
        {"in": e[0], "dim": e[1], "out": e[2]}
        for e in _literal_to_json(_block("fft/fft_test.go", "var fftnTests = []fftnTest{"))]
    out["reverseBitsTests"] = [
        {"in": e[0], "sz": e[1], "out": e[2]}
        for e in _literal_to_json(
            _block("fft/fft_test.go", "var reverseBitsTests = []reverseBitsTest{"))]
    src = open(os.path.join(REF, "fft/fft_test.go")).read()
    ex = re.findall(r"// X\((\d)\) = ([\d.\-]+) ∠ ([\d.\-]+)°", src)
    out["exampleFFTReal"] = [{"k": int(k), "mag": float(m), "deg": float(d)} for k, m, d in ex]
    out["pwelchTests"] = [
        {"fs": e[0], "x": e[2], "p": e[3], "freqs": e[4]}
        for e in _literal_to_json(
            _block("spectral/pwelch_test.go", "var pwelchTests = []pwelchTest{"))]
    out["segmentTests"] = {
        "x": [1, 2, 3, 4, 5, 6, 7, 8, 9, 10],  # spectral/spectral_test.go:59
        "cases": [{"size": e[0], "noverlap": e[1], "out": e[2]}
                  for e in _literal_to_json(
                      _block("spectral/spectral_test.go", "var segmentTests = []segmentTest{"))],
    }
    out["windowTests"] = [
        {"L": e[0], "hamming": e[1], "hann": e[2], "bartlett": e[3], "flattop": e[4],
         "blackman": e[5]}
        for e in _literal_to_json(_block("window/window_test.go", "var windowTests = []windowTest{"))]
    out["wavTests"] = wav_tests()
    out["dsputilsSegmentTests"] = [
        {"segs": e[0], "noverlap": e[1], "slices": e[2]}
        for e in _literal_to_json(
            _block("dsputils/dsputils_test.go", "var segmentTests = []segmentTest{"))]
    return out


def wav_tests() -> dict:
    src = open(os.path.join(REF, "wav/wav_test.go")).read()
    res = {}
    for name in ("small.wav", "float.wav"):
        blk = _block("wav/wav_test.go", f'"{name}": {{')
        fields = {}
        for key, expr in re.findall(r"(\w+):\s*([0-9][0-9 /]*)[,\n]", blk):
            if not re.fullmatch(r"[0-9 /]+", expr):
                continue
            parts = [int(v) for v in expr.split("/")]
            v = parts[0]
            for d in parts[1:]:
                v //= d
            fields[key] = v
        res[name] = fields
    assert "checkHeader" in src  # the file also holds header tests (not data)
    return res


def wav_fixtures() -> None:
    import shutil
    dst = os.path.join(HERE, "wav")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(REF, "wav/small.wav"), os.path.join(dst, "small.wav"))
    b = open(os.path.join(REF, "wav/float.wav"), "rb").read()
    assert b[36:40] == b"data"  # RIFF(12) + fmt chunk(8 + 16) + data header(8) = 44
    open(os.path.join(dst, "float_head.wav"), "wb").write(b[:44 + 65536])


def _nrel(a, b) -> float:
    a = np.asarray(a)
    b = np.asarray(b)
    d = np.linalg.norm((a - b).ravel())
    n = np.linalg.norm(b.ravel())
    return float(d / n) if n else float(d)


def full_precision() -> None:
    seed = 0x5EED
    fft_sizes = [2, 3, 4, 5, 6, 7, 8, 12, 16, 17, 31, 32, 64, 100, 128, 256, 1000, 1024,
                 3000, 4096]
    arrays = {}
    for n in fft_sizes:
        x = oracle.fill_uniform(2 * n, seed, n).view(np.complex128)
        y = oracle.fft(x)
        yi = oracle.ifft(x)
        e = _nrel(y, np.fft.fft(x))
        ei = _nrel(yi, np.fft.ifft(x))
        assert e < 1e-12 and ei < 1e-12, (n, e, ei)
        arrays[f"fft_in_{n}"] = x
        arrays[f"fft_out_{n}"] = y
        arrays[f"ifft_out_{n}"] = yi
    # FFT2 cases (col pass then row pass), incl. Bluestein axes
    for r, c in [(2, 3), (3, 5), (4, 8), (16, 16), (6, 10), (64, 32)]:
        x = oracle.fill_uniform(2 * r * c, seed, 1000 * r + c).view(np.complex128).reshape(r, c)
        y = oracle.fft2(x)
        yi = oracle.fft2(x, inverse=True)
        assert _nrel(y, np.fft.fft2(x)) < 1e-12
        assert _nrel(yi, np.fft.ifft2(x)) < 1e-12
        arrays[f"fft2_in_{r}x{c}"] = x
        arrays[f"fft2_out_{r}x{c}"] = y
        arrays[f"ifft2_out_{r}x{c}"] = yi
    np.savez_compressed(os.path.join(HERE, "golden_fft.npz"), **arrays)

    # Pwelch: multi-segment, 50 % overlap, nfft 4096, Fs 1 (and a Pad case)
    import scipy.signal as ss
    parr = {}
    n = 1 << 15
    t = np.arange(n)
    x = np.sin(2 * np.pi * 0.1234 * t) + 0.5 * oracle.fill_uniform(n, seed, 77)
    for name, kw in {"nfft4096_ov2048": dict(nfft=4096, noverlap=2048, fs=1.0),
                     "nfft1024_ov0_fs2": dict(nfft=1024, noverlap=0, fs=2.0),
                     "nfft512_ov256_pad1024": dict(nfft=512, noverlap=256, pad=1024, fs=1.0),
                     "nfft256_hamming_scaleoff": dict(nfft=256, noverlap=128, fs=3.0,
                                                      window_kind="hamming", scale_off=True)
                     }.items():
        p, f = oracle.pwelch(x, **kw)
        if "pad" not in kw and kw.get("window_kind", "hann") == "hann" and not kw.get("scale_off"):
            nfft, nov = kw["nfft"], kw["noverlap"]
            fr, pr = ss.welch(x, fs=kw["fs"], window=ss.get_window("hann", nfft, fftbins=False),
                              nperseg=nfft, noverlap=nov, detrend=False, scaling="density",
                              average="mean", return_onesided=True)
            assert _nrel(p, pr) < 1e-12, (name, _nrel(p, pr))
            assert _nrel(f, fr) < 1e-15
        parr[f"{name}_pxx"] = p
        parr[f"{name}_freqs"] = f
    parr["x"] = x
    parr["hann4096"] = oracle.window("hann", 4096)
    np.savez_compressed(os.path.join(HERE, "golden_pwelch.npz"), **parr)


def main():
    vec = reference_vectors()
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(vec, f, indent=1)
    full_precision()
    wav_fixtures()
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
