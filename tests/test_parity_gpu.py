"""GPU parity: the HIP path through the C ABI against the oracle (CPU
restatement of the reference) and the reference's own golden vectors.

Tolerances: the north star's 1e-9 normwise relative for every
complex128 result; the reference's known-answer tables with its own
Float64Equal (1e-8, dsputils/compare.go:94-96) because their constants carry
8-9 digits. Measured errors are ~1e-15 (powers of 2) and ~1e-13 (Bluestein)."""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, cpx, nrel, row_nrel

pytestmark = pytest.mark.gpu

TOL = 1e-9  # north star: within 1e-9 relative for complex128


def f64eq(a, b):
    if abs(a - b) <= 1e-8:
        return True
    return b != 0 and abs(1 - a / b) <= 1e-8


def close_c(a, b):
    return len(a) == len(b) and all(f64eq(x.real, y.real) and f64eq(x.imag, y.imag)
                                    for x, y in zip(a, b))


def close_f(a, b):
    return len(a) == len(b) and all(f64eq(x, y) for x, y in zip(a, b))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gdsp):
    if gdsp.device_count() < 1:
        pytest.fail("gpu test without a visible HIP device")


# ---- reference known answers (fft/fft_test.go, spectral/*_test.go) ----------
def test_TestFFT(gdsp, refvec):
    for case in refvec["fftTests"]:
        out = cpx(case["out"])
        assert close_c(gdsp.fft.FFTReal(case["in"]), out), case
        assert close_c(gdsp.fft.IFFT(out), np.asarray(case["in"], np.complex128)), case


def test_TestFFT2(gdsp, refvec):
    for case in refvec["fft2Tests"]:
        out = [cpx(r) for r in case["out"]]
        y = gdsp.fft.FFT2Real(case["in"])
        assert all(close_c(a, b) for a, b in zip(y, out))
        yi = gdsp.fft.IFFT2(out)
        x = np.asarray(case["in"], np.complex128)
        assert all(close_c(a, b) for a, b in zip(yi, x))


def test_ExampleFFTReal(gdsp, refvec):
    a = [math.sin(2 * math.pi * n / 8.0) + 0.5 * math.sin(2 * math.pi * n / 4.0 + 3 * math.pi / 4)
         for n in range(8)]
    X = gdsp.fft.FFTReal(a)
    for e in refvec["exampleFFTReal"]:
        z = X[e["k"]]
        r, th = abs(z), math.degrees(math.atan2(z.imag, z.real))
        if f64eq(r, 0):
            th = 0
        assert f"{r:.1f}" == f"{e['mag']:.1f}" and f"{th:.1f}" == f"{e['deg']:.1f}"


def test_TestFFTMulti(gdsp, oracle):
    # fft/fft_test.go:251-259 (no assertion in the reference; we check it)
    N = 1 << 8
    a = np.arange(N) / N
    assert nrel(gdsp.fft.FFT(a), oracle.fft(a)) < TOL


def test_TestPwelch(gdsp, refvec):
    for c in refvec["pwelchTests"]:
        p, f = gdsp.spectral.Pwelch(c["x"], c["fs"], gdsp.spectral.PwelchOptions())
        assert close_f(p, c["p"]) and close_f(f, c["freqs"])


# ---- full-precision fixtures and the oracle ----------------------------------
def test_golden_fft(gdsp, golden_fft):
    for key in sorted(golden_fft):
        if not key.startswith("fft_in_"):
            continue
        n = key[len("fft_in_"):]
        x = golden_fft[key]
        assert nrel(gdsp.fft.FFT(x), golden_fft[f"fft_out_{n}"]) < TOL, n
        assert nrel(gdsp.fft.IFFT(x), golden_fft[f"ifft_out_{n}"]) < TOL, n


def test_golden_fft2(gdsp, golden_fft):
    for key in sorted(golden_fft):
        if not key.startswith("fft2_in_"):
            continue
        s = key[len("fft2_in_"):]
        x = golden_fft[key]
        assert nrel(gdsp.fft.FFT2(x), golden_fft[f"fft2_out_{s}"]) < TOL, s
        assert nrel(gdsp.fft.IFFT2(x), golden_fft[f"ifft2_out_{s}"]) < TOL, s


SIZES = [2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 17, 31, 32, 33, 64, 100, 128, 255, 256, 512, 1000,
         1024, 2048, 3000, 4096, 4097, 5000, 8192, 10000, 16384, 32768, 65536, 1 << 17,
         1 << 20, 1 << 22, 1 << 24, 100000]


@pytest.mark.parametrize("n", SIZES)
def test_fft_sizes_vs_oracle(gdsp, oracle, n):
    rng = np.random.default_rng(n)
    batch = 3 if n <= 65536 else 1
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    y = gdsp.fft.FFTBatch(x)
    yi = gdsp.fft.FFTBatch(x, inverse=True)
    ref = oracle.fft_rows(x)
    refi = oracle.ifft_rows(x)
    assert row_nrel(y, ref) < TOL
    assert row_nrel(yi, refi) < TOL
    # single-call API for the first row
    assert nrel(gdsp.fft.FFT(x[0]), ref[0]) < TOL


@pytest.mark.parametrize("log2n,batch", [(17, 1), (17, 16), (17, 17), (18, 3), (19, 4),
                                          (19, 5), (20, 1), (20, 2), (20, 3), (21, 1)])
def test_fourstep_split_by_batch(gdsp, oracle, log2n, batch):
    # exec_fourstep takes rows of 4096 when batch * 2^(log2n-13) <= 256 and of
    # 8192 above: both sides of the boundary, forward / inverse / real input
    n = 1 << log2n
    rng = np.random.default_rng(log2n * 100 + batch)
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL


@pytest.mark.parametrize("log2n,batch", [(15, 1), (15, 6), (16, 1), (16, 3), (17, 2), (18, 1),
                                          (18, 2)])
def test_fourstep_two_pass(gdsp, oracle, log2n, batch):
    # 2^15..2^18: column pass + rows with the transpose fused into their store
    # (rowfft_t_kernel), forward / inverse / real input, and in place on the
    # device
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    n = 1 << log2n
    rng = np.random.default_rng(log2n * 10 + batch)
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    ref = oracle.fft_rows(x)
    assert row_nrel(gdsp.fft.FFTBatch(x), ref) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    xt = torch.from_numpy(x).cuda()
    D.fft_batch(xt, xt)
    torch.cuda.synchronize()
    assert row_nrel(xt.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("n,batch", [(10000, 3), (12000, 2), (48000, 3), (196608, 1), (160000, 2)])
def test_mixed_fourstep_two_pass(gdsp, oracle, n, batch):
    # n = L * 2^k: the column pass, then rows of 2^k whose store carries the
    # transpose (rowfft_t_kernel with R = L, not a power of 2; the last
    # workgroup's rows run past batch * L), forward / inverse / real / in place
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(n).kind == 6
    rng = np.random.default_rng(n + batch)
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    ref = oracle.fft_rows(x)
    assert row_nrel(gdsp.fft.FFTBatch(x), ref) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    xt = torch.from_numpy(x).cuda()
    D.fft_batch(xt, xt)
    torch.cuda.synchronize()
    assert row_nrel(xt.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("n,batch", [(9000, 5), (44100, 2), (50000, 3), (88200, 1), (100000, 2),
                                     (600000, 1), (1000000, 1)])
def test_mixed_rows_two_pass(gdsp, oracle, n, batch):
    # n = L * C with C <= 1024 smooth (not a power of 2): the column pass, then
    # rows of C by the runtime-compiled rowt_fixed_kernel with the transpose in
    # their store; forward / inverse / real / in place
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(n).kind == 6
    rng = np.random.default_rng(n + 7 * batch)
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    ref = oracle.fft_rows(x)
    assert row_nrel(gdsp.fft.FFTBatch(x), ref) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    xt = torch.from_numpy(x).cuda()
    D.fft_batch(xt, xt)
    torch.cuda.synchronize()
    assert row_nrel(xt.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("n,batch", [(10571, 3), (9889, 2)])
def test_mixed_rows_short_columns(gdsp, oracle, n, batch):
    # lengths whose only two-pass split has columns of <= 25 points: 10571 =
    # 11 x 961 and 9889 = 11 x 899 (the balanced divisors are primes 29 / 31,
    # which are chirp-z lengths, not mixed rows): the single-radix column pass
    # (colradix_kernel) + runtime-compiled rows of C with the transpose in
    # their store (mixrows_build's short-column branch)
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    p = D.plan(n)
    assert p.kind == 6 and p.n1 * p.n2 == n, (p.kind, p.n1, p.n2)
    assert p.n1 <= 25, (p.n1, p.n2)
    rng = np.random.default_rng(n + 3 * batch)
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    ref = oracle.fft_rows(x)
    assert row_nrel(gdsp.fft.FFTBatch(x), ref) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    xt = torch.from_numpy(x).cuda()
    D.fft_batch(xt, xt)
    torch.cuda.synchronize()
    assert row_nrel(xt.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("n", [2, 4, 8, 16, 32, 64, 128, 256])
def test_short_rows_many_blocks(gdsp, oracle, n):
    # short transforms stage whole workgroup chunks through LDS: several
    # blocks and a ragged last one, forward / inverse / real input
    rng = np.random.default_rng(100 + n)
    batch = (1 << 15) // n + 7
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL


@pytest.mark.parametrize("n", [1, 2, 8, 1024, 3000, 4096, 1 << 18])
def test_fft_real(gdsp, oracle, n):
    rng = np.random.default_rng(7 + n)
    x = rng.uniform(-1, 1, (4, n))
    assert row_nrel(gdsp.fft.FFTRealBatch(x), oracle.fft_rows(x.astype(np.complex128))) < TOL
    assert nrel(gdsp.fft.FFTReal(x[0]), oracle.fft_real(x[0])) < TOL
    assert nrel(gdsp.fft.IFFTReal(x[0]), oracle.ifft_real(x[0])) < TOL


@pytest.mark.parametrize("n", [1, 5, 1024, 3000, 4096, 1500, 12289, 1 << 18])
def test_fft_real_batch_device(gdsp, oracle, n):
    """gdsp_fft_real_batch_device: float64 device rows read by the kernels
    themselves (every plan kind: LDS, mixed radix, chirp-z on M = 6144 / 3072,
    output-split chirp-z, four-step), forward and inverse, against the oracle;
    an overlapping output is refused."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(40 + n)
    batch = 3 if n < (1 << 18) else 1
    x = rng.uniform(-1, 1, (batch, n))
    xt = torch.from_numpy(x).cuda()
    for inv in (False, True):
        y = D.fft_real_batch(xt, inverse=inv).cpu().numpy()
        ref = oracle.ifft_rows(x.astype(np.complex128)) if inv else oracle.fft_rows(
            x.astype(np.complex128))
        assert row_nrel(y, ref) < TOL, (n, inv)
    for chirpz in ((True,) if n >= 2 else ()):
        y = D.fft_real_batch(xt, chirpz=chirpz).cpu().numpy()
        assert row_nrel(y, oracle.fft_rows(x.astype(np.complex128))) < TOL, (n, "chirpz")
    if n >= 8:
        buf = torch.empty(2 * batch * n, dtype=torch.complex128, device="cuda")
        src = buf.view(torch.float64)[: batch * n].view(batch, n)
        with pytest.raises(gdsp.GDSPError):
            D.fft_real_batch(src, out=buf[: batch * n].view(batch, n))


def test_batch_4096_vs_oracle(gdsp, oracle):
    # the headline configuration's transform on a 1024-row sample
    x = oracle.fill_uniform(2 * 4096 * 1024, 0x5EED).view(np.complex128).reshape(1024, 4096)
    y = gdsp.fft.FFTBatch(x)
    assert row_nrel(y, oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(y, inverse=True), x) < TOL


def test_batch_3000_vs_oracle(gdsp, oracle):
    x = oracle.fill_uniform(2 * 3000 * 256, 0x5EED, 11).view(np.complex128).reshape(256, 3000)
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL


@pytest.mark.parametrize("n", [2, 5, 16, 1000, 4096, 257, 3001])  # (257, 3001: Rader)
def test_convolve(gdsp, oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    y = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    assert nrel(gdsp.fft.Convolve(x, y), oracle.convolve(x, y)) < TOL


@pytest.mark.parametrize("shape", [(1, 1), (1, 8), (8, 1), (2, 3), (3, 5), (16, 16), (64, 32),
                                   (6, 10), (100, 7), (128, 256), (512, 300), (1024, 1024),
                                   (16, 1000), (2048, 48), (4096, 33), (65536, 8), (32, 5),
                                   # a dimension on the output-split chirp-z (in-place rows)
                                   (3, 8209), (8209, 2),
                                   # prime dimensions on Rader's algorithm (rows; columns
                                   # through the transposes)
                                   (17, 3001), (3001, 16), (37, 41)])
def test_fft2_vs_oracle(gdsp, oracle, shape):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    x = rng.uniform(-1, 1, shape) + 1j * rng.uniform(-1, 1, shape)
    assert nrel(gdsp.fft.FFT2(x), oracle.fft2(x)) < TOL
    assert nrel(gdsp.fft.IFFT2(x), oracle.fft2(x, inverse=True)) < TOL
    xr = rng.uniform(-1, 1, shape)
    assert nrel(gdsp.fft.FFT2Real(xr), oracle.fft2(xr)) < TOL
    assert nrel(gdsp.fft.IFFT2Real(xr), oracle.fft2(xr, inverse=True)) < TOL


# ---- Pwelch ---------------------------------------------------------------------
def test_pwelch_golden(gdsp, golden_pwelch):
    x = golden_pwelch["x"]
    S = gdsp.spectral
    cases = {
        "nfft4096_ov2048": (1.0, S.PwelchOptions(NFFT=4096, Noverlap=2048)),
        "nfft1024_ov0_fs2": (2.0, S.PwelchOptions(NFFT=1024)),
        "nfft512_ov256_pad1024": (1.0, S.PwelchOptions(NFFT=512, Noverlap=256, Pad=1024)),
        "nfft256_hamming_scaleoff": (3.0, S.PwelchOptions(NFFT=256, Noverlap=128,
                                                          Window=gdsp.window.Hamming,
                                                          Scale_off=True)),
    }
    for name, (fs, o) in cases.items():
        p, f = S.Pwelch(x, fs, o)
        assert nrel(p, golden_pwelch[f"{name}_pxx"]) < TOL, name
        assert nrel(f, golden_pwelch[f"{name}_freqs"]) == 0.0, name


WINDOWS = {"hann": "Hann", "hamming": "Hamming", "rectangular": "Rectangular",
           "bartlett": "Bartlett", "flattop": "FlatTop", "blackman": "Blackman"}


@pytest.mark.parametrize("n,nfft,nov,pad,win", [
    (100, 0, 0, 0, "hann"),            # default options, zero-padded single segment
    (5000, 256, 128, 0, "hann"),
    (5001, 256, 100, 0, "hamming"),    # odd segment count
    (10000, 1024, 512, 4096, "blackman"),
    (10000, 1024, 0, 512, "hann"),     # Pad < NFFT quirk (pwelch.go:108 vs :124)
    (7777, 300, 150, 0, "bartlett"),   # non-power-of-2 segment (materialised path)
    (4000, 8, 4, 0, "flattop"),        # tiny segments
    (1 << 16, 16384, 8192, 0, "hann"),
    (4096, 4096, 0, 0, "rectangular"),  # exactly one segment
    # half overlap (the carried-sample kernel): even/odd segment counts, Pad < NFFT
    (40960, 4096, 2048, 0, "hann"),
    (38913, 4096, 2048, 0, "hann"),
    (20000, 64, 32, 0, "blackman"),
    (20000, 32, 16, 16, "hann"),
    (100000, 8192, 4096, 2048, "hamming"),
    (8191, 8192, 4096, 0, "hann"),     # shorter than NFFT: one zero-padded segment
    # smooth non-power-of-2 lengths: the fused mixed-radix Pwelch kernels
    (30000, 1000, 500, 0, "hann"),
    (20001, 3000, 1500, 0, "hann"),
    (12345, 960, 0, 1200, "hamming"),  # Pad > NFFT, both smooth
    (9999, 1500, 700, 0, "blackman"),
    (50000, 4095, 2000, 0, "hann"),    # 13*7*5*3*3: five passes
    (30000, 810, 400, 0, "hann"),      # no compiled specialisation: runtime radices
    (60000, 6000, 3000, 0, "hann"),    # specialisation above 4096 (re/im exchange)
    (20000, 360, 180, 0, "bartlett"),  # three passes, radix 3 in the middle
    (9000, 100, 0, 0, "hann"),         # two passes, many workers per block
    # compiled specialisations (pwelch_fixed_kernel): several workers per block,
    # odd segment counts, no overlap
    (200000, 480, 240, 0, "hann"),
    (100000, 2000, 1000, 0, "hamming"),
    (70001, 1536, 768, 0, "blackman"),
    (50000, 1000, 0, 0, "rectangular"),
    (3001, 12, 5, 0, "bartlett"),      # two tiny passes
    # odd strides (segments 8-byte but not 16-byte aligned), odd segment
    # counts, Pad > NFFT: on 3000's own Pwelch list (15 5 5 8, specspw), on
    # 2000's 10 10 20, and in the radix-25-first LDS-DMA form (3200's 25 8 16,
    # 2275's runtime-compiled 25 13 7)
    (30011, 3000, 1499, 0, "hann"),
    (40000, 2000, 999, 0, "hamming"),
    (25001, 2900, 1000, 3000, "blackman"),
    (50001, 3200, 1599, 0, "hann"),
    (60001, 2275, 1100, 0, "hann"),    # runtime-compiled (hipRTC) list
    # materialised path: a single-radix length, and a Bluestein length
    (5000, 7, 3, 0, "hann"),
    (100000, 5000, 2500, 0, "flattop"),
])
def test_pwelch_vs_oracle(gdsp, oracle, n, nfft, nov, pad, win):
    rng = np.random.default_rng(n + nfft)
    x = rng.standard_normal(n)
    o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov, Pad=pad,
                                    Window=getattr(gdsp.window, WINDOWS[win]))
    p, f = gdsp.spectral.Pwelch(x, 2.5, o)
    pr, fr = oracle.pwelch(x, 2.5, nfft=nfft, pad=pad, noverlap=nov, window_kind=win)
    assert nrel(p, pr) < TOL
    assert nrel(f, fr) == 0.0


def _spec_lengths():
    # every compiled specialisation (go-dsp_amd/csrc/fft_specs*.hip), read from
    # the sources so a changed or added radix list is covered without editing
    # this file
    import math
    import re
    from pathlib import Path
    csrc = Path(__file__).resolve().parent.parent / "go-dsp_amd" / "csrc"
    out = set()
    for f in csrc.glob("fft_specs*.hip"):
        for m in re.finditer(r"Spec<([\d, ]+)>", f.read_text()):
            out.add(math.prod(int(v) for v in m.group(1).split(",")))
    return sorted(out)


@pytest.mark.parametrize("nfft", _spec_lengths())
def test_pwelch_every_specialisation(gdsp, oracle, nfft):
    """The fused Pwelch (pwelch_fixed_kernel) of each compiled radix list at
    half overlap with an odd segment count (a partnerless last pair) and at
    Noverlap 0, against the reference restatement (spectral/pwelch.go:104-122),
    and the list's batched FFT forward / inverse."""
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(nfft).kind == 5, nfft
    rng = np.random.default_rng(nfft)
    for nov, nseg in ((nfft // 2, 7), (0, 4)):
        n = (nseg - 1) * (nfft - nov) + nfft + 3
        x = rng.standard_normal(n)
        o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov)
        p, f = gdsp.spectral.Pwelch(x, 3.0, o)
        pr, fr = oracle.pwelch(x, 3.0, nfft=nfft, noverlap=nov)
        assert nrel(p, pr) < TOL and nrel(f, fr) == 0.0, (nfft, nov)
    xb = rng.uniform(-1, 1, (3, nfft)) + 1j * rng.uniform(-1, 1, (3, nfft))
    assert row_nrel(gdsp.fft.FFTBatch(xb), oracle.fft_rows(xb)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(xb, inverse=True), oracle.ifft_rows(xb)) < TOL


def _wave_cases():
    # pwelch_wave_kernel (F = 64 ... 2048): half overlap with odd and even
    # segment counts (the last group partial: S = 64 / T slots per wave), no
    # overlap, another overlap, and Pad > NFFT (the clamped, masked loop)
    out = []
    for lf in range(6, 12):
        f = 1 << lf
        segs = 3 + 4000 // (f // 64)
        out += [(f, f // 2, 0, segs | 1, "hann"), (f, f // 2, 0, segs & ~1, "hamming"),
                (f, 0, 0, segs + 2, "blackman"), (f, f // 4, 0, segs + 1, "hann"),
                (f - 5, (f - 5) // 2, f, segs | 1, "bartlett")]
    # several groups per worker (more groups than the launch's workers)
    return out + [(256, 128, 0, 32767, "hann"), (1024, 0, 0, 8193, "hann")]


@pytest.mark.parametrize("nfft,nov,pad,segs,win", _wave_cases())
def test_pwelch_wave_kernels_vs_oracle(gdsp, oracle, nfft, nov, pad, segs, win):
    rng = np.random.default_rng(nfft * 7 + nov + segs)
    stride = nfft - nov
    n = (segs - 1) * stride + nfft + int(rng.integers(0, stride))  # tail shorter than a stride
    x = rng.uniform(-1, 1, n)
    o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov, Pad=pad,
                                    Window=getattr(gdsp.window, WINDOWS[win]))
    p, f = gdsp.spectral.Pwelch(x, 1.0, o)
    pr, fr = oracle.pwelch(x, 1.0, nfft=nfft, pad=pad, noverlap=nov, window_kind=win)
    assert nrel(p, pr) < TOL
    assert nrel(f, fr) == 0.0


def _random_pwelch_cases(count=36, seed=20261018):
    # options drawn across every Pwelch kernel family: powers of 2 from 8 to
    # 16384 (wave, row, half and general kernels), smooth NFFTs (compiled and
    # runtime-compiled mixed radix), a prime (materialised path); Noverlap
    # anywhere below NFFT (the half-overlap case on purpose a quarter of the
    # time); Pad 0, below NFFT (the pwelch.go:108 quirk) or above it
    rng = np.random.default_rng(seed)
    nffts = [8, 32, 64, 100, 128, 256, 480, 512, 1000, 1024, 1500, 2000, 2048, 2400, 3000, 4096,
             1031, 8192, 16384]
    out = []
    for _ in range(count):
        nfft = int(rng.choice(nffts))
        nov = nfft // 2 if rng.random() < 0.25 else int(rng.integers(0, nfft))
        r = rng.random()
        pad = 0 if r < 0.5 else (nfft // 2 if r < 0.6 else nfft + int(rng.integers(1, nfft + 1)))
        nseg = int(rng.integers(1, 40))
        n = (nseg - 1) * (nfft - nov) + nfft + int(rng.integers(0, nfft))
        win = str(rng.choice(list(WINDOWS)))
        out.append((n, nfft, nov, pad, win))
    return out


@pytest.mark.parametrize("n,nfft,nov,pad,win", _random_pwelch_cases())
def test_pwelch_random_options_vs_oracle(gdsp, oracle, n, nfft, nov, pad, win):
    rng = np.random.default_rng(n * 31 + nfft)
    x = rng.standard_normal(n)
    o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov, Pad=pad,
                                    Window=getattr(gdsp.window, WINDOWS[win]))
    p, f = gdsp.spectral.Pwelch(x, 3.0, o)
    pr, fr = oracle.pwelch(x, 3.0, nfft=nfft, pad=pad, noverlap=nov, window_kind=win)
    assert nrel(p, pr) < TOL
    assert nrel(f, fr) == 0.0


# A negative Noverlap (spectral/spectral.go:22-43 allows it) puts the segments
# farther apart than NFFT: the LDS-DMA fused kernels (radix-25 first pass:
# 3200 = 25 8 16, 3000 = 25 15 8) must not stage a pair wider than their stage
# (ADVICE r05), and strides beyond 2^22 samples take the 64-bit materialised
# path instead of the fused kernels' 32-bit offsets.
@pytest.mark.parametrize("n,nfft,nov", [
    (200000, 3200, -1), (200000, 3200, -700), (150000, 3000, -5), (150000, 3000, -3000),
    (60000, 256, -100), (60000, 1024, -3), (120000, 2048, -1), (200000, 4096, -10),
    ((1 << 23) + 9000, 256, -((1 << 22) + 100)), ((1 << 23) + 9000, 3200, -((1 << 22) + 1)),
])
def test_pwelch_negative_noverlap(gdsp, oracle, n, nfft, nov):
    rng = np.random.default_rng(n + nfft - nov)
    x = rng.standard_normal(n)
    o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov)
    p, _ = gdsp.spectral.Pwelch(x, 2.0, o)
    pr, _ = oracle.pwelch(x, 2.0, nfft=nfft, noverlap=nov)
    assert p.size == pr.size and nrel(p, pr) < TOL


# ---- edge cases and conventions --------------------------------------------------
def test_edge_cases(gdsp):
    F = gdsp.fft
    assert F.FFT([]).size == 0
    assert F.FFT([3 + 4j])[0] == 3 + 4j
    assert F.IFFT([3 + 4j])[0] == 3 + 4j
    with pytest.raises(gdsp.Panic):
        F.IFFT([])
    with pytest.raises(gdsp.Panic, match="arrays not of equal size"):
        F.Convolve([1, 2], [1, 2, 3])
    with pytest.raises(gdsp.Panic, match="empty input array"):
        F.FFT2([])
    with pytest.raises(gdsp.Panic, match="ragged input array"):
        F.FFT2([[1, 2], [3]])
    p, f = gdsp.spectral.Pwelch([], 0, gdsp.spectral.PwelchOptions())
    assert p.size == 0 and f.size == 0
    with pytest.raises(gdsp.Panic):
        gdsp.spectral.Pwelch([1.0], 1, None)


def test_inputs_not_mutated(gdsp):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(3000) + 1j * rng.standard_normal(3000)
    keep = x.copy()
    gdsp.fft.FFT(x)
    gdsp.fft.IFFT(x)
    assert np.array_equal(x, keep)


def test_plan_kinds(gdsp):
    import torch  # noqa: F401  (device plumbing)
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(1).kind == 0
    assert D.plan(4096).kind == 1
    assert D.plan(1 << 16).kind == 2
    assert D.plan(3000).kind == 5  # 2^3 3 5^3: mixed radix
    assert D.plan(4097).kind in (3, 8)  # 17 * 241: prime-factor Rader where it wins the race
    assert D.plan(2062).kind == 3  # 2 * 1031, 1030 = 2 * 5 * 103: fused Bluestein
    assert D.plan(10000).kind == 6  # 16 x 625: mixed four-step (power-of-2 columns)
    assert D.plan(44100).kind == 6  # 25 x 1764: mixed four-step (single-radix columns)
    assert D.plan(5000).kind == 5  # a compiled specialisation above 4096 (25*25*8)
    assert D.plan(5400).kind == 5  # smooth, no compiled specialisation: hipRTC-compiled one
    # prime, NextPowerOf2(2n-1) = 32768: output-split chirp-z, 2 parts on M = 16384
    assert D.plan(8209).kind == 3 and D.plan(8209).parts == 2 and D.plan(8209).m == 16384
    assert D.plan(16411).kind == 4  # prime beyond the parts' reach: composed Bluestein
    # four-step rows on the output-split chirp-z (power-of-2 / single-radix columns)
    assert (D.plan(64 * 8209).kind, D.plan(64 * 8209).n2) == (6, 8209)
    assert (D.plan(2 * 10007).kind, D.plan(2 * 10007).n2) == (6, 10007)
    assert D.plan(8191 * 64).kind == 6  # power-of-2 columns, chirp-z rows of 8191
    assert (D.plan(3001).kind, D.plan(3001).m) in ((7, 3000), (3, 6144))  # prime: Rader (raced)
    assert D.plan(3067).kind == 3  # prime, 3066 = 2 * 3 * 7 * 73: no radix list, chirp-z
    assert D.plan(3000, chirpz=True).kind == 3
    assert D.plan(10000, chirpz=True).kind == 4
    assert D.plan(4096, chirpz=True).kind == 3  # forced chirp-z on a power of 2


# every prime in the mixed-radix set, products of them, the largest lengths it
# takes, and neighbours that fall back to Bluestein (17, 19*...)
MIXED = [3, 5, 6, 7, 10, 11, 12, 13, 14, 18, 20, 21, 22, 24, 25, 26, 27, 39, 48, 49, 60, 77,
         81, 96, 100, 121, 125, 143, 169, 243, 343, 360, 625, 720, 729, 1000, 1001, 1331, 1536,
         2048 + 1024, 2187, 2197, 2401, 2500, 3000, 3125, 3375, 3840, 4000, 4095, 4050, 19 * 5,
         17 * 3,
         # the compiled specialisations (fft_specs*.hip): group 0, and the
         # two-pass / three-pass / above-4096 (re/im exchange) lists of 1-3
         480, 960, 1200, 1500, 1920, 2000, 2400,
         120, 160, 500, 600, 640, 750, 768, 800, 900, 1152, 1600, 2160, 2880, 4500, 5000,
         5120, 6000, 6400, 7500, 8000,
         # four-step row lengths (two to four passes, radix 7 included)
         375, 882, 1125, 1764, 1875, 2250, 3528, 3750, 6250,
         # 44.1 kHz audio frame lengths (radix 7 twice)
         441, 735, 1323, 1470, 2205, 2646, 2940, 4410, 5880]


@pytest.mark.parametrize("n", MIXED)
def test_mixed_radix_vs_oracle(gdsp, oracle, n):
    if n > 4096:  # specialisations only beyond the runtime-radix kernel
        D = __import__("importlib").import_module("go-dsp_amd.device")
        assert D.plan(n).kind == 5, n
    rng = np.random.default_rng(1000 + n)
    batch = 5
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = rng.uniform(-1, 1, (batch, n))
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL


# 2049 .. 3072: the fused chirp-z on M = 6144 (chirpz6k.hip; with
# GDSP_ALGO_CHIRPZ_POW2, M = 8192 with the n-aware pruning, n <= 12 T), 3073
# and 4093 M = 8192 without pruning
@pytest.mark.parametrize("n", [3, 5, 100, 2049, 3000, 3072, 3073, 4093, 4097, 10000])
def test_chirpz_plan_vs_oracle(gdsp, oracle, n):
    # the reference's own algorithm (Bluestein) on the device API, against the
    # oracle and against the default plan for the same length
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(2000 + n)
    x = rng.uniform(-1, 1, (7, n)) + 1j * rng.uniform(-1, 1, (7, n))
    xt = torch.from_numpy(x).cuda()
    yc = D.fft_batch(xt, chirpz=True).cpu().numpy()
    yd = D.fft_batch(xt).cpu().numpy()
    ref = oracle.fft_rows(x)
    assert row_nrel(yc, ref) < TOL and row_nrel(yd, ref) < TOL
    yci = D.fft_batch(xt, inverse=True, chirpz=True).cpu().numpy()
    assert row_nrel(yci, oracle.ifft_rows(x)) < TOL


# The fused chirp-z on M = 16 * RB * 16 (chirpz6k.hpp): the smallest such M
# >= 2n - 1 over the kept pass-B radices (chirpz6k.hip kC6RB), 129 <= n <=
# 3200 (RB <= 6: several transforms per workgroup), where bluestein.go:70 pads
# to NextPowerOf2(2n - 1) (and keeps it outside that range or where smaller);
# the four-pass kernel (R1, R2) for 4097 <= n <= 6144. Per entry the first
# and last prime of its range, the ranges' ends, and lengths that are smooth
# (3072 = 2^10 * 3, 1500, 1536: the mixed-radix kernel by default, chirp-z
# only when forced)
C6_RB = [3, 4, 5, 6, 9, 10, 12, 13, 14, 15, 16, 18, 20, 21, 24, 25]
C6K = [129, 131, 200, 251, 257, 383, 389, 509, 521, 523, 631, 641, 709, 761, 769, 887, 907, 1021,
       1024,
       1025, 1031, 1151, 1153, 1279, 1283, 1399, 1409, 1531, 1543, 1663, 1667, 1789, 1801,
       1913, 1931, 2039, 2049, 2053, 2297, 2307, 2309, 2557, 2579, 2687, 2689, 2729, 2803, 2819,
       3000, 3001, 3067, 3071, 3072, 3073, 3079, 3191, 3203, 3323, 3329, 3583, 3593, 3833,
       3847, 4093, 4096, 1500, 1536, 2062,
       3449, 3457, 4099, 4603, 4621, 5119, 5147, 5351, 5381, 5749, 5779, 6143, 6151, 6911, 6917,
       7159, 7177, 7673, 7681, 8059, 8069, 8191, 4097, 8192, 6000]


# the four-pass kernel's (R1, R2) (chirpz4_kernel, M = 256 R1 R2; chirpz6k.hip kC4)
C4_RR = [(6, 6), (8, 5), (8, 6)]


def c6_m(n):  # (the power of 2 below 129 and where it is smaller)
    pow2 = 1 << (2 * n - 2).bit_length()
    if n < 129:
        return pow2
    cands = [next((256 * rb for rb in C6_RB if 256 * rb >= 2 * n - 1), pow2),
             next((256 * a * b for a, b in C4_RR if 256 * a * b >= 2 * n - 1), pow2)]
    return min(cands + [pow2])


@pytest.mark.parametrize("n", C6K)
def test_chirpz6k_vs_oracle(gdsp, oracle, n):
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    pc = D.plan(n, chirpz=True)
    m, m_ref = c6_m(n), 1 << (2 * n - 2).bit_length()
    assert (pc.kind, pc.m) == (3, m), (n, pc.kind, pc.m)
    rng = np.random.default_rng(6144 + n)
    for batch in (1, 5):
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        xt = torch.from_numpy(x).cuda()
        ref = oracle.fft_rows(x)
        assert row_nrel(D.fft_batch(xt, chirpz=True).cpu().numpy(), ref) < TOL
        yi = D.fft_batch(xt, inverse=True, chirpz=True).cpu().numpy()
        assert row_nrel(yi, oracle.ifft_rows(x)) < TOL
        # in place: every row is read into registers before its first store
        xc = xt.clone()
        D.fft_batch(xc, xc, chirpz=True)
        torch.cuda.synchronize()
        assert row_nrel(xc.cpu().numpy(), ref) < TOL
    # host API (default plan: chirp-z for the primes, mixed radix when smooth)
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    xr = rng.uniform(-1, 1, (3, n))
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    # the reference's M on request (GDSP_ALGO_CHIRPZ_POW2), same results
    F.SetAlgorithm(F.ALGO_CHIRPZ_POW2)
    try:
        assert D.plan(n, chirpz=True).m == m_ref
        y8 = D.fft_batch(xt, chirpz=True).cpu().numpy()
    finally:
        F.SetAlgorithm(0)
    assert row_nrel(y8, ref) < TOL


@pytest.mark.parametrize("n,batch", [(3000, 65536), (1151, 65536), (2297, 32768), (2687, 32768),
                                     (3191, 32768), (311, 65537), (523, 65535), (700, 65533),
                                     (4603, 16384), (6143, 16384), (8191, 8192)])
def test_chirpz6k_large_batch_properties(gdsp, n, batch):
    """A full-occupancy grid (65 536 rows of n = 3000, the BASELINE shape; the
    pass-B radices 9, 18, 21 and 25 — the last one held to 128 VGPRs with 8
    spilled — and 3, 5, 6, several transforms per workgroup with a partial
    last one, at 2^24-2^27 samples): linearity and the forward/inverse round
    trip on every row, and eight rows against a float64 direct DFT (numpy)."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(n, chirpz=True).m == c6_m(n)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.complex(torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5,
                      torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5)
    y = D.fft_batch(x, chirpz=True)
    z = D.fft_batch(y, inverse=True, chirpz=True)
    err = ((z - x).abs().amax(dim=1) / x.abs().amax(dim=1)).max().item()
    # (the reference's unreduced chirp angle, bluestein.go:53: ~1e-12 above n = 4096)
    assert err < (1e-12 if n <= 3200 else 1e-11), err
    y2 = D.fft_batch(2.0 * x[:64] - 1j * x[64:128], chirpz=True)
    lin = ((y2 - (2.0 * y[:64] - 1j * y[64:128])).abs().max() / y[:128].abs().max()).item()
    assert lin < 1e-13, lin
    rows = [r % batch for r in (0, 1, 777, 4096, 30000, batch - 2, batch - 1, 12345)]
    xs = x[rows].cpu().numpy()
    ref = np.fft.fft(xs, axis=1)
    assert row_nrel(y[rows].cpu().numpy(), ref) < TOL


# smooth lengths beyond one kernel: four-step over one-kernel factors
# (audio rates 44100 = 210^2, 48000; 2^16 * 3; 10^6) and neighbours that are
# not smooth (8209 prime, 4100 = 4 * 25 * 41) and stay Bluestein
MIXED4 = [4100, 5000, 6000, 8190, 10000, 44100, 48000, 3 << 16, 8209, 100000, 1000000,
          # single-radix columns (25 x 3528, 25 x 882, 9 x 2187) and power-of-2
          # columns (16 x 1875): three passes
          88200, 22050, 19683, 30000,
          # runtime-compiled mixed-radix columns (colfixed_kernel): 16-column
          # tiles (125 x 3125, 75 x 8000, 125 x 8008, 243 x 6561), 8 columns
          # (343 x 2401) and 4 columns (630 x 7875): three passes
          390625, 600000, 1001000, 1594323, 823543, 4961250,
          # 17 * 2^16: power-of-2 columns, rows of 2176 = 17 * 128
          1114112,
          # rows through the fused chirp-z kernel: 64 x 8191, 100 x 4099,
          # 143 x 1009, 91 x 7919
          524224, 409900, 144287, 720629,
          # rows through the output-split chirp-z: 64 x 8209, 2 x 10007, 3 x 12289
          525376, 20014, 36867]


@pytest.mark.parametrize("n", MIXED4)
def test_mixed_fourstep_vs_oracle(gdsp, oracle, n):
    rng = np.random.default_rng(3000 + n)
    batch = 3 if n <= 100000 else 1
    x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
    y = gdsp.fft.FFTBatch(x)
    if n > 2000000:
        # The reference's chirp angle pi/n*k^2 is not reduced (bluestein.go:53),
        # so its own error grows with n: at 4961250 the oracle is 5.5e-10
        # normwise and 1.1e-9 max-abs from the exact DFT, against 7e-16 for
        # the engine (scripts/archive/acc_probe.py). Here the bound against the oracle
        # is the reference tests' own 1e-8 (Float64Equal), the engine is held
        # to the exact DFT, and the inverse to a round trip (the oracle takes
        # ~16 s per transform at this size).
        assert row_nrel(y, oracle.fft_rows(x)) < 1e-8
        assert row_nrel(y, np.fft.fft(x, axis=1)) < 1e-13
        assert row_nrel(gdsp.fft.FFTBatch(y, inverse=True), x) < TOL
        return
    assert row_nrel(y, oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = rng.uniform(-1, 1, (batch, n))
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL


def test_mixed_fourstep_in_place_device(gdsp, oracle):
    # device API with in == out and a batch that spans transposes' tails
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    n, batch = 44100, 5
    x = oracle.fill_uniform(2 * n * batch, 0x5EED, 7).view(np.complex128).reshape(batch, n)
    xt = torch.from_numpy(x).cuda()
    D.fft_batch(xt, out=xt)
    assert D.plan(n).kind == 6
    assert row_nrel(xt.cpu().numpy(), oracle.fft_rows(x)) < TOL


def test_mixed_radix_large_batch(gdsp, oracle):
    # grid wider than one launch's tail handling: odd batch, transforms per
    # workgroup > 1 (n = 12: 4 per group of 16 threads)
    for n, batch in [(12, 1001), (3000, 333), (100, 4099)]:
        x = oracle.fill_uniform(2 * n * batch, 0x5EED, n).view(np.complex128).reshape(batch, n)
        y = gdsp.fft.FFTBatch(x)
        assert row_nrel(y, oracle.fft_rows(x)) < TOL, n
        assert row_nrel(gdsp.fft.FFTBatch(y, inverse=True), x) < TOL, n


def test_TestFFTN(gdsp, refvec):
    # fft/fft_test.go:225-239
    U = gdsp.dsputils
    for c in refvec["fftnTests"]:
        m = U.MakeMatrix(U.ToComplex(c["in"]), c["dim"])
        o = U.MakeMatrix(cpx(c["out"]), c["dim"])
        assert gdsp.fft.FFTN(m).PrettyClose(o)
        assert gdsp.fft.IFFTN(o).PrettyClose(m)


@pytest.mark.parametrize("dims", [[2, 2, 3], [5], [16, 16], [3, 5, 7], [64, 1, 32], [32, 16, 8, 4],
                                  [1024, 16], [2048, 9], [7, 100, 3], [4, 4096], [2, 3, 3000],
                                  [600, 20], [2, 1, 1, 2], [8209, 2], [2, 3, 8209],
                                  [3, 257, 4], [37, 41]])  # (prime axes: Rader)
def test_fftn_vs_oracle(gdsp, oracle, dims):
    rng = np.random.default_rng(sum(dims))
    n = int(np.prod(dims))
    x = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    m = gdsp.dsputils.MakeMatrix(x, dims)
    assert nrel(gdsp.fft.FFTN(m).list, oracle.fftn(x, dims)) < TOL
    assert nrel(gdsp.fft.IFFTN(m).list, oracle.fftn(x, dims, inverse=True)) < TOL


@pytest.mark.parametrize("shape", [(8, 6, 5), (3, 1024, 7), (4096, 12), (100, 3000), (2, 2048, 9)])
def test_fft_axis_device(gdsp, oracle, shape):
    # gdsp_fft_axis_device: one axis of computeFFTN (fft.go:172-185)
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(sum(shape))
    x = rng.uniform(-1, 1, shape) + 1j * rng.uniform(-1, 1, shape)
    xt = torch.from_numpy(x).cuda()
    for axis in range(len(shape)):
        for inv in (False, True):
            got = D.fft_axis(xt, axis, inverse=inv).cpu().numpy()
            m = np.moveaxis(x, axis, -1)
            lines = m.reshape(-1, shape[axis])
            ref = (oracle.ifft_rows if inv else oracle.fft_rows)(lines)
            ref = np.moveaxis(ref.reshape(m.shape), -1, axis)
            assert row_nrel(got.reshape(-1, 1).T, ref.reshape(-1, 1).T) < TOL, (axis, inv)


def test_fft2_sharded_one_rank(gdsp, oracle):
    # the multi-GPU FFT2 driver at world size 1 (no collective)
    import torch
    Dd = __import__("importlib").import_module("go-dsp_amd.distributed")
    for R, C in [(64, 48), (1024, 1000), (8192, 16)]:
        x = oracle.fill_uniform(2 * R * C, 0x5EED, R + C).view(np.complex128).reshape(R, C)
        for inv in (False, True):
            y = Dd.fft2_sharded(torch.from_numpy(x).cuda(), R, inverse=inv).cpu().numpy()
            assert nrel(y, oracle.fft2(x, inverse=inv)) < TOL, (R, C, inv)


def test_concurrent_host_calls(gdsp, oracle):
    # the reference's FFT is safe to call from many goroutines (RWMutex-guarded
    # caches): host-pointer calls from 8 threads at once, each
    # with its own lengths (plan builds race on first use), all correct
    import threading
    sizes = [4096, 3000, 1000, 8192, 100, 5000, 44100, 17]
    errs, fails = {}, []

    def work(i):
        try:
            n = sizes[i]
            rng = np.random.default_rng(50 + i)
            for _ in range(6):
                x = rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))
                y = gdsp.fft.FFTBatch(x)
                z = gdsp.fft.FFTBatch(y, inverse=True)
                e = max(row_nrel(y, oracle.fft_rows(x)), row_nrel(z, x))
                errs[i] = max(errs.get(i, 0.0), e)
            p, _ = gdsp.spectral.Pwelch(rng.standard_normal(3000), 1.0,
                                        gdsp.spectral.PwelchOptions(NFFT=256))
            assert np.all(np.isfinite(p))
        except Exception as ex:  # surfaced below
            fails.append((i, repr(ex)))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(sizes))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not fails, fails
    assert max(errs.values()) < TOL, errs


def test_concurrent_runtime_compiled_plans(gdsp, oracle):
    # six threads whose first call each builds a plan through hipRTC at the
    # same time (lengths used nowhere else in the suite): one-kernel mixed
    # radix (1890, 2310, 5292, 6930, 2730) and a runtime-compiled column pass
    # (700000 = 100 x 7000)
    import threading
    sizes = [1890, 2310, 5292, 6930, 2730, 700000]
    errs, fails = {}, []

    def work(i):
        try:
            n = sizes[i]
            rng = np.random.default_rng(90 + i)
            b = 1 if n > 100000 else 3
            x = rng.standard_normal((b, n)) + 1j * rng.standard_normal((b, n))
            y = gdsp.fft.FFTBatch(x)
            z = gdsp.fft.FFTBatch(y, inverse=True)
            errs[i] = max(row_nrel(y, oracle.fft_rows(x)), row_nrel(z, x))
        except Exception as ex:  # surfaced below
            fails.append((i, repr(ex)))

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(sizes))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not fails, fails
    assert max(errs.values()) < TOL, errs


def test_random_lengths_every_plan_kind(gdsp, oracle):
    # 40 seeded random lengths in [2, 40000]: powers of 2, compiled and
    # runtime-radix mixed lengths, both four-step column forms, the general
    # five-pass form and fused / composed Bluestein, forward, inverse and real
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(20261016)
    lengths = sorted(set(int(v) for v in rng.integers(2, 40001, 40)))
    kinds = set()
    for n in lengths:
        batch = 2
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL, n
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL, n
        assert row_nrel(gdsp.fft.FFTRealBatch(x.real.copy()),
                        oracle.fft_rows(x.real.astype(np.complex128))) < TOL, n
        kinds.add(D.plan(n).kind)
    assert {3, 4} <= kinds, kinds  # random lengths are mostly Bluestein's


def test_random_smooth_lengths(gdsp, oracle):
    # seeded random 13-smooth lengths up to 200000: one-kernel mixed radix
    # (compiled or runtime radices), the power-of-2-column and single-radix-
    # column four-steps and the general five-pass form
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(7)
    lengths = set()
    while len(lengths) < 40:
        n = 1
        for p, emax in ((2, 10), (3, 6), (5, 5), (7, 3), (11, 1), (13, 1)):
            n *= p ** int(rng.integers(0, emax + 1))
        if 2 <= n <= 200000 and n & (n - 1):
            lengths.add(n)
    kinds = set()
    for n in sorted(lengths):
        batch = 2
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL, n
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL, n
        kinds.add(D.plan(n).kind)
    assert {5, 6} <= kinds, kinds


def test_random_lengths_beyond_one_kernel(gdsp, oracle):
    # seeded arbitrary lengths in (8192, 300000]: three-pass splits with
    # mixed-radix or chirp-z rows, the five-pass form and the composed
    # chirp-z (a prime factor above 8192), forward and inverse
    D = __import__("importlib").import_module("go-dsp_amd.device")
    rng = np.random.default_rng(424242)
    kinds = set()
    for n in sorted(set(int(v) for v in rng.integers(8193, 300001, 14))):
        x = rng.uniform(-1, 1, (1, n)) + 1j * rng.uniform(-1, 1, (1, n))
        assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL, n
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL, n
        kinds.add(D.plan(n).kind)
    assert {4, 6} <= kinds, kinds


def test_random_large_smooth_lengths(gdsp, oracle):
    # seeded random 13-smooth lengths in (200000, 2000000]: the three-pass
    # column splits (power-of-2, single-radix and runtime-compiled mixed-radix
    # columns) and whatever falls through to the five-pass form. Forward only
    # (the oracle takes 0.5-2 s per transform here); the inverse path is the
    # same kernels with conj in / conj + scale out, covered at smaller sizes.
    rng = np.random.default_rng(11)
    lengths = set()
    while len(lengths) < 8:
        n = 1
        for p, emax in ((2, 12), (3, 8), (5, 6), (7, 4), (11, 2), (13, 2)):
            n *= p ** int(rng.integers(0, emax + 1))
        if 200000 < n <= 2000000 and n & (n - 1):
            lengths.add(n)
    for n in sorted(lengths):
        x = rng.uniform(-1, 1, (1, n)) + 1j * rng.uniform(-1, 1, (1, n))
        assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL, n


@pytest.mark.parametrize("n,kind", [(810, 5), (1001, 5), (4095, 5), (4320, 5), (5400, 5),
                                    (6144, 5), (7000, 5), (7680, 5), (8190, 5), (6561, 5),
                                    (7290, 5), (4802, 5), (7938, 5), (8191, 3),
                                    # radices 17, 19, 23 (runtime-compiled lists only)
                                    (323, 5), (529, 5), (4352, 5), (7600, 5), (6900, 5),
                                    (7429, 5), (899, 5), (7936, 5), (6293, 5)])
def test_jit_specialisations(gdsp, oracle, n, kind):
    # smooth lengths without a compiled specialisation get one compiled at
    # plan creation (mixed_jit.hip, hipRTC); above 4096 they would otherwise
    # be Bluestein. 8190 = 15 * 13 * 7 * 6, 6561 = 9^4 and 7290 = 10 * 9^3 need
    # 683-810 threads per transform (radix 6/9/13 passes); 4802 = 2 * 7^4 and
    # 7938 = 2 * 3^4 * 7^2 have no list shorter than five passes; 8191 is prime
    # (8190's list needs 683 threads per transform: chirp-z, kind 3).
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(n).kind == kind, n
    rng = np.random.default_rng(4000 + n)
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTRealBatch(x.real.copy()),
                    oracle.fft_rows(x.real.astype(np.complex128))) < TOL


@pytest.mark.parametrize("nfft,nov", [(810, 405), (5400, 2700), (8190, 4095)])
def test_jit_pwelch(gdsp, oracle, nfft, nov):
    rng = np.random.default_rng(nfft)
    x = rng.standard_normal(40 * nfft)
    o = gdsp.spectral.PwelchOptions(NFFT=nfft, Noverlap=nov)
    p, f = gdsp.spectral.Pwelch(x, 3.0, o)
    pr, fr = oracle.pwelch(x, 3.0, nfft=nfft, noverlap=nov)
    assert nrel(p, pr) < TOL and nrel(f, fr) == 0.0


@pytest.mark.parametrize("n", [17, 101, 1009, 2053, 2741, 3001, 3571])
def test_chirpz_primes(gdsp, oracle, n):
    # primes take the fused chirp-z kernel (M = NextPowerOf2(2n - 1), as
    # bluestein.go:70), forward, inverse and real input
    rng = np.random.default_rng(7000 + n)
    x = rng.uniform(-1, 1, (5, n)) + 1j * rng.uniform(-1, 1, (5, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
    xr = x.real.copy()
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL


def _dev_lib() -> str:
    """The development build (make -C go-dsp_amd/csrc DEV=1, built by
    __graft_entry__.build()): the measured-and-rejected kernels below and
    their switches live only there."""
    path = os.path.join(REPO, "go-dsp_amd", "lib_dev", "libgdspfft.so")
    if not os.path.exists(path):
        pytest.skip("development build (go-dsp_amd/lib_dev) not built")
    return path


# the wave-resident chirp-z kernel (fft_wave.hip, development build,
# gdsp_dev_fft_batch_chirpz_wave):
# Q = M/2048 waves per transform, Q = 1 (n <= 1024), 2, 4; the edges of each
# range, primes, and batches that leave the last workgroup partly empty (2 or
# 4 transforms per workgroup at Q = 2, 1). Its exchanges are a wave-local LDS
# transpose and a v_permlane32_swap (no workgroup barrier inside a transform).
WAVE_N = [513, 700, 1009, 1023, 1024, 1025, 1500, 2039, 2047, 2048, 2049, 2053, 3000, 3072,
          3073, 4093, 4095, 4096]

_DEV_CHIRPZ = r'''
import ctypes, importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle, torch
L = importlib.import_module("go-dsp_amd._lib")
assert L.is_dev_build()
lib = L.lib()
fn = getattr(lib, os.environ["DEV_FN"])
def row_nrel(a, b):
    return max(np.linalg.norm(x - y) / np.linalg.norm(y) for x, y in zip(a, b))
def run(x, inverse):
    xt = torch.from_numpy(x).cuda()
    yt = torch.empty_like(xt)
    st = fn(x.shape[1], ctypes.c_void_p(xt.data_ptr()), ctypes.c_void_p(yt.data_ptr()),
            x.shape[0], int(inverse), None)
    assert st == 0, st
    torch.cuda.synchronize()
    return yt.cpu().numpy()
for n in [int(v) for v in os.environ["DEV_N"].split()]:
    if os.environ["DEV_FN"].endswith("wave"):
        m = 1 << (2 * n - 2).bit_length()  # bluestein.go:70
        assert lib.gdsp_dev_chirpz_wave_q(n) == m // 2048, n
    rng = np.random.default_rng(9000 + n)
    for batch in (1, 5, 7):
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        e = row_nrel(run(x, False), oracle.fft_rows(x))
        ei = row_nrel(run(x, True), oracle.ifft_rows(x))
        assert e < 1e-9 and ei < 1e-9, (n, batch, e, ei)
print("ok")
'''


def _run_dev(code, **env):
    env = dict(os.environ, REPO=REPO, GDSP_LIB=_dev_lib(), **env)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_chirpz_wave_kernel():
    _run_dev(_DEV_CHIRPZ, DEV_FN="gdsp_dev_fft_batch_chirpz_wave", DEV_N=" ".join(map(str, WAVE_N)))


SHFL_N = [2049, 2500, 3000, 3001, 4095, 4096]


def test_chirpz_shuffle_kernel():
    """The M = 8192 chirp-z kernel whose FFTs keep one exchange inside the
    wave (bluestein_shfl.hip, development build) against the oracle: forward
    and inverse, batch 1 and ragged 5 / 7, over 2049 <= n <= 4096."""
    _run_dev(_DEV_CHIRPZ, DEV_FN="gdsp_dev_fft_batch_chirpz_shfl", DEV_N=" ".join(map(str, SHFL_N)))


def test_pwelch_shuffle_kernel():
    """The NFFT 4096 / 50 % Pwelch kernel with the in-wave second exchange
    (pwelch_shfl.hip, development build: DPP row shifts and
    v_permlane16/32_swap) against the oracle: even and odd segment counts, a
    one-pair call, and Hann / Hamming windows."""
    _run_dev(_PW_DEV, DEV_FN="gdsp_dev_pwelch4096_shfl_accumulate")


_PW_DEV = r'''
import ctypes, importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle, torch
g = importlib.import_module("go-dsp_amd")
L = g._lib.lib()
P = lambda t: ctypes.c_void_p(t.data_ptr())
for n, win in ((40960, "hann"), (38913, "hann"), (6144, "hann"), (100000, "hamming"), (8192, "hann")):
    x = np.random.default_rng(n).standard_normal(n)
    w = getattr(g.window, win.capitalize())(4096)
    S = g.spectral.segment_count(n, 4096, 2048)
    xt = torch.from_numpy(x).cuda()
    wt = torch.tensor(np.asarray(w, np.float64)).cuda()
    acc = torch.zeros(4096, dtype=torch.float64, device="cuda")
    assert getattr(L, os.environ["DEV_FN"])(P(xt), n, 0, S, P(wt), P(acc), None) == 0
    p, f = g.spectral.finalize(acc.cpu().numpy(), S, 4096, 4096, np.asarray(w), 2.0, False)
    pr, fr = oracle.pwelch(x, 2.0, nfft=4096, noverlap=2048, window_kind=win)
    e = np.linalg.norm(p - pr) / np.linalg.norm(pr)
    assert e < 1e-9, (n, win, e)
print("ok")
'''


def test_pwelch_three_wave_kernel():
    """The NFFT 4096 / 50 % row kernel reshaped for three workgroups per CU
    (pwelch_row3.hip, development build: the next pair by LDS-DMA, a half-size
    exchange, 42 spilled VGPRs at the 168-VGPR cap) against the oracle, on the
    same cases as the shuffle kernel."""
    _run_dev(_PW_DEV, DEV_FN="gdsp_dev_pwelch4096_row3_accumulate")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4096, 3000, 1 << 20, 8209, 5400])
def test_ensure_radix2_factors_then_fft(gdsp, oracle, n):
    """fft.EnsureRadix2Factors (radix2.go:35-37) pre-builds the plan the next
    fft.FFT uses, as BenchmarkFFT does before timing (fft_test.go:273)."""
    gdsp.fft.EnsureRadix2Factors(n)
    gdsp.fft.EnsureRadix2Factors(n)  # idempotent
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    assert nrel(gdsp.fft.FFT(x), oracle.fft(x)) < (1e-8 if n > 2000000 else 1e-9)
    # chirp-z lengths carry the reference's unreduced chirp angle (~1e-12 at 8209)
    assert nrel(gdsp.fft.IFFT(gdsp.fft.FFT(x)), x) < 1e-11


@pytest.mark.gpu
def test_chirpz_convolution_length_selection():
    """Which convolution length M the composed chirp-z takes (gdsp_plan_info),
    and that every selectable path agrees with the oracle: by default 8209
    runs as the output-split chirp-z (2 parts on M = 16384) and 16411 on the
    reference's NextPowerOf2(2n-1) (bluestein.go:70), whose FFT takes two HBM
    passes (2^15..2^20; a smooth M <= 0.55 of it is taken only outside that
    range); GDSP_ALGO_NO_CHIRPZ_PARTS puts 8209 on the composed chirp-z too,
    GDSP_ALGO_CHIRPZ_POW2 forces the power of 2, and GDSP_ALGO_CHIRPZ_UNFUSED
    takes the unfused composition (gdsp_set_algorithm)."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
import torch
flags = int(os.environ["ALGO"])
g.fft.SetAlgorithm(flags)
pow2 = bool(flags & g.fft.ALGO_CHIRPZ_POW2)
parts = not flags & g.fft.ALGO_NO_CHIRPZ_PARTS
rng = np.random.default_rng(8)
for n in (8209, 16411):
    p = D.plan(n)
    ref_m = 1 << (2 * n - 2).bit_length()
    if parts and n == 8209:
        assert (p.kind, p.parts, p.m) == (3, 2, 16384), (n, p.kind, p.parts, p.m)
    else:
        assert p.kind == 4 and p.parts == 1, (n, p.kind, p.parts)
    if p.kind == 3:
        pass
    else:
        assert p.m == ref_m, (n, p.m, pow2)
    assert D.plan(n, chirpz=True).m == ref_m
    x = rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))
    for inv in (False, True):
        y = g.fft.FFTBatch(x, inverse=inv)
        ref = oracle.ifft_rows(x) if inv else oracle.fft_rows(x)
        err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
        assert err < 1e-9, (n, inv, err)
print("ok", flags)
'''
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    for extra in (0, F.ALGO_NO_CHIRPZ_PARTS, F.ALGO_CHIRPZ_POW2 | F.ALGO_NO_CHIRPZ_PARTS,
                  F.ALGO_CHIRPZ_UNFUSED | F.ALGO_NO_CHIRPZ_PARTS):
        env = dict(os.environ, REPO=REPO, ALGO=str(extra))
        r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0 and "ok" in r.stdout, (extra, r.stdout + r.stderr[-3000:])


@pytest.mark.gpu
def test_chirpz_composed_two_pass_fft_m():
    """The composed chirp-z on a power-of-2 M in 2^15..2^20 runs both FFT_M as
    the two-pass four-step with the b-hat and output steps in the rows'
    transposed store (rowfft_t_kernel modes 2 and 3): primes whose
    NextPowerOf2(2n-1) is each of those M (GDSP_ALGO_CHIRPZ_POW2, so the
    reference's M), batch 2, forward / inverse / real, against the oracle."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"]); sys.path.insert(0, os.path.join(os.environ["REPO"], "oracle"))
import numpy as np, oracle
g = importlib.import_module("go-dsp_amd")
D = importlib.import_module("go-dsp_amd.device")
g.fft.SetAlgorithm(g.fft.ALGO_CHIRPZ_POW2 | g.fft.ALGO_NO_CHIRPZ_PARTS)
rng = np.random.default_rng(15)
for n, lm in ((16381, 15), (16411, 16), (40009, 17), (65537, 18), (200003, 19), (262147, 20)):
    p = D.plan(n)
    assert p.kind == 4 and p.m == 1 << lm, (n, p.kind, p.m)
    x = rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))
    for inv in (False, True):
        y = g.fft.FFTBatch(x, inverse=inv)
        ref = oracle.ifft_rows(x) if inv else oracle.fft_rows(x)
        err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(y, ref))
        assert err < 1e-9, (n, inv, err)
    xr = x.real.copy()
    yr = g.fft.FFTRealBatch(xr)
    ref = oracle.fft_rows(xr.astype(np.complex128))
    err = max(np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(yr, ref))
    assert err < 1e-9, (n, "real", err)
print("ok")
'''
    env = dict(os.environ, REPO=REPO)
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr[-3000:]


# primes whose NextPowerOf2(2n-1) is 32768: 2 parts (8209, 10007, 10909), 3
# (11003, 12281), 4 (12289), 6 (13999), 8 (14563, the largest length with P <= 8)
PARTS = [(8209, 2), (10007, 2), (10909, 2), (11003, 3), (12281, 3), (12289, 4), (13999, 6),
         (14563, 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,parts", PARTS)
def test_chirpz_output_parts_vs_oracle(gdsp, oracle, n, parts):
    """Output-split chirp-z (bluestein_kernel PARTS): X[k0 + k], k < ceil(n/P),
    from P fused circular convolutions of M = 16384 >= n + ceil(n/P) - 1, for
    lengths whose reference M = NextPowerOf2(2n-1) = 32768 exceeds one kernel
    (bluestein.go:68-94). Forward, inverse and real input against the oracle
    (which runs the reference's M = 32768), batch 3 so row offsets are covered."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    p = D.plan(n)
    assert (p.kind, p.parts, p.m) == (3, parts, 16384), (n, p.kind, p.parts, p.m)
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    xt = torch.from_numpy(x).cuda()
    assert row_nrel(D.fft_batch(xt).cpu().numpy(), oracle.fft_rows(x)) < TOL
    assert row_nrel(D.fft_batch(xt, inverse=True).cpu().numpy(), oracle.ifft_rows(x)) < TOL
    xr = rng.uniform(-1, 1, (2, n))
    assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
    # an output tail the last part leaves partly empty, and the forced
    # chirp-z plan (reference M, composed) agreeing with it
    yc = D.fft_batch(xt[:1], chirpz=True).cpu().numpy()
    assert row_nrel(D.fft_batch(xt[:1]).cpu().numpy(), yc) < TOL


@pytest.mark.gpu
def test_chirpz_output_parts_in_place_large_batch(gdsp, oracle):
    """The parts of a row run in different workgroups, so an in-place call
    (in == out, and the four-step rows, which transform in place) must not let
    one part overwrite a row another has not read yet: large batches, so that
    parts of one row are not resident together, against the out-of-place
    result and sampled rows against the oracle."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    for n, batch in ((8209, 4096), (2 * 10007, 1024)):
        x = torch.empty((batch, n), dtype=torch.complex128, device="cuda")
        D.fill_uniform(x, 0xC0FFEE)
        y = D.fft_batch(x)
        D.fft_batch(x, x)
        torch.cuda.synchronize()
        # a race shows as O(1) errors; the same kernels in the same order agree
        assert float((x - y).abs().max() / y.abs().max()) < 1e-13, n
        D.fill_uniform(x, 0xC0FFEE)
        rows = [0, batch // 2, batch - 1]
        xs = x[rows].cpu().numpy()
        assert row_nrel(y[rows].cpu().numpy(), oracle.fft_rows(xs)) < TOL


# ---- Rader's algorithm (rader_fixed_kernel, plan kind 7) ---------------------
# primes whose n - 1 has a radix list: small (one pass: 17 -> 16; TPW > 1 with
# ragged last blocks), power-of-2 n - 1 (257), compiled-specialisation lists
# (3001 -> 25*15*8, 1201 -> 1200), runtime-compiled ones (2053 -> 2052 = 4 *
# 27 * 19, 2377 -> 2376 = 8 * 27 * 11), and n - 1 above 4096 (re/im LDS
# halves: 4801, 6007, 7681)
RADER = [17, 19, 23, 29, 31, 37, 41, 61, 97, 101, 257, 641, 1009, 1201, 1531, 2053, 2311, 2377,
         3001, 4801, 6007, 7681]


@pytest.mark.parametrize("n", RADER)
def test_rader_vs_oracle(gdsp, oracle, n):
    """Rader's algorithm against the reference restatement (its Bluestein,
    fft/bluestein.go:68-94) and numpy's float64 DFT: forward, inverse, real
    input, batches 1 and 7, in place on the device, and the same rows through
    the chirp-z plan (GDSP_ALGO_NO_RADER)."""
    D = __import__("importlib").import_module("go-dsp_amd.device")
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    # the default plan races Rader against chirp-z and keeps the faster
    assert D.plan(n).kind in (3, 7)
    F.SetAlgorithm(F.ALGO_NO_RACE)  # Rader itself
    try:
        _rader_checks(gdsp, oracle, D, F, n)
    finally:
        F.SetAlgorithm(0)


def _rader_checks(gdsp, oracle, D, F, n):
    import torch
    p = D.plan(n)
    assert (p.kind, p.m, p.runtime_compiled) == (7, n - 1, True), (n, p.kind, p.m)
    rng = np.random.default_rng(7000 + n)
    for batch in (1, 7):
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        ref = oracle.fft_rows(x)
        y = gdsp.fft.FFTBatch(x)
        assert row_nrel(y, ref) < TOL
        assert row_nrel(y, np.fft.fft(x, axis=1)) < 1e-13  # Rader itself is exact to roundoff
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
        xr = rng.uniform(-1, 1, (batch, n))
        assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
        xt = torch.from_numpy(x).cuda()
        D.fft_batch(xt, xt)
        torch.cuda.synchronize()
        assert row_nrel(xt.cpu().numpy(), ref) < TOL
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    assert nrel(gdsp.fft.FFT(x[0]), oracle.fft(x[0])) < TOL
    F.SetAlgorithm(F.ALGO_NO_RADER | F.ALGO_NO_RACE)
    try:
        assert D.plan(n).kind == 3
        yc = gdsp.fft.FFTBatch(x)
    finally:
        F.SetAlgorithm(F.ALGO_NO_RACE)
    assert row_nrel(yc, oracle.fft_rows(x)) < TOL


@pytest.mark.parametrize("n", [1031, 2039, 3067, 4099, 59, 2729, 8009, 8191])
def test_primes_without_radix_list_stay_chirpz(gdsp, oracle, n):
    # n - 1 with a prime factor above 31 (1030 = 2 * 5 * 103, 2038 = 2 * 1019, ...),
    # or whose list needs radix 29 / 31 (58 = 2 * 29, 2728 = 8 * 11 * 31) or
    # more than 640 threads per transform (8008 = 13 * 11 * 7 * 8: 728; 8190 =
    # 15 * 13 * 7 * 6: 683)
    D = __import__("importlib").import_module("go-dsp_amd.device")
    assert D.plan(n).kind == 3
    rng = np.random.default_rng(n)
    x = rng.uniform(-1, 1, (2, n)) + 1j * rng.uniform(-1, 1, (2, n))
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL


def test_rader_large_batch_properties(gdsp):
    """A full-occupancy grid of the prime 3001 (65 536 rows, the bench's
    prime3001 shape): forward/inverse round trip and linearity on every row,
    eight rows against numpy's float64 DFT."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    n, batch = 3001, 65536
    assert D.plan(n).kind in (3, 7)
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.complex(torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5,
                      torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5)
    y = D.fft_batch(x)
    z = D.fft_batch(y, inverse=True)
    err = ((z - x).abs().amax(dim=1) / x.abs().amax(dim=1)).max().item()
    assert err < 1e-12, err
    y2 = D.fft_batch(2.0 * x[:64] - 1j * x[64:128])
    lin = ((y2 - (2.0 * y[:64] - 1j * y[64:128])).abs().max() / y[:128].abs().max()).item()
    assert lin < 1e-13, lin
    rows = [0, 1, 777, 4096, 30000, 65534, 65535, 12345]
    xs = x[rows].cpu().numpy()
    assert row_nrel(y[rows].cpu().numpy(), np.fft.fft(xs, axis=1)) < 1e-13


# ---- prime-factor Rader (rader_pfa_kernel, plan kind 8) ---------------------------
# composites n = M * P <= 8192, P > 31 the largest prime factor with a Rader
# plan, gcd(M, P) = 1: the reference's Bluestein (fft/bluestein.go:68-94) on
# NextPowerOf2(2n - 1) replaced by the Good-Thomas map and M Rader transforms
PFA_CASES = [74, 111, 185, 259, 333, 407, 481, 518, 666, 777, 888, 925, 1147, 1184, 82, 129,
             265, 427, 803, 1067, 1111, 1507, 2222, 2410, 3027, 4097, 5045, 6010, 7206, 8072,
             8116]


def _pfa_split(n):
    f, m, d = [], n, 2
    while d * d <= m:
        while m % d == 0:
            f.append(d)
            m //= d
        d += 1
    if m > 1:
        f.append(m)
    P = max(f)
    return n // P, P


@pytest.mark.parametrize("n", PFA_CASES)
def test_rader_pfa_vs_oracle(gdsp, oracle, n):
    """Forward, inverse, real input, in place, batches 1 and 7, against the
    oracle (the reference's Bluestein restated) and numpy's float64 DFT; the
    forced chirp-z plan (GDSP_ALGO_NO_RADER) on the same rows."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    M, P = _pfa_split(n)
    # the default plan races kind 8 against the chirp-z plan and keeps the
    # faster: either way the oracle's results
    assert D.plan(n).kind in (3, 8)
    x = np.random.default_rng(n).uniform(-1, 1, (3, n)).astype(np.complex128)
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    # the prime-factor kernel itself, without the race
    F.SetAlgorithm(F.ALGO_NO_RACE)
    try:
        _pfa_checks(gdsp, oracle, D, F, n, M, P)
    finally:
        F.SetAlgorithm(0)


def _pfa_checks(gdsp, oracle, D, F, n, M, P):
    import torch
    p = D.plan(n)
    assert (p.kind, p.n1, p.n2, p.m, p.runtime_compiled) == (8, M, P, P - 1, True), \
        (n, p.kind, p.n1, p.n2, p.m)
    rng = np.random.default_rng(8000 + n)
    for batch in (1, 7):
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        ref = oracle.fft_rows(x)
        y = gdsp.fft.FFTBatch(x)
        assert row_nrel(y, ref) < TOL
        assert row_nrel(y, np.fft.fft(x, axis=1)) < 1e-13
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
        xr = rng.uniform(-1, 1, (batch, n))
        assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
        xt = torch.from_numpy(x).cuda()
        D.fft_batch(xt, xt)
        torch.cuda.synchronize()
        assert row_nrel(xt.cpu().numpy(), ref) < TOL
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    assert nrel(gdsp.fft.FFT(x[0]), oracle.fft(x[0])) < TOL
    assert nrel(gdsp.fft.IFFT(x[1]), oracle.ifft(x[1])) < TOL
    F.SetAlgorithm(F.ALGO_NO_RADER | F.ALGO_NO_RACE)
    try:
        assert D.plan(n).kind in (3, 4)
        yc = gdsp.fft.FFTBatch(x)
    finally:
        F.SetAlgorithm(F.ALGO_NO_RACE)
    assert row_nrel(yc, oracle.fft_rows(x)) < TOL


def test_rader_pfa_every_cofactor(gdsp, oracle):
    """Every cofactor M = 2 ... 32 beside P = 37 (36 = the Rader list): the
    native in-register DFTs and the coprime splits (14 = 2 x 7, 18 = 2 x 9,
    21, 22, 24, 26, 28, 30); 27 = 3^3 has neither (chirp-z)."""
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    F.SetAlgorithm(F.ALGO_NO_RACE)
    try:
        _pfa_cofactors(oracle)
    finally:
        F.SetAlgorithm(0)


def _pfa_cofactors(oracle):
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    for M in range(2, 33):
        n = 37 * M
        if M == 27:
            assert D.plan(n).kind == 3, n
            continue
        assert D.plan(n).kind == 8, (n, D.plan(n).kind)
        g = torch.Generator(device="cuda").manual_seed(M)
        x = torch.complex(torch.rand(301, n, dtype=torch.float64, device="cuda", generator=g) - 0.5,
                          torch.rand(301, n, dtype=torch.float64, device="cuda", generator=g) - 0.5)
        y = D.fft_batch(x)
        rows = [0, 150, 300]
        xs = x[rows].cpu().numpy()
        assert row_nrel(y[rows].cpu().numpy(), oracle.fft_rows(xs)) < TOL, n
        assert row_nrel(y[rows].cpu().numpy(), np.fft.fft(xs, axis=1)) < 1e-13, n
        z = D.fft_batch(y, inverse=True)
        assert float(((z - x).abs().amax(dim=1) / x.abs().amax(dim=1)).max()) < 1e-12, n


def test_rader_pfa_large_batch_properties(gdsp):
    """65 536 rows of 3027 = 3 x 1009 (the bench's shape): round trip and
    linearity on every row, eight rows against numpy."""
    import torch
    D = __import__("importlib").import_module("go-dsp_amd.device")
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    n, batch = 3027, 65536
    F.SetAlgorithm(F.ALGO_NO_RACE)
    try:
        _pfa_large_batch(D, n, batch)
    finally:
        F.SetAlgorithm(0)


def _pfa_large_batch(D, n, batch):
    import torch
    assert D.plan(n).kind == 8
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.complex(torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5,
                      torch.rand(batch, n, dtype=torch.float64, device="cuda", generator=g) - 0.5)
    y = D.fft_batch(x)
    z = D.fft_batch(y, inverse=True)
    err = ((z - x).abs().amax(dim=1) / x.abs().amax(dim=1)).max().item()
    assert err < 1e-12, err
    y2 = D.fft_batch(2.0 * x[:64] - 1j * x[64:128])
    lin = ((y2 - (2.0 * y[:64] - 1j * y[64:128])).abs().max() / y[:128].abs().max()).item()
    assert lin < 1e-13, lin
    rows = [0, 1, 777, 4096, 30000, 65534, 65535, 12345]
    xs = x[rows].cpu().numpy()
    assert row_nrel(y[rows].cpu().numpy(), np.fft.fft(xs, axis=1)) < 1e-13


# ---- chirp-z on a smooth convolution length (bluestein_fixed_kernel) ---------------
# the fused chirp-z (plan kind 3) with L >= 2n - 1 smooth instead of
# bluestein.go:70's NextPowerOf2(2n - 1) where the lane-cost model expects it
# cheaper: the same linear convolution, hence the same DFT
# (lengths where the lane-cost model has a smooth L below the fused kernel's M
# of round 6: 1031 on 2160 against 2304, 5209 / 5402 / 5519 on 10800 / 11520
# against 12288)
BLUFIX_CASES = [1031, 5209, 5402, 5519]


@pytest.mark.parametrize("n", BLUFIX_CASES)
def test_chirpz_smooth_l_vs_oracle(gdsp, oracle, n):
    D = __import__("importlib").import_module("go-dsp_amd.device")
    F = __import__("importlib").import_module("go-dsp_amd.fft")
    assert D.plan(n).kind == 3  # (smooth L or not: the race decides)
    x = np.random.default_rng(n).uniform(-1, 1, (3, n)).astype(np.complex128)
    assert row_nrel(gdsp.fft.FFTBatch(x), oracle.fft_rows(x)) < TOL
    F.SetAlgorithm(F.ALGO_NO_RACE)  # the model's candidate, L smooth
    try:
        _blufix_checks(gdsp, oracle, D, F, n)
    finally:
        F.SetAlgorithm(0)


def _blufix_checks(gdsp, oracle, D, F, n):
    import torch
    p = D.plan(n)
    L = p.m
    assert p.kind == 3 and p.runtime_compiled and L >= 2 * n - 1 and L & (L - 1), (n, p.kind, L)
    assert int(np.prod(p.radices)) == L and max(p.radices) <= 16, p.radices
    rng = np.random.default_rng(9000 + n)
    for batch in (1, 7):
        x = rng.uniform(-1, 1, (batch, n)) + 1j * rng.uniform(-1, 1, (batch, n))
        ref = oracle.fft_rows(x)
        y = gdsp.fft.FFTBatch(x)
        assert row_nrel(y, ref) < TOL
        assert row_nrel(y, np.fft.fft(x, axis=1)) < 1e-11  # the chirp's unreduced angle (bluestein.go:53)
        assert row_nrel(gdsp.fft.FFTBatch(x, inverse=True), oracle.ifft_rows(x)) < TOL
        xr = rng.uniform(-1, 1, (batch, n))
        assert row_nrel(gdsp.fft.FFTRealBatch(xr), oracle.fft_rows(xr.astype(np.complex128))) < TOL
        xt = torch.from_numpy(x).cuda()
        D.fft_batch(xt, xt)
        torch.cuda.synchronize()
        assert row_nrel(xt.cpu().numpy(), ref) < TOL
    x = rng.uniform(-1, 1, (3, n)) + 1j * rng.uniform(-1, 1, (3, n))
    assert nrel(gdsp.fft.FFT(x[0]), oracle.fft(x[0])) < TOL
    F.SetAlgorithm(F.ALGO_CHIRPZ_POW2 | F.ALGO_NO_RACE)
    try:
        q = D.plan(n)
        assert q.kind == 3 and q.m & (q.m - 1) == 0, (q.kind, q.m)
        yc = gdsp.fft.FFTBatch(x)
    finally:
        F.SetAlgorithm(F.ALGO_NO_RACE)
    assert row_nrel(yc, oracle.fft_rows(x)) < TOL
