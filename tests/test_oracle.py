"""Pins the CPU restatement (oracle/) to the reference's own golden vectors
(Float64Equal semantics, dsputils/compare.go:24,94-96) and to independent
oracles (numpy pocketfft, scipy.signal.welch). CPU only."""
import math

import numpy as np
import pytest

from conftest import cpx, nrel


def float64_equal(a, b):
    return abs(a - b) <= 1e-8 or abs(1 - a / b) <= 1e-8 if b != 0 else abs(a - b) <= 1e-8


def close_c(a, b):
    return len(a) == len(b) and all(
        float64_equal(x.real, y.real) and float64_equal(x.imag, y.imag) for x, y in zip(a, b))


def close_f(a, b):
    return len(a) == len(b) and all(float64_equal(x, y) for x, y in zip(a, b))


def test_fft_reference_vectors(oracle, refvec):
    # fft/fft_test.go:197-209 (TestFFT): FFTReal(in) ~ out, IFFT(out) ~ in
    assert len(refvec["fftTests"]) == 13
    for case in refvec["fftTests"]:
        out = cpx(case["out"])
        assert close_c(oracle.fft_real(case["in"]), out), case
        assert close_c(oracle.ifft(out), np.asarray(case["in"], np.complex128)), case


def test_fft2_reference_vectors(oracle, refvec):
    # fft/fft_test.go:211-223 (TestFFT2)
    for case in refvec["fft2Tests"]:
        x = np.asarray(case["in"], np.float64).astype(np.complex128)
        out = np.array([cpx(r) for r in case["out"]])
        y = oracle.fft2(x)
        assert all(close_c(a, b) for a, b in zip(y, out))
        yi = oracle.fft2(out, inverse=True)
        assert all(close_c(a, b) for a, b in zip(yi, x))


def test_fftn_reference_vectors(oracle, refvec):
    # fft/fft_test.go:225-239 (TestFFTN): FFTN(in) ~ out, IFFTN(out) ~ in
    assert refvec["fftnTests"]
    for case in refvec["fftnTests"]:
        x = np.asarray(case["in"], np.float64).astype(np.complex128)
        out = cpx(case["out"])
        assert close_c(oracle.fftn(x, case["dim"]), out), case["dim"]
        assert close_c(oracle.fftn(out, case["dim"], inverse=True), x), case["dim"]
    # and against numpy's N-D transform on a seeded ragged shape
    rng = np.random.default_rng(5)
    z = rng.standard_normal((3, 5, 7)) + 1j * rng.standard_normal((3, 5, 7))
    ref = np.fft.fftn(z).ravel()
    assert np.linalg.norm(oracle.fftn(z, [3, 5, 7]) - ref) / np.linalg.norm(ref) < 1e-12


def test_reverse_bits(oracle, refvec):
    # fft/fft_test.go:241-249
    for c in refvec["reverseBitsTests"]:
        assert oracle.reverse_bits(c["in"], c["sz"]) == c["out"]


def test_example_fft_real(oracle, refvec):
    # fft/fft_test.go:283-320 (ExampleFFTReal, printed to 0.1)
    a = [math.sin(2 * math.pi * n / 8.0) + 0.5 * math.sin(2 * math.pi * n / 4.0 + 3 * math.pi / 4)
         for n in range(8)]
    X = oracle.fft_real(a)
    for e in refvec["exampleFFTReal"]:
        r, th = abs(X[e["k"]]), math.degrees(math.atan2(X[e["k"]].imag, X[e["k"]].real))
        if float64_equal(r, 0):
            th = 0
        assert f"{r:.1f}" == f"{e['mag']:.1f}" and f"{th:.1f}" == f"{e['deg']:.1f}"


def test_pwelch_reference_vectors(oracle, refvec):
    # spectral/pwelch_test.go:48-60
    for c in refvec["pwelchTests"]:
        p, f = oracle.pwelch(c["x"], c["fs"])
        assert close_f(p, c["p"]) and close_f(f, c["freqs"])


def test_segment_reference_vectors(oracle, refvec):
    # spectral/spectral_test.go:58-67
    x = refvec["segmentTests"]["x"]
    for c in refvec["segmentTests"]["cases"]:
        segs = oracle.segment(x, c["size"], c["noverlap"])
        assert [list(s) for s in segs] == [[float(v) for v in r] for r in c["out"]]


@pytest.mark.parametrize("kind", ["hann", "hamming", "bartlett", "flattop", "blackman"])
def test_window_reference_vectors(oracle, refvec, kind):
    # window/window_test.go:61-94
    for c in refvec["windowTests"]:
        assert close_f(oracle.window(kind, c["L"]), c[kind])


def test_radix2_factor_table(oracle):
    # radix2.go:24-69: T_4 exact, doubling construction
    t4 = oracle.radix2_factors(4)
    assert list(t4) == [1, -1j, -1, 1j]
    t = oracle.radix2_factors(4096)
    k = np.arange(4096)
    assert np.max(np.abs(t - np.exp(-2j * np.pi * k / 4096))) < 1e-15
    assert np.array_equal(t[::2], oracle.radix2_factors(2048))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8, 12, 16, 100, 1024, 3000, 4096])
def test_oracle_vs_numpy(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    # non-powers of 2 go through Bluestein, whose chirp angle pi/n*k*k is not
    # reduced mod 2n (fft/bluestein.go:53): ~1e-12 against the exact DFT at
    # n = 3000, a property of the reference itself
    tol = 1e-12 if n & (n - 1) == 0 else 1e-11
    assert nrel(oracle.fft(x), np.fft.fft(x)) < tol
    assert nrel(oracle.ifft(x), np.fft.ifft(x)) < tol
    if n > 1:
        y = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        ref = np.fft.ifft(np.fft.fft(x) * np.fft.fft(y))
        assert nrel(oracle.convolve(x, y), ref) < tol


def test_golden_fixtures_match_oracle(oracle, golden_fft, golden_pwelch):
    for key in golden_fft:
        if key.startswith("fft_in_"):
            n = key[len("fft_in_"):]
            x = golden_fft[key]
            assert nrel(oracle.fft(x), golden_fft[f"fft_out_{n}"]) == 0.0
            assert nrel(oracle.ifft(x), golden_fft[f"ifft_out_{n}"]) == 0.0
    p, _ = oracle.pwelch(golden_pwelch["x"], 1.0, nfft=4096, noverlap=2048)
    assert nrel(p, golden_pwelch["nfft4096_ov2048_pxx"]) == 0.0


def test_pwelch_vs_scipy(oracle):
    ss = pytest.importorskip("scipy.signal")
    rng = np.random.default_rng(3)
    x = rng.standard_normal(20000)
    for nfft, nov in [(256, 128), (1024, 512), (512, 0)]:
        p, f = oracle.pwelch(x, 10.0, nfft=nfft, noverlap=nov)
        fr, pr = ss.welch(x, fs=10.0, window=ss.get_window("hann", nfft, fftbins=False),
                          nperseg=nfft, noverlap=nov, detrend=False, scaling="density")
        assert nrel(p, pr) < 1e-12 and nrel(f, fr) < 1e-15


def test_fill_uniform_range(oracle):
    u = oracle.fill_uniform(100000, 0x5EED)
    assert u.min() >= -1 and u.max() < 1 and abs(u.mean()) < 0.01


@pytest.mark.parametrize("nfft,nov", [(4096, 2048), (256, 0), (1000, 300), (512, -7)])
def test_pwelch_chunked_equals_one_pass(oracle, nfft, nov):
    """The chunked oracle the full-size GPU checks use (segment ranges on
    host threads, combined by segment count) is the one-pass restatement of
    spectral/pwelch.go:74-145 up to the order of the float64 additions."""
    x = oracle.fill_uniform((1 << 20) + 777, 0x5EED)
    a, fa = oracle.pwelch(x, 1.0, nfft=nfft, noverlap=nov)
    b, fb = oracle.pwelch_chunked(x, 1.0, nfft, nov, nthreads=4, chunks=37)
    assert a.size == b.size and np.array_equal(fa, fb)
    assert nrel(b, a) < 1e-13
