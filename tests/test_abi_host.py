"""CPU-only checks of the drop-in boundary and the host logic: the C-ABI
library loads and exports every symbol include/gdsp_fft.h declares, compute
entry points fail loudly without a GPU (no CPU fallback), and the host-side
mirror (windows, dsputils, Segment, Pwelch finalisation) matches the
reference's tables and the oracle."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, nrel


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.strip()}


def test_library_exports_every_header_symbol(gdsp):
    L = gdsp._lib.lib()
    names = gdsp._lib.header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
        assert n in gdsp._lib.SIGNATURES, n


def test_product_library_exports_no_dev_query(gdsp):
    # include/gdsp_fft_dev.h's queries belong to the development build only
    dev_names = gdsp._lib.header_functions(gdsp._lib.DEV_HEADER_PATH)
    assert sorted(dev_names) == sorted(gdsp._lib.DEV_SIGNATURES)
    prod = _exported(os.path.join(REPO, "go-dsp_amd", "lib", "libgdspfft.so"))
    public = {n for n in prod if n.startswith("gdsp_")}
    assert public == set(gdsp._lib.header_functions()), public ^ set(gdsp._lib.header_functions())
    assert not public & set(dev_names)


def test_dev_library_exports_both_headers():
    path = os.path.join(REPO, "go-dsp_amd", "lib_dev", "libgdspfft.so")
    if not os.path.exists(path):
        pytest.skip("development build not built")
    sys.path.insert(0, REPO)
    import importlib
    _lib = importlib.import_module("go-dsp_amd._lib")
    have = _exported(path)
    for n in _lib.header_functions() + _lib.header_functions(_lib.DEV_HEADER_PATH):
        assert n in have, n


def test_version_and_status_strings(gdsp):
    L = gdsp._lib.lib()
    assert b"gfx950" in L.gdsp_version()
    assert L.gdsp_status_string(2) == b"arrays not of equal size"
    assert L.gdsp_status_string(3) == b"empty input array"
    assert L.gdsp_status_string(4) == b"ragged input array"


def test_no_cpu_fallback_without_gpu(gdsp):
    if gdsp.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(gdsp.GDSPError) as e:
        gdsp.fft.FFT(np.arange(8.0))
    assert e.value.status == gdsp._lib.GDSP_ERR_NO_DEVICE
    with pytest.raises(gdsp.GDSPError):
        gdsp.spectral.Pwelch(np.arange(100.0), 1.0, gdsp.spectral.PwelchOptions())


def test_panics_before_device(gdsp):
    with pytest.raises(gdsp.Panic, match="arrays not of equal size"):
        gdsp.fft.Convolve([1, 2], [1])
    with pytest.raises(gdsp.Panic, match="ragged input array"):
        gdsp.fft.FFT2([[1, 2, 3], [1]])
    with pytest.raises(gdsp.Panic, match="empty input array"):
        gdsp.fft.FFT2([])
    with pytest.raises(gdsp.Panic):
        gdsp.fft.IFFT([])
    with pytest.raises(gdsp.Panic):
        gdsp.spectral.Pwelch([1.0, 2.0], 1.0, None)
    with pytest.raises(gdsp.Panic, match="divide by zero"):
        gdsp.spectral.Segment(np.arange(10.0), 4, 4)


def test_segment_tables(gdsp, refvec, oracle):
    x = refvec["segmentTests"]["x"]
    for c in refvec["segmentTests"]["cases"]:
        segs = gdsp.spectral.Segment(x, c["size"], c["noverlap"])
        assert [list(s) for s in segs] == [[float(v) for v in r] for r in c["out"]]
    for lx, size, nov in [(10, 10, 0), (9, 10, 0), (2 ** 30, 4096, 2048), (100, 7, 3)]:
        assert gdsp.spectral.segment_count(lx, size, nov) == oracle.segment_count(lx, size, nov)


@pytest.mark.parametrize("kind", ["Hann", "Hamming", "Bartlett", "FlatTop", "Blackman"])
def test_window_tables(gdsp, refvec, kind):
    f = getattr(gdsp.window, kind)
    for c in refvec["windowTests"]:
        assert gdsp.dsputils.PrettyClose(f(c["L"]), c[kind.lower()])
    o = gdsp.window.Rectangular(10)
    gdsp.window.Apply(o, gdsp.window.Hamming)
    assert gdsp.dsputils.PrettyClose(o, refvec["windowTests"][2]["hamming"])


def test_hann_c_abi_matches_oracle(gdsp, oracle):
    out = np.empty(4096)
    gdsp._lib.check(gdsp._lib.lib().gdsp_window_hann(4096, out.ctypes.data_as(ctypes.c_void_p)))
    assert np.array_equal(out, oracle.window("hann", 4096))
    assert np.array_equal(gdsp.window.Hann(4096), out)


def test_dsputils(gdsp):
    U = gdsp.dsputils
    assert U.IsPowerOf2(0) and U.IsPowerOf2(4096) and not U.IsPowerOf2(3000)
    assert U.NextPowerOf2(5999) == 8192 and U.NextPowerOf2(4096) == 4096
    assert list(U.ZeroPadF([1, 2], 4)) == [1, 2, 0, 0]
    assert U.ZeroPad2([1, 2, 3]).size == 4
    assert U.Float64Equal(1.0, 1.0 + 5e-9) and not U.Float64Equal(1.0, 1.1)


def test_pwelch_finalize_host(gdsp, oracle):
    # finalisation on the host from accumulators built on the CPU: the unpacked
    # per-segment |X_k|^2 sums (what the materialised GPU path accumulates)
    rng = np.random.default_rng(1)
    x = rng.standard_normal(3000)
    nfft, nov = 256, 128
    nseg = oracle.segment_count(x.size, nfft, nov)
    w = oracle.window("hann", nfft)
    acc = np.zeros(nfft)
    for s in range(nseg):
        X = oracle.fft_real(x[s * 128:s * 128 + nfft] * w)
        acc += np.abs(X) ** 2
    p, f = gdsp.spectral.finalize(acc, nseg, nfft, nfft, w, 4.0, False)
    pr, fr = oracle.pwelch(x, 4.0, nfft=nfft, noverlap=nov)
    assert nrel(p, pr) < 1e-12 and np.array_equal(f, fr)


def test_worker_pool_size_recorded(gdsp):
    gdsp.fft.SetWorkerPoolSize(-3)
    assert gdsp._lib.lib().gdsp_worker_pool_size() == 0
    gdsp.fft.SetWorkerPoolSize(4)
    assert gdsp._lib.lib().gdsp_worker_pool_size() == 4


def test_matrix_reference_table(gdsp):
    # dsputils/matrix_test.go:23-47 (TestMakeMatrix)
    U = gdsp.dsputils
    m = U.MakeMatrix([1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 4, 3, 2, 1],
                     [2, 3, 4])
    assert U.PrettyCloseC(m.Dim([1, 0, -1]), U.ToComplex([3, 4, 5, 6]))
    assert U.PrettyCloseC(m.Dim([0, -1, 2]), U.ToComplex([3, 7, 1]))
    assert U.PrettyCloseC(m.Dim([-1, 1, 3]), U.ToComplex([8, 0]))
    s = U.ToComplex([10, 11, 12])
    i = [1, -1, 3]
    m.SetDim(s, i)
    assert U.PrettyCloseC(m.Dim(i), s)
    m.SetValue(14 + 0j, i)
    assert U.ComplexEqual(m.Value(i), 14 + 0j)
    with pytest.raises(gdsp.Panic):
        U.MakeMatrix([1, 2, 3], [2, 2])
    with pytest.raises(gdsp.Panic):
        U.MakeMatrix([], [0])
    with pytest.raises(gdsp.Panic):
        m.Dim([-1, -1, 0])
    assert [list(r) for r in U.MakeMatrix2([[1, 2], [3, 4]]).To2D()] == [[1, 2], [3, 4]]


def test_dsputils_segment_reference_table(gdsp, refvec):
    # dsputils/dsputils_test.go:41-58 (TestSegment)
    U = gdsp.dsputils
    x = np.arange(16, dtype=np.float64).astype(np.complex128)
    for c in refvec["dsputilsSegmentTests"]:
        v = U.Segment(x, c["segs"], c["noverlap"])
        want = [x[a:b] for a, b in c["slices"]]
        assert U.PrettyClose2(v, want)
    # longest length that fits, trailing entries dropped; and the panic
    v = U.Segment(np.arange(10), 4, 0.0)
    assert [list(s) for s in v] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    v = U.Segment(np.arange(10), 2, 0.25)
    assert [len(s) for s in v] == [5, 5]  # 2*(6-1)+1 = 11 > 10, so length 5, overlap 1
    assert list(v[1]) == [4, 5, 6, 7, 8]
    with pytest.raises(gdsp.Panic, match="too many segments"):
        U.Segment(np.arange(3), 4, 0.0)


def test_ensure_radix2_factors_without_gpu(gdsp):
    """fft.EnsureRadix2Factors (radix2.go:35-37) builds a device plan: without a
    GPU it fails loudly; a negative length is rejected before any device."""
    with pytest.raises(gdsp.GDSPError) as e:
        gdsp.fft.EnsureRadix2Factors(-1)
    assert e.value.status == gdsp._lib.GDSP_ERR_INVALID
    if gdsp.device_count() == 0:
        with pytest.raises(gdsp.GDSPError) as e:
            gdsp.fft.EnsureRadix2Factors(4096)
        assert e.value.status == gdsp._lib.GDSP_ERR_NO_DEVICE


def test_ifft2_of_empty_rows_panics(gdsp):
    """computeFFT2 on rows x 0: FFT2 returns the empty rows; IFFT2 calls IFFT
    on an empty row, which panics (fft/fft.go:40, :149-151)."""
    L = gdsp._lib.lib()
    buf = np.zeros(2)
    p = buf.ctypes.data_as(gdsp._lib._P)
    assert L.gdsp_fft2(p, p, 3, 0, 0) == gdsp._lib.GDSP_OK
    assert L.gdsp_fft2(p, p, 3, 0, 1) == gdsp._lib.GDSP_ERR_EMPTY
    assert L.gdsp_fft2_real(p, p, 3, 0, 1) == gdsp._lib.GDSP_ERR_EMPTY


def test_algorithm_selection_flags(gdsp):
    """gdsp_set_algorithm: known flags are kept, unknown bits are rejected and
    leave the selection unchanged (no device needed)."""
    F = gdsp.fft
    prev = F.Algorithm()
    try:
        F.SetAlgorithm(F.ALGO_GENERIC_MIXED | F.ALGO_CHIRPZ_POW2)
        assert F.Algorithm() == F.ALGO_GENERIC_MIXED | F.ALGO_CHIRPZ_POW2
        with pytest.raises(gdsp.GDSPError) as e:
            F.SetAlgorithm(1 << 20)
        assert e.value.status == gdsp._lib.GDSP_ERR_INVALID
        assert F.Algorithm() == F.ALGO_GENERIC_MIXED | F.ALGO_CHIRPZ_POW2
        F.SetAlgorithm(F.ALGO_DEFAULT)
        assert F.Algorithm() == 0
    finally:
        F.SetAlgorithm(prev)


def test_multi_stats_readable_without_gpu(gdsp):
    """gdsp_multi_stats reads the split-call counters; without a GPU no call
    can have been split."""
    s = gdsp.fft.MultiStats()
    assert set(s) == {"batch_calls", "pwelch_calls", "rccl_reduces", "host_reduces"}
    assert all(v >= 0 for v in s.values())
    if gdsp.device_count() == 0:
        assert all(v == 0 for v in s.values())


def _lib_sym(name, restype, argtypes):
    lib = ctypes.CDLL(os.path.join(REPO, "go-dsp_amd", "lib", "libgdspfft.so"))
    f = lib[name]
    f.restype, f.argtypes = restype, argtypes
    return f


def test_chirpz_convolution_length_rule():
    """The fused chirp-z's convolution length (gdsp::chirpz6k_m, host logic, no
    GPU): for every 1 <= n <= 16384, the smallest kept M = 256 RB (three-pass)
    or 256 R1 R2 (four-pass) >= 2n - 1, not above NextPowerOf2(2n - 1)
    (bluestein.go:70), from n = 129 on; else 0 (the power-of-2 kernels). The
    radices chirpz6k_radices reports multiply to M."""
    m_of = _lib_sym("_ZN4gdsp10chirpz6k_mEl", ctypes.c_int, [ctypes.c_int64])
    rad_of = _lib_sym("_ZN4gdsp16chirpz6k_radicesElPi", ctypes.c_int,
                      [ctypes.c_int64, ctypes.POINTER(ctypes.c_int)])
    rb3 = [3, 4, 5, 6, 9, 10, 12, 13, 14, 15, 16, 18, 20, 21, 24, 25]
    rr4 = [(6, 6), (8, 5), (8, 6)]
    for n in range(1, 16385):
        p2 = 1 << (2 * n - 2).bit_length() if n > 1 else 1
        cand = [256 * r for r in rb3 if 256 * r >= 2 * n - 1][:1] + \
               [256 * a * b for a, b in rr4 if 256 * a * b >= 2 * n - 1][:1]
        want = min(cand) if n >= 129 and cand and min(cand) <= p2 else 0
        got = m_of(n)
        assert got == want, (n, got, want)
        if got:
            r = (ctypes.c_int * 4)()
            k = rad_of(got, r)
            assert k in (3, 4) and r[0] == 16 and r[k - 1] == 16, (n, list(r[:k]))
            assert int(np.prod(r[:k])) == got
            assert got >= 2 * n  # n <= M/2: the kernels' KN = 8 input / output registers


def test_smooth_l_candidates_of_the_gpu_tests():
    """gdsp::blufix_length (the lane-cost model's smooth L, host logic): the
    lengths test_chirpz_smooth_l_vs_oracle (-m gpu) runs have a candidate below
    the fused kernel's M of radices <= 16, and the lengths the four-pass kernel
    took from it (4099, 4402) have none."""
    m_of = _lib_sym("_ZN4gdsp10chirpz6k_mEl", ctypes.c_int, [ctypes.c_int64])
    rad_of = _lib_sym("_ZN4gdsp16chirpz6k_radicesElPi", ctypes.c_int,
                      [ctypes.c_int64, ctypes.POINTER(ctypes.c_int)])
    IP = ctypes.POINTER(ctypes.c_int)
    bl = _lib_sym("_ZN4gdsp13blufix_lengthEllPKiiPiS2_", ctypes.c_int,
                  [ctypes.c_int64, ctypes.c_int64, IP, ctypes.c_int, IP, IP])

    def candidate(n):
        m = m_of(n)
        r = (ctypes.c_int * 4)()
        k = rad_of(m, r)
        rad, np_ = (ctypes.c_int * 4)(), ctypes.c_int(0)
        L = bl(n, m, r, k, rad, ctypes.byref(np_))
        return m, L, list(rad[:np_.value])

    for n in (1031, 5209, 5402, 5519):
        m, L, rad = candidate(n)
        assert 2 * n - 1 <= L < m and int(np.prod(rad)) == L and max(rad) <= 16, (n, m, L, rad)
    for n in (4099, 4402):
        assert candidate(n)[1] == 0
