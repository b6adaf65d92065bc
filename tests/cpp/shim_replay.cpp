// shim_replay.cpp — the cgo shim (go/fft/fft_gpu.go, go/spectral/pwelch_gpu.go,
// go/wav/wav_gpu.go) replayed call for call in C++, because no Go toolchain
// exists on either box. Each goshim:: function below is its Go namesake
// transcribed: the same C-ABI calls with the same arguments in the same
// order, the same flattening of [][]complex128 and dsputils.Matrix, the same
// status -> panic mapping (a GoPanic exception carrying the string the Go
// panic would carry). Like the shim, no goshim:: function computes a
// transform on the host: every n, down to 1, goes through the C ABI (the
// oracle, oracle/oracle.c, is only the checker below).
//
// Checks: every shim function against the oracle on the GPU, the reference's
// own tables (fft_test.go, pwelch_test.go; argv[1], written by
// tests/test_cpp_mirror.py) and every panic. Exit 0 = all pass.
#include <array>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "gdsp_fft.h"
#include "oracle.h"

using complex128 = std::complex<double>;

// ---- the Go runtime's behaviour the shim relies on ---------------------------

struct GoPanic : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// x[0] on an empty slice (the reference's IFFT, fft.go:40)
template <class T>
static void index0(const std::vector<T> &x) {
  if (x.empty()) throw GoPanic("runtime error: index out of range [0] with length 0");
}

namespace goshim {

// ---- go/fft/fft_gpu.go --------------------------------------------------------

static void check(int st) {
  switch (st) {
    case GDSP_OK:
      return;
    case GDSP_ERR_UNEQUAL:
    case GDSP_ERR_EMPTY:
    case GDSP_ERR_RAGGED:
    case GDSP_ERR_DIVIDE_BY_ZERO:
      throw GoPanic(gdsp_status_string(st));
  }
  throw GoPanic(std::string("gdspfft: ") + gdsp_status_string(st) + ": " + gdsp_last_error());
}

static double *cplx(std::vector<complex128> &x) {
  return x.empty() ? nullptr : reinterpret_cast<double *>(x.data());
}
static const double *cplx(const std::vector<complex128> &x) {
  return x.empty() ? nullptr : reinterpret_cast<const double *>(x.data());
}
static const double *real64(const std::vector<double> &x) { return x.empty() ? nullptr : x.data(); }

static std::vector<complex128> ToComplex(const std::vector<double> &x) {
  return std::vector<complex128>(x.begin(), x.end());
}

std::vector<complex128> FFT(const std::vector<complex128> &x) {
  std::vector<complex128> r(x.size());
  check(gdsp_fft(cplx(x), cplx(r), (int64_t)x.size()));
  return r;
}

std::vector<complex128> IFFT(const std::vector<complex128> &x) {
  index0(x);
  const size_t n = x.size();
  std::vector<complex128> r(n);
  check(gdsp_ifft(cplx(x), cplx(r), (int64_t)n));
  return r;
}

std::vector<complex128> FFTReal(const std::vector<double> &x) {
  std::vector<complex128> r(x.size());
  check(gdsp_fft_real(real64(x), cplx(r), (int64_t)x.size()));
  return r;
}

std::vector<complex128> IFFTReal(const std::vector<double> &x) {
  index0(x);
  std::vector<complex128> r(x.size());
  check(gdsp_ifft_real(real64(x), cplx(r), (int64_t)x.size()));
  return r;
}

std::vector<complex128> Convolve(const std::vector<complex128> &x, const std::vector<complex128> &y) {
  if (x.size() != y.size()) throw GoPanic("arrays not of equal size");
  std::vector<complex128> r(x.size());
  check(gdsp_convolve(cplx(x), cplx(y), cplx(r), (int64_t)x.size()));
  return r;
}

using Rows = std::vector<std::vector<complex128>>;
using RealRows = std::vector<std::vector<double>>;

template <class R>
static void rows2D(const R &x, int64_t &rows, int64_t &cols) {
  if (x.empty()) throw GoPanic("empty input array");
  rows = (int64_t)x.size();
  cols = (int64_t)x[0].size();
  for (size_t i = 1; i < x.size(); ++i)
    if ((int64_t)x[i].size() != cols) throw GoPanic("ragged input array");
}

static Rows split2D(const std::vector<complex128> &flat, int64_t rows, int64_t cols) {
  Rows r((size_t)rows);
  for (int64_t i = 0; i < rows; ++i)
    r[(size_t)i].assign(flat.begin() + i * cols, flat.begin() + (i + 1) * cols);
  return r;
}

static Rows fft2(const Rows &x, int inverse) {
  int64_t rows, cols;
  rows2D(x, rows, cols);
  std::vector<complex128> flat((size_t)(rows * cols));
  for (int64_t i = 0; i < rows; ++i)
    std::copy(x[(size_t)i].begin(), x[(size_t)i].end(), flat.begin() + i * cols);
  std::vector<complex128> out(flat.size());
  check(gdsp_fft2(cplx(flat), cplx(out), rows, cols, inverse));
  return split2D(out, rows, cols);
}

static Rows fft2Real(const RealRows &x, int inverse) {
  int64_t rows, cols;
  rows2D(x, rows, cols);
  std::vector<double> flat((size_t)(rows * cols));
  for (int64_t i = 0; i < rows; ++i)
    std::copy(x[(size_t)i].begin(), x[(size_t)i].end(), flat.begin() + i * cols);
  std::vector<complex128> out(flat.size());
  check(gdsp_fft2_real(real64(flat), cplx(out), rows, cols, inverse));
  return split2D(out, rows, cols);
}

Rows FFT2(const Rows &x) { return fft2(x, 0); }
Rows IFFT2(const Rows &x) { return fft2(x, 1); }
Rows FFT2Real(const RealRows &x) { return fft2Real(x, 0); }
Rows IFFT2Real(const RealRows &x) { return fft2Real(x, 1); }

// dsputils.Matrix as the shim sees it: dims + the public Value(idx) accessor
struct Matrix {
  std::vector<int> dims;
  std::vector<complex128> list;  // row-major (matrix.go:37-57)
  complex128 Value(const std::vector<int> &idx) const {
    size_t off = 0;
    for (size_t d = 0; d < dims.size(); ++d) off = off * (size_t)dims[d] + (size_t)idx[d];
    return list[off];
  }
};

static Matrix fftn(const Matrix &m, int inverse) {
  const auto &dims = m.dims;
  std::vector<int64_t> cdims(dims.size());
  size_t n = 1;
  for (size_t i = 0; i < dims.size(); ++i) {
    cdims[i] = dims[i];
    n *= (size_t)dims[i];
  }
  std::vector<complex128> flat(n);
  std::vector<int> idx(dims.size(), 0);
  for (size_t i = 0; i < n; ++i) {
    flat[i] = m.Value(idx);
    for (int d = (int)dims.size() - 1; d >= 0; --d) {
      if (++idx[(size_t)d] < dims[(size_t)d]) break;
      idx[(size_t)d] = 0;
    }
  }
  std::vector<complex128> out(n);
  check(gdsp_fftn(cplx(flat), cplx(out), cdims.data(), (int)dims.size(), inverse));
  return Matrix{dims, out};
}

Matrix FFTN(const Matrix &m) { return fftn(m, 0); }
Matrix IFFTN(const Matrix &m) { return fftn(m, 1); }

void SetWorkerPoolSize(int n) { gdsp_set_worker_pool_size(n < 0 ? 0 : n); }
void EnsurePlan(int input_len) { check(gdsp_ensure_plan(input_len)); }
void EnsureRadix2Factors(int input_len) { EnsurePlan(input_len); }
unsigned reverseBits(unsigned v, unsigned s) {  // fft_gpu.go's, for fft_test.go:242-247
  unsigned r = 0;
  for (unsigned i = 0; i < s; ++i) r = r << 1 | ((v >> i) & 1u);
  return r;
}

std::vector<complex128> FFTBatch(const std::vector<complex128> &x, int n, bool inverse) {
  if (n <= 0 || x.size() % (size_t)n != 0) throw GoPanic("arrays not of equal size");
  std::vector<complex128> r(x.size());
  check(gdsp_fft_batch(cplx(x), cplx(r), n, (int64_t)(x.size() / (size_t)n), inverse ? 1 : 0));
  return r;
}

std::vector<complex128> FFTRealBatch(const std::vector<double> &x, int n) {
  if (n <= 0 || x.size() % (size_t)n != 0) throw GoPanic("arrays not of equal size");
  std::vector<complex128> r(x.size());
  check(gdsp_fft_real_batch(real64(x), cplx(r), n, (int64_t)(x.size() / (size_t)n)));
  return r;
}

void SetDevices(const std::vector<int> &ids) {
  std::vector<int> c(ids.begin(), ids.end());
  check(gdsp_set_devices(c.empty() ? nullptr : c.data(), (int)c.size()));
}

std::vector<complex128> FFTBatchMulti(const std::vector<complex128> &x, int n, bool inverse) {
  if (n <= 0 || x.size() % (size_t)n != 0) throw GoPanic("arrays not of equal size");
  std::vector<complex128> r(x.size());
  check(gdsp_fft_batch_multi(cplx(x), cplx(r), n, (int64_t)(x.size() / (size_t)n),
                             inverse ? 1 : 0, nullptr, 0));
  return r;
}

// ---- go/spectral/pwelch_gpu.go ------------------------------------------------

using WindowFunc = std::function<std::vector<double>(int)>;

std::vector<double> Hann(int L) {  // window.Hann (window.go:62-76) as the shim's default
  std::vector<double> r((size_t)L);
  if (or_window(OR_WIN_HANN, L, r.data()) != OR_OK) throw std::runtime_error("or_window");
  return r;
}

struct PwelchOptions {
  int NFFT = 0;
  WindowFunc Window;
  int Pad = 0;
  int Noverlap = 0;
  bool Scale_off = false;
};

void Pwelch(const std::vector<double> &x, double Fs, const PwelchOptions *o,
            std::vector<double> &Pxx, std::vector<double> &freqs) {
  if (x.empty()) {
    Pxx.clear();
    freqs.clear();
    return;
  }
  if (!o) throw GoPanic("runtime error: invalid memory address or nil pointer dereference");
  int nfft = o->NFFT, pad = o->Pad;
  WindowFunc wf = o->Window;
  if (nfft == 0) nfft = 256;
  if (!wf) wf = Hann;
  if (pad == 0) pad = nfft;
  const int flen = pad > nfft ? pad : nfft;
  const auto wseg = wf(flen), wnfft = wf(nfft);
  const int lp = pad / 2 + 1;
  Pxx.assign((size_t)lp, 0.0);
  freqs.assign((size_t)lp, 0.0);
  int64_t got = 0;
  const int st = gdsp_pwelch(x.data(), (int64_t)x.size(), Fs, nfft, pad, o->Noverlap, wseg.data(),
                             wnfft.data(), o->Scale_off ? 1 : 0, Pxx.data(), freqs.data(), &got);
  switch (st) {
    case GDSP_OK:
      break;
    case GDSP_ERR_DIVIDE_BY_ZERO:
      throw GoPanic(gdsp_status_string(st));
    case GDSP_ERR_INVALID:
      throw GoPanic(gdsp_last_error());
    default:
      throw GoPanic(std::string("gdspfft: ") + gdsp_status_string(st) + ": " + gdsp_last_error());
  }
  Pxx.resize((size_t)got);
  freqs.resize((size_t)got);
}

// ---- go/wav/wav_gpu.go (the conversion of (*Wav).ReadFloats) ---------------------

// w.AudioFormat / w.BitsPerSample / the raw bytes io.ReadFull returned
std::vector<float> ReadFloats(int audio_format, int bits, const std::vector<uint8_t> &raw, int n,
                              std::string *err) {
  int size = 0;
  if (audio_format == 1) {
    if (bits == 8 || bits == 16) size = bits / 8;
    else {
      *err = "wav: unknown bits per sample: " + std::to_string(bits);
      return {};
    }
  } else if (audio_format == 3) {
    size = 4;
  } else {
    *err = "wav: unknown audio format";
    return {};
  }
  if (raw.size() < (size_t)n * (size_t)size) {
    *err = "unexpected EOF";
    return {};
  }
  std::vector<float> f((size_t)n);
  if (n == 0) return f;
  const int st = gdsp_wav_read_floats(raw.data(), n, audio_format, bits, f.data(), 0);
  if (st != GDSP_OK)
    throw GoPanic(std::string("gdspfft: ") + gdsp_status_string(st) + ": " + gdsp_last_error());
  return f;
}

}  // namespace goshim

// ==============================================================================
// checks
// ==============================================================================

static int failures = 0, checks = 0;
#define EXPECT(cond, what)                                   \
  do {                                                       \
    ++checks;                                                \
    if (!(cond)) {                                           \
      ++failures;                                            \
      std::cerr << "FAIL " << what << " (" #cond ")\n";      \
    }                                                        \
  } while (0)

template <class F>
static std::string panics(F f) {
  try {
    f();
  } catch (const GoPanic &p) {
    return p.what();
  }
  return "";
}

static double nrel(const std::vector<complex128> &a, const std::vector<complex128> &b) {
  double num = 0, den = 0;
  if (a.size() != b.size()) return 1e300;
  for (size_t i = 0; i < a.size(); ++i) {
    num += std::norm(a[i] - b[i]);
    den += std::norm(b[i]);
  }
  return den == 0 ? std::sqrt(num) : std::sqrt(num / den);
}
static double nrel(const std::vector<double> &a, const std::vector<double> &b) {
  double num = 0, den = 0;
  if (a.size() != b.size()) return 1e300;
  for (size_t i = 0; i < a.size(); ++i) {
    num += (a[i] - b[i]) * (a[i] - b[i]);
    den += b[i] * b[i];
  }
  return den == 0 ? std::sqrt(num) : std::sqrt(num / den);
}
static bool f64eq(double a, double b) {  // dsputils.Float64Equal, compare.go:94-96
  return std::fabs(a - b) <= 1e-8 || std::fabs(1 - a / b) <= 1e-8;
}
static bool close_c(const std::vector<complex128> &a, const std::vector<complex128> &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!f64eq(a[i].real(), b[i].real()) || !f64eq(a[i].imag(), b[i].imag())) return false;
  return true;
}

static std::vector<complex128> randc(size_t n, uint64_t seed) {
  std::vector<double> d(2 * n);
  or_fill_uniform(d.data(), (int64_t)d.size(), seed, 0);
  std::vector<complex128> r(n);
  for (size_t i = 0; i < n; ++i) r[i] = {d[2 * i], d[2 * i + 1]};
  return r;
}
static std::vector<double> randr(size_t n, uint64_t seed) {
  std::vector<double> d(n);
  or_fill_uniform(d.data(), (int64_t)n, seed, 0);
  return d;
}
static std::vector<complex128> oracle1(const std::vector<complex128> &x, bool inv) {
  std::vector<complex128> r(x.size());
  (inv ? or_ifft : or_fft)(reinterpret_cast<const double *>(x.data()),
                           reinterpret_cast<double *>(r.data()), (int64_t)x.size());
  return r;
}

static std::vector<double> readd(std::istream &in, size_t n) {
  std::vector<double> v(n);
  for (auto &x : v) in >> x;
  return v;
}
static std::vector<complex128> readc(std::istream &in, size_t n) {
  std::vector<complex128> v(n);
  for (auto &x : v) {
    double a, b;
    in >> a >> b;
    x = {a, b};
  }
  return v;
}

static void reference_tables(const char *path) {
  // fft_test.go / pwelch_test.go tables
  {
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream in(line);
      std::string kind;
      in >> kind;
      if (kind == "FFT") {  // TestFFT, fft_test.go:197-209
        size_t n;
        in >> n;
        auto x = readd(in, n);
        auto out = readc(in, n);
        EXPECT(close_c(goshim::FFTReal(x), out), "FFTReal n=" << n);
        EXPECT(close_c(goshim::IFFT(out), goshim::ToComplex(x)), "IFFT n=" << n);
      } else if (kind == "FFT2") {  // TestFFT2, fft_test.go:211-223
        size_t r, c;
        in >> r >> c;
        goshim::RealRows x(r);
        for (auto &row : x) row = readd(in, c);
        goshim::Rows out(r);
        for (auto &row : out) row = readc(in, c);
        auto got = goshim::FFT2Real(x);
        bool ok = got.size() == r;
        for (size_t i = 0; ok && i < r; ++i) ok = close_c(got[i], out[i]);
        EXPECT(ok, "FFT2Real " << r << "x" << c);
        auto back = goshim::IFFT2(out);
        ok = back.size() == r;
        for (size_t i = 0; ok && i < r; ++i) ok = close_c(back[i], goshim::ToComplex(x[i]));
        EXPECT(ok, "IFFT2 " << r << "x" << c);
      } else if (kind == "FFTN") {  // TestFFTN, fft_test.go:225-239
        size_t nd;
        in >> nd;
        std::vector<int> dims(nd);
        size_t n = 1;
        for (auto &d : dims) {
          in >> d;
          n *= (size_t)d;
        }
        auto x = readd(in, n);
        auto out = readc(in, n);
        goshim::Matrix m{dims, goshim::ToComplex(x)};
        EXPECT(close_c(goshim::FFTN(m).list, out), "FFTN");
        EXPECT(close_c(goshim::IFFTN(goshim::Matrix{dims, out}).list, goshim::ToComplex(x)),
               "IFFTN");
      } else if (kind == "PWELCH") {  // TestPwelch, pwelch_test.go:48-60
        double fs;
        size_t n, lp;
        in >> fs >> n;
        auto x = readd(in, n);
        in >> lp;
        auto p = readd(in, lp), fr = readd(in, lp);
        std::vector<double> gp, gf;
        goshim::PwelchOptions o;
        goshim::Pwelch(x, fs, &o, gp, gf);
        bool ok = gp.size() == lp && gf.size() == lp;
        for (size_t i = 0; ok && i < lp; ++i) ok = f64eq(gp[i], p[i]) && f64eq(gf[i], fr[i]);
        EXPECT(ok, "Pwelch table");
      }
    }
  }
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::cerr << "usage: shim_replay vectors.txt\n";
    return 2;
  }
  reference_tables(argv[1]);

  // FFT / IFFT / FFTReal / IFFTReal / Convolve at every kind of length (all
  // on the GPU: the shim has no host transform), against the restatement of
  // the reference
  for (size_t n : {1ul, 2ul, 5ul, 1000ul, 1024ul, 1025ul, 1500ul, 2048ul, 3000ul, 4095ul, 4096ul,
                   5000ul, 65536ul}) {
    auto x = randc(n, 100 + n);
    EXPECT(nrel(goshim::FFT(x), oracle1(x, false)) < 1e-9, "FFT n=" << n);
    EXPECT(nrel(goshim::IFFT(x), oracle1(x, true)) < 1e-9, "IFFT n=" << n);
    auto xr = randr(n, 200 + n);
    auto want = oracle1(goshim::ToComplex(xr), false);
    EXPECT(nrel(goshim::FFTReal(xr), want) < 1e-9, "FFTReal n=" << n);
    EXPECT(nrel(goshim::IFFTReal(xr), oracle1(goshim::ToComplex(xr), true)) < 1e-9,
           "IFFTReal n=" << n);
    auto y = randc(n, 300 + n);
    std::vector<complex128> cv(n);
    or_convolve(reinterpret_cast<const double *>(x.data()),
                reinterpret_cast<const double *>(y.data()), reinterpret_cast<double *>(cv.data()),
                (int64_t)n);
    EXPECT(nrel(goshim::Convolve(x, y), cv) < 1e-9, "Convolve n=" << n);
  }
  // the input is never modified (fft.go:76-80, radix2.go:84-85)
  {
    auto x = randc(8192, 7), keep = x;
    (void)goshim::FFT(x);
    (void)goshim::IFFT(x);
    EXPECT(x == keep, "FFT/IFFT leave x untouched");
  }
  // panics
  EXPECT(panics([] { goshim::IFFT({}); }).find("index out of range") != std::string::npos,
         "IFFT([]) panics");
  EXPECT(panics([] { goshim::IFFTReal({}); }).find("index out of range") != std::string::npos,
         "IFFTReal([]) panics");
  EXPECT(goshim::FFT({}).empty() && panics([] { goshim::FFT({}); }).empty(), "FFT([]) is []");
  EXPECT(panics([] { goshim::Convolve({1.0, 2.0}, {1.0}); }) == "arrays not of equal size",
         "Convolve unequal");
  EXPECT(panics([] { goshim::FFT2({}); }) == "empty input array", "FFT2 empty");
  EXPECT(panics([] { goshim::FFT2({{1.0, 2.0, 3.0}, {1.0}}); }) == "ragged input array",
         "FFT2 ragged");
  EXPECT(panics([] { goshim::FFT2Real({{1.0, 2.0}, {1.0}}); }) == "ragged input array",
         "FFT2Real ragged");
  EXPECT(panics([] { goshim::FFTBatch(std::vector<complex128>(10), 4, false); }) ==
             "arrays not of equal size",
         "FFTBatch ragged");

  // FFT2 family against the restatement (computeFFT2: columns, then rows)
  for (auto rc : {std::pair<int, int>{64, 100}, {3000, 7}, {8, 4096}}) {
    const int r = rc.first, c = rc.second;
    auto flat = randc((size_t)r * c, 400 + r);
    goshim::Rows x((size_t)r);
    for (int i = 0; i < r; ++i) x[(size_t)i].assign(flat.begin() + i * c, flat.begin() + (i + 1) * c);
    for (int inv = 0; inv < 2; ++inv) {
      std::vector<complex128> want(flat.size());
      or_fft2(reinterpret_cast<const double *>(flat.data()), reinterpret_cast<double *>(want.data()),
              r, c, inv);
      auto got = inv ? goshim::IFFT2(x) : goshim::FFT2(x);
      std::vector<complex128> g;
      for (auto &row : got) g.insert(g.end(), row.begin(), row.end());
      EXPECT(nrel(g, want) < 1e-9, "FFT2 " << r << "x" << c << " inv=" << inv);
    }
    goshim::RealRows xr((size_t)r);
    auto fr = randr((size_t)r * c, 500 + r);
    for (int i = 0; i < r; ++i) xr[(size_t)i].assign(fr.begin() + i * c, fr.begin() + (i + 1) * c);
    std::vector<complex128> frc(fr.begin(), fr.end()), want(fr.size());
    or_fft2(reinterpret_cast<const double *>(frc.data()), reinterpret_cast<double *>(want.data()), r,
            c, 0);
    std::vector<complex128> g;
    for (auto &row : goshim::FFT2Real(xr)) g.insert(g.end(), row.begin(), row.end());
    EXPECT(nrel(g, want) < 1e-9, "FFT2Real " << r << "x" << c);
  }
  // FFTN through the Matrix flattening
  for (auto dims : {std::vector<int>{4, 6, 5}, std::vector<int>{2, 3, 3000}, std::vector<int>{7}}) {
    size_t n = 1;
    for (int d : dims) n *= (size_t)d;
    goshim::Matrix m{dims, randc(n, 600 + n)};
    std::vector<int64_t> cd(dims.begin(), dims.end());
    for (int inv = 0; inv < 2; ++inv) {
      std::vector<complex128> want(n);
      or_fftn(reinterpret_cast<const double *>(m.list.data()),
              reinterpret_cast<double *>(want.data()), cd.data(), (int)cd.size(), inv);
      auto got = inv ? goshim::IFFTN(m) : goshim::FFTN(m);
      EXPECT(got.dims == dims && nrel(got.list, want) < 1e-9, "FFTN dims " << dims.size()
                                                                            << " inv=" << inv);
    }
  }
  // batched entries
  {
    const int n = 4096, b = 33;
    auto x = randc((size_t)n * b, 9);
    auto y = goshim::FFTBatch(x, n, false);
    auto z = goshim::FFTBatchMulti(x, n, true);
    auto xr = randr((size_t)n * b, 10);
    auto yr = goshim::FFTRealBatch(xr, n);
    double e = 0, ei = 0, er = 0;
    for (int r = 0; r < b; ++r) {
      std::vector<complex128> row(x.begin() + r * n, x.begin() + (r + 1) * n);
      std::vector<complex128> rr(xr.begin() + r * n, xr.begin() + (r + 1) * n);
      e = std::max(e, nrel({y.begin() + r * n, y.begin() + (r + 1) * n}, oracle1(row, false)));
      ei = std::max(ei, nrel({z.begin() + r * n, z.begin() + (r + 1) * n}, oracle1(row, true)));
      er = std::max(er, nrel({yr.begin() + r * n, yr.begin() + (r + 1) * n}, oracle1(rr, false)));
    }
    EXPECT(e < 1e-9 && ei < 1e-9 && er < 1e-9, "FFTBatch/FFTBatchMulti/FFTRealBatch");
  }
  goshim::EnsurePlan(1 << 20);
  goshim::EnsureRadix2Factors(3000);
  // fft_test.go:183-247 (TestReverseBits) through the shim's helper
  for (auto t : {std::array<unsigned, 3>{0, 1, 0}, {1, 2, 2}, {1, 4, 8}, {2, 4, 4}, {3, 4, 12}})
    EXPECT(goshim::reverseBits(t[0], t[1]) == t[2], "reverseBits " << t[0] << "," << t[1]);
  {
    goshim::SetDevices({0});
    int d[4] = {-1, -1, -1, -1};
    EXPECT(gdsp_get_devices(d, 4) == 1 && d[0] == 0, "SetDevices([0])");
    goshim::SetDevices({});  // back to the calling thread's current device
    EXPECT(panics([] { goshim::SetDevices({999}); }).find("gdspfft:") == 0, "SetDevices bad id");
  }
  goshim::SetWorkerPoolSize(-3);
  EXPECT(gdsp_worker_pool_size() == 0, "SetWorkerPoolSize(-3) records 0");
  goshim::SetWorkerPoolSize(6);
  EXPECT(gdsp_worker_pool_size() == 6, "SetWorkerPoolSize(6)");
  goshim::SetWorkerPoolSize(0);

  // Pwelch: options, windows, the Pad quirk, Scale_off, panics
  {
    auto x = randr(50000, 11);
    struct Case {
      int nfft, pad, nov, win;
      bool scale_off;
    };
    for (Case c : {Case{4096, 0, 2048, OR_WIN_HANN, false}, Case{1000, 2048, 250, OR_WIN_HAMMING, false},
                   Case{1024, 512, 0, OR_WIN_BLACKMAN, true}, Case{0, 0, 0, OR_WIN_HANN, false},
                   Case{3000, 0, 1500, OR_WIN_FLATTOP, true}}) {
      goshim::PwelchOptions o;
      o.NFFT = c.nfft;
      o.Pad = c.pad;
      o.Noverlap = c.nov;
      o.Scale_off = c.scale_off;
      if (c.win != OR_WIN_HANN) {
        const int kind = c.win;
        o.Window = [kind](int L) {
          std::vector<double> w((size_t)L);
          or_window(kind, L, w.data());
          return w;
        };
      }
      std::vector<double> p, f;
      goshim::Pwelch(x, 3.0, &o, p, f);
      const int nfft = c.nfft ? c.nfft : 256, pad = c.pad ? c.pad : nfft;
      std::vector<double> pr((size_t)(pad / 2 + 1)), fr(pr.size());
      int64_t lp = 0;
      or_pwelch(x.data(), (int64_t)x.size(), 3.0, c.nfft, c.pad, c.nov, c.win, c.scale_off ? 1 : 0,
                pr.data(), fr.data(), &lp);
      EXPECT((int64_t)p.size() == lp && nrel(p, pr) < 1e-9 && nrel(f, fr) < 1e-15,
             "Pwelch nfft=" << c.nfft << " pad=" << c.pad << " nov=" << c.nov);
    }
    std::vector<double> p, f;
    goshim::PwelchOptions o;
    goshim::Pwelch({}, 1.0, &o, p, f);
    EXPECT(p.empty() && f.empty(), "Pwelch([]) is empty");
    o.NFFT = 256;
    o.Noverlap = 256;
    EXPECT(panics([&] { goshim::Pwelch(x, 1.0, &o, p, f); }) == "integer divide by zero",
           "Pwelch Noverlap == NFFT");
    o.Noverlap = 300;
    EXPECT(panics([&] { goshim::Pwelch(x, 1.0, &o, p, f); }).find("makeslice") != std::string::npos,
           "Pwelch Noverlap > NFFT");
    EXPECT(!panics([&] { goshim::Pwelch(x, 1.0, nullptr, p, f); }).empty(), "Pwelch nil options");
  }

  // wav ReadFloats conversion: PCM8, PCM16, float32 against the restatement
  {
    std::vector<uint8_t> raw(4 * 3001);
    auto d = randr(raw.size() / 8 + 1, 12);
    std::memcpy(raw.data(), d.data(), raw.size());
    for (auto fb : {std::pair<int, int>{1, 8}, {1, 16}, {3, 32}}) {
      const int n = 3001;
      std::string err;
      auto got = goshim::ReadFloats(fb.first, fb.second, raw, n, &err);
      std::vector<float> want((size_t)n);
      or_wav_floats(raw.data(), n, fb.first, fb.second, want.data());
      bool same = err.empty() && got.size() == want.size();
      for (size_t i = 0; same && i < got.size(); ++i)
        same = std::memcmp(&got[i], &want[i], sizeof(float)) == 0 ||
               (std::isnan(got[i]) && std::isnan(want[i]));
      EXPECT(same, "ReadFloats format " << fb.first << "/" << fb.second << " bit-exact");
    }
    std::string err;
    goshim::ReadFloats(1, 24, raw, 4, &err);
    EXPECT(err == "wav: unknown bits per sample: 24", "ReadFloats PCM24");
    err.clear();
    goshim::ReadFloats(2, 16, raw, 4, &err);
    EXPECT(err == "wav: unknown audio format", "ReadFloats format 2");
  }

  std::cout << "checks " << checks << " failures " << failures << "\n";
  return failures ? 1 : 0;
}
