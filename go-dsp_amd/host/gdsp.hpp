// gdsp.hpp — C++17 host mirror of go-dsp's Go API (packages fft, spectral,
// window, dsputils) over the libgdspfft C ABI (include/gdsp_fft.h).
//
// Same names, argument meaning and error behaviour as the reference: results
// are new vectors, inputs are never modified, and where Go panics this header
// throws gdsp::Panic with the reference's message. Every transform runs on the
// GPU; a missing device surfaces as gdsp::Error (GDSP_ERR_NO_DEVICE).
#pragma once

#include <cmath>
#include <cstdio>
#include <istream>
#include <complex>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "gdsp_fft.h"

namespace gdsp {

struct Error : std::runtime_error {
  int status;
  Error(int st, const std::string &m) : std::runtime_error(m), status(st) {}
};

// Raised where the Go reference panics.
struct Panic : Error {
  using Error::Error;
};

inline void check(int st, const char *what) {
  if (st == GDSP_OK) return;
  const std::string msg = gdsp_status_string(st);
  if (st == GDSP_ERR_UNEQUAL || st == GDSP_ERR_EMPTY || st == GDSP_ERR_RAGGED ||
      st == GDSP_ERR_DIVIDE_BY_ZERO)
    throw Panic(st, msg);
  throw Error(st, std::string(what) + ": " + msg + " (" + gdsp_last_error() + ")");
}

using complex = std::complex<double>;  // layout == Go complex128 == (re, im) doubles

namespace dsputils {  // dsputils/dsputils.go, dsputils/compare.go

constexpr double closeFactor = 1e-8;

inline std::vector<complex> ToComplex(const std::vector<double> &x) {
  return std::vector<complex>(x.begin(), x.end());
}
inline std::vector<std::vector<complex>> ToComplex2(const std::vector<std::vector<double>> &x) {
  std::vector<std::vector<complex>> r;
  for (auto &v : x) r.push_back(ToComplex(v));
  return r;
}
inline bool IsPowerOf2(long long x) { return (x & (x - 1)) == 0; }
inline long long NextPowerOf2(long long x) {
  if (IsPowerOf2(x)) return x;
  return (long long)std::pow(2.0, std::ceil(std::log2((double)x)));
}
inline std::vector<double> ZeroPadF(const std::vector<double> &x, size_t length) {
  if (x.size() >= length) return x;
  std::vector<double> r(length, 0.0);
  std::copy(x.begin(), x.end(), r.begin());
  return r;
}
inline bool Float64Equal(double a, double b) {
  return std::fabs(a - b) <= closeFactor || std::fabs(1 - a / b) <= closeFactor;
}
inline bool ComplexEqual(complex a, complex b) {
  return Float64Equal(a.real(), b.real()) && Float64Equal(a.imag(), b.imag());
}
inline bool PrettyClose(const std::vector<double> &a, const std::vector<double> &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!Float64Equal(a[i], b[i])) return false;
  return true;
}
inline bool PrettyCloseC(const std::vector<complex> &a, const std::vector<complex> &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!ComplexEqual(a[i], b[i])) return false;
  return true;
}
inline bool PrettyClose2(const std::vector<std::vector<complex>> &a,
                         const std::vector<std::vector<complex>> &b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (!PrettyCloseC(a[i], b[i])) return false;
  return true;
}

// dsputils.Segment — dsputils/dsputils.go:89-120: segs equal-length copies
// of x with a fractional overlap (the reference returns slices; a C++ caller
// gets the values). Throws Panic("too many segments") when none fits.
inline std::vector<std::vector<complex>> Segment(const std::vector<complex> &x, int segs,
                                                 double noverlap) {
  const int lx = (int)x.size();
  int length = lx, step = 0;
  for (; length > 0; --length) {
    const int overlap = (int)((double)length * noverlap);
    if (segs * (length - overlap) + overlap <= lx) {
      step = length - overlap;
      break;
    }
  }
  if (length == 0) throw Panic(GDSP_ERR_INVALID, "too many segments");
  std::vector<std::vector<complex>> r((size_t)segs);
  for (int n = 0; n < segs; ++n) r[(size_t)n].assign(x.begin() + n * step, x.begin() + n * step + length);
  return r;
}

// dsputils.Matrix — dsputils/matrix.go:21-216 (row-major N-D complex128).
struct Matrix {
  std::vector<complex> list;
  std::vector<int> dims, offsets;

  int offset(const std::vector<int> &d) const {  // :93-107
    if (d.size() != dims.size()) throw Panic(GDSP_ERR_INVALID, "incorrect dimensions");
    int i = 0;
    for (size_t n = 0; n < d.size(); ++n) {
      if (d[n] > dims[n]) throw Panic(GDSP_ERR_INVALID, "incorrect dimensions");
      i += d[n] * offsets[n];
    }
    return i;
  }
  std::vector<int> indexes(const std::vector<int> &d) const {  // :110-142
    int ax = -1;
    for (size_t n = 0; n < d.size(); ++n) {
      if (d[n] == -1) {
        if (ax >= 0) throw Panic(GDSP_ERR_INVALID, "only one dimension index allowed");
        ax = (int)n;
      } else if (d[n] >= dims[n]) {
        throw Panic(GDSP_ERR_INVALID, "dimension out of bounds");
      }
    }
    if (ax == -1) throw Panic(GDSP_ERR_INVALID, "must specify one dimension index");
    int x = 0;
    for (size_t n = 0; n < d.size(); ++n)
      if (d[n] >= 0) x += offsets[n] * d[n];
    std::vector<int> r(dims[ax]);
    for (int j = 0; j < dims[ax]; ++j) r[j] = x + offsets[ax] * j;
    return r;
  }
  std::vector<int> Dimensions() const { return dims; }
  std::vector<complex> Dim(const std::vector<int> &d) const {
    std::vector<complex> r;
    for (int i : indexes(d)) r.push_back(list[i]);
    return r;
  }
  void SetDim(const std::vector<complex> &x, const std::vector<int> &d) {
    auto inds = indexes(d);
    if (x.size() != inds.size()) throw Panic(GDSP_ERR_INVALID, "incorrect array length");
    for (size_t n = 0; n < inds.size(); ++n) list[inds[n]] = x[n];
  }
  complex Value(const std::vector<int> &d) const { return list[offset(d)]; }
  void SetValue(complex v, const std::vector<int> &d) { list[offset(d)] = v; }
  bool PrettyClose(const Matrix &n) const { return dims == n.dims && PrettyCloseC(list, n.list); }
};

inline Matrix MakeMatrix(const std::vector<complex> &x, const std::vector<int> &dims) {  // :37-57
  Matrix m;
  m.offsets.assign(dims.size(), 0);
  int length = 1;
  for (int i = (int)dims.size() - 1; i >= 0; --i) {
    if (dims[i] < 1) throw Panic(GDSP_ERR_INVALID, "invalid dimensions");
    m.offsets[i] = length;
    length *= dims[i];
  }
  if ((int)x.size() != length) throw Panic(GDSP_ERR_INVALID, "incorrect dimensions");
  m.list = x;
  m.dims = dims;
  return m;
}

}  // namespace dsputils

namespace fft {  // fft/fft.go

using Matrix = std::vector<std::vector<complex>>;

inline const double *cp(const std::vector<complex> &v) {
  return reinterpret_cast<const double *>(v.data());
}
inline double *mp(std::vector<complex> &v) { return reinterpret_cast<double *>(v.data()); }

// fft.FFT — fft/fft.go:72-87
inline std::vector<complex> FFT(const std::vector<complex> &x) {
  std::vector<complex> r(x.size());
  check(gdsp_fft(cp(x), mp(r), (int64_t)x.size()), "FFT");
  return r;
}
// fft.IFFT — fft/fft.go:35-52 (panics on an empty slice)
inline std::vector<complex> IFFT(const std::vector<complex> &x) {
  std::vector<complex> r(x.size());
  check(gdsp_ifft(cp(x), mp(r), (int64_t)x.size()), "IFFT");
  return r;
}
// fft.FFTReal — fft/fft.go:25-27
inline std::vector<complex> FFTReal(const std::vector<double> &x) {
  std::vector<complex> r(x.size());
  check(gdsp_fft_real(x.data(), mp(r), (int64_t)x.size()), "FFTReal");
  return r;
}
// fft.IFFTReal — fft/fft.go:30-32
inline std::vector<complex> IFFTReal(const std::vector<double> &x) {
  std::vector<complex> r(x.size());
  check(gdsp_ifft_real(x.data(), mp(r), (int64_t)x.size()), "IFFTReal");
  return r;
}
// fft.Convolve — fft/fft.go:55-69
inline std::vector<complex> Convolve(const std::vector<complex> &x,
                                     const std::vector<complex> &y) {
  if (x.size() != y.size()) throw Panic(GDSP_ERR_UNEQUAL, "arrays not of equal size");
  std::vector<complex> r(x.size());
  check(gdsp_convolve(cp(x), cp(y), mp(r), (int64_t)x.size()), "Convolve");
  return r;
}

// computeFFT2's checks (fft/fft.go:124-136), then one flattened device call
template <class T>
inline std::vector<T> flatten(const std::vector<std::vector<T>> &x, size_t &cols) {
  if (x.empty()) throw Panic(GDSP_ERR_EMPTY, "empty input array");
  cols = x[0].size();
  std::vector<T> f;
  f.reserve(x.size() * cols);
  for (auto &row : x) {
    if (row.size() != cols) throw Panic(GDSP_ERR_RAGGED, "ragged input array");
    f.insert(f.end(), row.begin(), row.end());
  }
  return f;
}
inline Matrix unflatten(const std::vector<complex> &f, size_t rows, size_t cols) {
  Matrix r(rows);
  for (size_t i = 0; i < rows; ++i) r[i].assign(f.begin() + i * cols, f.begin() + (i + 1) * cols);
  return r;
}
inline Matrix fft2(const Matrix &x, int inverse) {
  size_t cols = 0;
  auto f = flatten(x, cols);
  std::vector<complex> o(f.size());
  check(gdsp_fft2(cp(f), mp(o), (int64_t)x.size(), (int64_t)cols, inverse), "FFT2");
  return unflatten(o, x.size(), cols);
}
inline Matrix fft2_real(const std::vector<std::vector<double>> &x, int inverse) {
  size_t cols = 0;
  auto f = flatten(x, cols);
  std::vector<complex> o(f.size());
  check(gdsp_fft2_real(f.data(), mp(o), (int64_t)x.size(), (int64_t)cols, inverse), "FFT2Real");
  return unflatten(o, x.size(), cols);
}
inline Matrix FFT2(const Matrix &x) { return fft2(x, 0); }                        // fft.go:109
inline Matrix IFFT2(const Matrix &x) { return fft2(x, 1); }                       // fft.go:119
inline Matrix FFT2Real(const std::vector<std::vector<double>> &x) { return fft2_real(x, 0); }   // :104
inline Matrix IFFT2Real(const std::vector<std::vector<double>> &x) { return fft2_real(x, 1); }  // :114

// Additive batched entry point: rows of one flat buffer.
inline std::vector<complex> FFTBatch(const std::vector<complex> &x, size_t n, bool inverse = false) {
  std::vector<complex> r(x.size());
  check(gdsp_fft_batch(cp(x), mp(r), (int64_t)n, n ? (int64_t)(x.size() / n) : 0, inverse),
        "FFTBatch");
  return r;
}

// fft.FFTN / IFFTN — fft.go:157-192
inline dsputils::Matrix fftn(const dsputils::Matrix &m, int inverse) {
  std::vector<int64_t> d(m.dims.begin(), m.dims.end());
  std::vector<complex> o(m.list.size());
  check(gdsp_fftn(cp(m.list), mp(o), d.data(), (int)d.size(), inverse), "FFTN");
  return dsputils::MakeMatrix(o, m.dims);
}
inline dsputils::Matrix FFTN(const dsputils::Matrix &m) { return fftn(m, 0); }
inline dsputils::Matrix IFFTN(const dsputils::Matrix &m) { return fftn(m, 1); }

// Multi-device (gdsp_fft.h "multi-device"): the GPUs large host calls split over.
inline void SetDevices(const std::vector<int> &devices) {
  check(gdsp_set_devices(devices.empty() ? nullptr : devices.data(), (int)devices.size()),
        "SetDevices");
}
inline std::vector<int> Devices() {
  std::vector<int> d((size_t)std::max(gdsp_get_devices(nullptr, 0), 0));
  d.resize((size_t)gdsp_get_devices(d.data(), (int)d.size()));
  return d;
}
// FFTBatch split over `devices` (empty: the device set), one row shard each.
inline std::vector<complex> FFTBatchMulti(const std::vector<complex> &x, size_t n,
                                          bool inverse = false,
                                          const std::vector<int> &devices = {}) {
  std::vector<complex> r(x.size());
  check(gdsp_fft_batch_multi(cp(x), mp(r), (int64_t)n, n ? (int64_t)(x.size() / n) : 0, inverse,
                             devices.empty() ? nullptr : devices.data(), (int)devices.size()),
        "FFTBatchMulti");
  return r;
}

// How the split calls went (gdsp_multi_stats).
struct MultiStats {
  int64_t batch_calls = 0, pwelch_calls = 0, rccl_reduces = 0, host_reduces = 0;
};
inline MultiStats GetMultiStats() {
  MultiStats m;
  check(gdsp_multi_stats(&m.batch_calls, &m.pwelch_calls, &m.rccl_reduces, &m.host_reduces),
        "MultiStats");
  return m;
}

// Algorithm selection (gdsp_fft.h GDSP_ALGO_*; no reference equivalent).
inline void SetAlgorithm(unsigned flags) { check(gdsp_set_algorithm(flags), "SetAlgorithm"); }
inline unsigned Algorithm() { return gdsp_get_algorithm(); }

inline void SetWorkerPoolSize(int n) { gdsp_set_worker_pool_size(n); }  // fft.go:95-101
inline void EnsureRadix2Factors(int input_len) {                        // radix2.go:35-37
  check(gdsp_ensure_plan(input_len), "EnsureRadix2Factors");
}

}  // namespace fft

namespace window {  // window/window.go

using Func = std::function<std::vector<double>(int)>;

inline void Apply(std::vector<double> &x, const Func &wf) {  // :25-29
  auto w = wf((int)x.size());
  for (size_t i = 0; i < w.size(); ++i) x[i] *= w[i];
}
inline std::vector<double> Rectangular(int L) { return std::vector<double>(L, 1.0); }  // :32-40
inline std::vector<double> sym(int L, const std::function<double(int, int)> &f) {
  std::vector<double> r(L > 0 ? L : 0, 0.0);
  if (L == 1) r[0] = 1;
  else
    for (int n = 0; n < L; ++n) r[n] = f(n, L - 1);
  return r;
}
inline std::vector<double> Hamming(int L) {  // :44-58
  return sym(L, [](int n, int N) { return 0.54 - 0.46 * std::cos(M_PI * 2 / N * n); });
}
inline std::vector<double> Hann(int L) {  // :62-76 (same table as gdsp_window_hann)
  std::vector<double> r(L > 0 ? L : 0);
  check(gdsp_window_hann(L, r.data()), "Hann");
  return r;
}
inline std::vector<double> Bartlett(int L) {  // :80-98
  std::vector<double> r(L > 0 ? L : 0, 0.0);
  if (L == 1) {
    r[0] = 1;
  } else if (L > 1) {
    const int N = L - 1;
    const double coef = 2.0 / N;
    int n = 0;
    for (; n <= N / 2; ++n) r[n] = coef * n;
    for (; n <= N; ++n) r[n] = 2 - coef * n;
  }
  return r;
}
inline std::vector<double> FlatTop(int L) {  // :102-135
  return sym(L, [](int n, int N) {
    const double f = n * (2 * M_PI / N);
    return 0.21557895 - 0.41663158 * std::cos(f) + 0.277263158 * std::cos(2 * f) -
           0.083578947 * std::cos(3 * f) + 0.006947368 * std::cos(4 * f);
  });
}
inline std::vector<double> Blackman(int L) {  // :138-152
  return sym(L, [](int n, int N) {
    return 0.42 + (-0.5 * std::cos(2 * M_PI * n / N)) + 0.08 * std::cos(4 * M_PI * n / N);
  });
}

}  // namespace window

namespace spectral {  // spectral/pwelch.go, spectral/spectral.go

struct PwelchOptions {  // pwelch.go:28-65
  int NFFT = 0;
  window::Func Window;  // empty = window.Hann
  int Pad = 0;
  int Noverlap = 0;
  bool Scale_off = false;
};

// spectral.Segment — spectral.go:22-47
inline std::vector<std::vector<double>> Segment(const std::vector<double> &x, int size,
                                                int noverlap) {
  int64_t n = 0;
  check(gdsp_segment_count((int64_t)x.size(), size, noverlap, &n), "Segment");
  std::vector<std::vector<double>> r((size_t)n);
  const int stride = size - noverlap;
  for (int64_t i = 0; i < n; ++i)
    r[(size_t)i].assign(x.begin() + i * stride, x.begin() + i * stride + size);
  return r;
}

// spectral.Pwelch — pwelch.go:74-145. A null options pointer is the
// reference's nil dereference: it throws Panic.
inline std::pair<std::vector<double>, std::vector<double>> Pwelch(const std::vector<double> &x,
                                                                  double Fs,
                                                                  const PwelchOptions *o) {
  if (x.empty()) return {{}, {}};
  if (!o) throw Panic(GDSP_ERR_INVALID, "invalid memory address or nil pointer dereference");
  const int nfft = o->NFFT ? o->NFFT : 256;
  const int pad = o->Pad ? o->Pad : nfft;
  const window::Func wf = o->Window ? o->Window : window::Func(window::Hann);
  const int flen = pad > nfft ? pad : nfft;
  const auto wseg = wf(flen), wnfft = wf(nfft);
  const int lp = pad / 2 + 1;
  std::vector<double> pxx(lp), freqs(lp);
  int64_t lpo = 0;
  check(gdsp_pwelch(x.data(), (int64_t)x.size(), Fs, nfft, pad, o->Noverlap, wseg.data(),
                    wnfft.data(), o->Scale_off ? 1 : 0, pxx.data(), freqs.data(), &lpo),
        "Pwelch");
  pxx.resize((size_t)lpo);
  freqs.resize((size_t)lpo);
  return {pxx, freqs};
}

// Pwelch split over `devices` (empty: the device set): segment shards and one
// in-process RCCL reduce of the per-bin sums (gdsp_pwelch_multi).
inline std::pair<std::vector<double>, std::vector<double>> PwelchMulti(
    const std::vector<double> &x, double Fs, const PwelchOptions *o,
    const std::vector<int> &devices = {}) {
  if (x.empty()) return {{}, {}};
  if (!o) throw Panic(GDSP_ERR_INVALID, "invalid memory address or nil pointer dereference");
  const int nfft = o->NFFT ? o->NFFT : 256;
  const int pad = o->Pad ? o->Pad : nfft;
  const window::Func wf = o->Window ? o->Window : window::Func(window::Hann);
  const int flen = pad > nfft ? pad : nfft;
  const auto wseg = wf(flen), wnfft = wf(nfft);
  const int lp = pad / 2 + 1;
  std::vector<double> pxx(lp), freqs(lp);
  int64_t lpo = 0;
  check(gdsp_pwelch_multi(x.data(), (int64_t)x.size(), Fs, nfft, pad, o->Noverlap, wseg.data(),
                          wnfft.data(), o->Scale_off ? 1 : 0, pxx.data(), freqs.data(), &lpo,
                          devices.empty() ? nullptr : devices.data(), (int)devices.size()),
        "PwelchMulti");
  pxx.resize((size_t)lpo);
  freqs.resize((size_t)lpo);
  return {pxx, freqs};
}

}  // namespace spectral

namespace wav {  // wav/wav.go

// An error value the reference returns (err.Error() as the message).
struct WavError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

constexpr int wavFormatPCM = 1, wavFormatIEEEFloat = 3;

// wav.Header — wav.go:37-45
struct Header {
  uint16_t AudioFormat = 0, NumChannels = 0;
  uint32_t SampleRate = 0, ByteRate = 0;
  uint16_t BlockAlign = 0, BitsPerSample = 0;
};

// wav.Wav — wav.go:48-56 (Duration: Go time.Duration, nanoseconds)
struct Wav : Header {
  int64_t Samples = 0;
  int64_t Duration = 0;
  std::istream *r = nullptr;
  int64_t remaining = 0;  // io.LimitReader over the data chunk

  int sample_bytes() const {
    if (AudioFormat == wavFormatPCM) {
      if (BitsPerSample == 8 || BitsPerSample == 16) return BitsPerSample / 8;
      throw WavError("wav: unknown bits per sample: " + std::to_string(BitsPerSample));
    }
    if (AudioFormat == wavFormatIEEEFloat) return 4;
    throw WavError("wav: unknown audio format");
  }
  // binary.Read of n samples: the raw little-endian bytes
  std::vector<unsigned char> read_raw(int64_t n) {
    const int64_t want = n * sample_bytes();
    const int64_t k = want < remaining ? want : remaining;
    std::vector<unsigned char> b((size_t)want);
    r->read(reinterpret_cast<char *>(b.data()), k);
    const int64_t got = r->gcount();
    remaining -= got;
    if (got == 0 && want > 0) throw WavError("EOF");
    if (got < want) throw WavError("unexpected EOF");
    return b;
  }
  // ReadFloats — wav.go:135-161, converted on the GPU
  std::vector<float> ReadFloats(int64_t n) {
    const auto raw = read_raw(n);
    std::vector<float> out((size_t)n);
    check(gdsp_wav_read_floats(raw.data(), n, AudioFormat, BitsPerSample, out.data(), 0),
          "wav.ReadFloats");
    return out;
  }
};

// wav.New — wav.go:59-107
inline Wav New(std::istream &r) {
  auto read_full = [&](unsigned char *b, int64_t n) {
    r.read(reinterpret_cast<char *>(b), n);
    const int64_t got = r.gcount();
    if (got == 0 && n > 0) throw WavError("EOF");
    if (got < n) throw WavError("unexpected EOF");
  };
  auto u16 = [](const unsigned char *p) { return (uint16_t)(p[0] | (p[1] << 8)); };
  auto u32 = [](const unsigned char *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
  };
  Wav w;
  unsigned char h[16];
  read_full(h, 12);
  if (std::string((char *)h, 4) != "RIFF") throw WavError("wav: missing RIFF");
  if (std::string((char *)h + 8, 4) != "WAVE") throw WavError("wav: missing WAVE");
  bool has_fmt = false;
  for (;;) {
    read_full(h, 8);
    const uint32_t sz = u32(h + 4);
    const std::string typ((char *)h, 4);
    if (typ == "fmt ") {
      if (sz < 16) throw WavError("wav: bad fmt size");
      std::vector<unsigned char> f(sz);
      read_full(f.data(), sz);
      w.AudioFormat = u16(&f[0]);
      w.NumChannels = u16(&f[2]);
      w.SampleRate = u32(&f[4]);
      w.ByteRate = u32(&f[8]);
      w.BlockAlign = u16(&f[12]);
      w.BitsPerSample = u16(&f[14]);
      if (w.AudioFormat != wavFormatPCM && w.AudioFormat != wavFormatIEEEFloat) {
        char m[64];
        snprintf(m, sizeof m, "wav: unknown audio format: %02x", w.AudioFormat);
        throw WavError(m);
      }
      has_fmt = true;
    } else if (typ == "data") {
      if (!has_fmt) throw WavError("wav: unexpected fmt chunk");
      w.Samples = (int64_t)sz / (int64_t)w.BitsPerSample * 8;
      w.Duration = w.Samples * 1000000000LL / (int64_t)w.SampleRate / (int64_t)w.NumChannels;
      w.r = &r;
      w.remaining = sz;
      return w;
    } else {
      r.ignore(sz);  // io.CopyN(ioutil.Discard, r, sz)
    }
  }
}

}  // namespace wav
}  // namespace gdsp
