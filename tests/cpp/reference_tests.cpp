// reference_tests.cpp — the reference's own tests (fft/fft_test.go,
// spectral/pwelch_test.go, spectral/spectral_test.go, window/window_test.go)
// re-expressed against the C++ host mirror (go-dsp_amd/host/gdsp.hpp), so
// they run through the C ABI on the GPU. The tables come from
// tests/golden/reference_vectors.json, flattened to text by
// tests/test_cpp_mirror.py (argv[1]). Exit code 0 = all pass.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>

#include "gdsp.hpp"

using namespace gdsp;

static int failures = 0, checks = 0;
#define EXPECT(cond, what)                                   \
  do {                                                       \
    ++checks;                                                \
    if (!(cond)) {                                           \
      ++failures;                                            \
      std::cerr << "FAIL " << what << " (" #cond ")\n";      \
    }                                                        \
  } while (0)

static std::vector<double> readd(std::istream &in, size_t n) {
  std::vector<double> v(n);
  for (auto &x : v) in >> x;
  return v;
}
static std::vector<complex> readc(std::istream &in, size_t n) {
  std::vector<complex> v(n);
  for (auto &x : v) {
    double a, b;
    in >> a >> b;
    x = {a, b};
  }
  return v;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    std::cerr << "usage: reference_tests vectors.txt\n";
    return 2;
  }
  // the additive entries: algorithm selection round trip, split-call counters
  fft::SetAlgorithm(GDSP_ALGO_CHIRPZ_POW2);
  EXPECT(fft::Algorithm() == GDSP_ALGO_CHIRPZ_POW2, "SetAlgorithm");
  fft::SetAlgorithm(GDSP_ALGO_DEFAULT);
  EXPECT(fft::GetMultiStats().batch_calls >= 0, "MultiStats");
  std::ifstream f(argv[1]);
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
      auto got = fft::FFTReal(x);
      std::ostringstream vals;
      for (auto &z : got) vals << z << " ";
      EXPECT(dsputils::PrettyCloseC(got, out), "FFTReal n=" << n << " got " << vals.str());
      EXPECT(dsputils::PrettyCloseC(fft::IFFT(out), dsputils::ToComplex(x)), "IFFT n=" << n);
    } else if (kind == "FFT2") {  // TestFFT2, fft_test.go:211-223
      size_t r, c;
      in >> r >> c;
      std::vector<std::vector<double>> x(r);
      for (auto &row : x) row = readd(in, c);
      fft::Matrix out(r);
      for (auto &row : out) row = readc(in, c);
      EXPECT(dsputils::PrettyClose2(fft::FFT2Real(x), out), "FFT2Real " << r << "x" << c);
      EXPECT(dsputils::PrettyClose2(fft::IFFT2(out), dsputils::ToComplex2(x)),
             "IFFT2 " << r << "x" << c);
    } else if (kind == "FFTN") {  // TestFFTN, fft_test.go:225-239
      size_t nd;
      in >> nd;
      std::vector<int> dims(nd);
      size_t n = 1;
      for (auto &d : dims) {
        in >> d;
        n *= d;
      }
      auto x = dsputils::ToComplex(readd(in, n));
      auto out = readc(in, n);
      auto m = dsputils::MakeMatrix(x, dims), o = dsputils::MakeMatrix(out, dims);
      EXPECT(fft::FFTN(m).PrettyClose(o), "FFTN");
      EXPECT(fft::IFFTN(o).PrettyClose(m), "IFFTN");
    } else if (kind == "WAV") {  // TestWav, wav_test.go:62-115 (+ ReadFloats)
      std::string path;
      int64_t fmt, ch, rate, brate, align, bits, samples, dur;
      in >> path >> fmt >> ch >> rate >> brate >> align >> bits >> samples >> dur;
      std::ifstream f(path, std::ios::binary);
      auto w = wav::New(f);
      EXPECT(w.AudioFormat == fmt && w.NumChannels == ch && w.SampleRate == rate &&
                 w.ByteRate == brate && w.BlockAlign == align && w.BitsPerSample == bits &&
                 w.Samples == samples && w.Duration == dur,
             "wav header " << path);
      const auto fl = w.ReadFloats(1024);
      std::ifstream g(path, std::ios::binary);
      g.seekg(44);
      bool ok = true;
      for (int i = 0; i < 1024; ++i) {  // wav.go:145-153 in float32 arithmetic
        float want;
        if (fmt == 3) {
          g.read(reinterpret_cast<char *>(&want), 4);
        } else {
          int16_t v;
          g.read(reinterpret_cast<char *>(&v), 2);
          volatile float num = (float)v - (-32768.0f);
          want = num / 65535.0f;
        }
        ok = ok && std::memcmp(&want, &fl[(size_t)i], 4) == 0;
      }
      EXPECT(ok, "wav ReadFloats " << path);
    } else if (kind == "PWELCH") {  // TestPwelch, pwelch_test.go:48-60
      double fs;
      size_t n, lp;
      in >> fs >> n;
      auto x = readd(in, n);
      in >> lp;
      auto p = readd(in, lp), fr = readd(in, lp);
      spectral::PwelchOptions o;
      auto res = spectral::Pwelch(x, fs, &o);
      EXPECT(dsputils::PrettyClose(res.first, p), "Pwelch Pxx n=" << n);
      EXPECT(dsputils::PrettyClose(res.second, fr), "Pwelch freqs n=" << n);
      // the same through the multi-device entry (RCCL reduce over the device set)
      auto rm = spectral::PwelchMulti(x, fs, &o);
      EXPECT(dsputils::PrettyClose(rm.first, p), "PwelchMulti Pxx n=" << n);
    } else if (kind == "SEG") {  // TestSegment, spectral_test.go:58-67
      size_t xl, nseg;
      int size, nov;
      in >> xl;
      auto x = readd(in, xl);
      in >> size >> nov >> nseg;
      auto segs = spectral::Segment(x, size, nov);
      bool ok = segs.size() == nseg;
      for (size_t s = 0; s < nseg; ++s) {
        auto want = readd(in, size);
        if (ok) ok = dsputils::PrettyClose(segs[s], want);
      }
      EXPECT(ok, "Segment size=" << size << " noverlap=" << nov);
    } else if (kind == "WIN") {  // TestWindowFunctions, window_test.go:61-94
      int L;
      in >> L;
      auto hm = readd(in, L), hn = readd(in, L), bt = readd(in, L), ft = readd(in, L),
           bk = readd(in, L);
      EXPECT(dsputils::PrettyClose(window::Hamming(L), hm), "Hamming L=" << L);
      EXPECT(dsputils::PrettyClose(window::Hann(L), hn), "Hann L=" << L);
      EXPECT(dsputils::PrettyClose(window::Bartlett(L), bt), "Bartlett L=" << L);
      auto o = window::Rectangular(L);
      window::Apply(o, window::Hamming);
      EXPECT(dsputils::PrettyClose(o, hm), "Apply L=" << L);
      EXPECT(dsputils::PrettyClose(window::FlatTop(L), ft), "FlatTop L=" << L);
      EXPECT(dsputils::PrettyClose(window::Blackman(L), bk), "Blackman L=" << L);
    }
  }
  // panics of the reference (fft.go:40,57,126,133) and empty-input conventions
  auto panics = [](auto fn) {
    try {
      fn();
    } catch (const Panic &) {
      return true;
    }
    return false;
  };
  EXPECT(panics([] { fft::Convolve({1, 2}, {1}); }), "Convolve unequal panics");
  EXPECT(panics([] { fft::IFFT({}); }), "IFFT empty panics");
  EXPECT(panics([] { fft::FFT2({}); }), "FFT2 empty panics");
  EXPECT(panics([] { fft::FFT2({{1, 2}, {3}}); }), "FFT2 ragged panics");
  EXPECT(fft::FFT({}).empty(), "FFT empty returns empty");
  EXPECT(spectral::Pwelch({}, 1, nullptr).first.empty(), "Pwelch empty returns empty");
  // TestSegment, dsputils/dsputils_test.go:41-58
  {
    std::vector<complex> x;
    for (int n = 0; n < 16; ++n) x.push_back(complex(n, 0));
    auto v = dsputils::Segment(x, 3, 0.5);
    std::vector<std::vector<complex>> want = {{x.begin(), x.begin() + 8},
                                              {x.begin() + 4, x.begin() + 12},
                                              {x.begin() + 8, x.begin() + 16}};
    EXPECT(dsputils::PrettyClose2(v, want), "dsputils.Segment");
  }
  // TestMakeMatrix, dsputils/matrix_test.go:23-47
  {
    std::vector<complex> v;
    for (double d : {1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 4, 3, 2, 1})
      v.push_back(d);
    auto m = dsputils::MakeMatrix(v, {2, 3, 4});
    EXPECT(dsputils::PrettyCloseC(m.Dim({1, 0, -1}), dsputils::ToComplex({3, 4, 5, 6})), "Dim 1");
    EXPECT(dsputils::PrettyCloseC(m.Dim({0, -1, 2}), dsputils::ToComplex({3, 7, 1})), "Dim 2");
    EXPECT(dsputils::PrettyCloseC(m.Dim({-1, 1, 3}), dsputils::ToComplex({8, 0})), "Dim 3");
    auto s3 = dsputils::ToComplex({10, 11, 12});
    m.SetDim(s3, {1, -1, 3});
    EXPECT(dsputils::PrettyCloseC(m.Dim({1, -1, 3}), s3), "SetDim");
    m.SetValue(complex(14, 0), {1, -1, 3});
    EXPECT(dsputils::ComplexEqual(m.Value({1, -1, 3}), complex(14, 0)), "SetValue");
  }
  // TestFFTMulti (fft_test.go:251-259) + a Bluestein batch through FFTBatch
  std::vector<complex> a(256);
  for (int i = 0; i < 256; ++i) a[i] = {i / 256.0, 0};
  auto A = fft::FFT(a);
  EXPECT(dsputils::ComplexEqual(A[0], complex(127.5, 0)), "FFTMulti DC");
  std::vector<complex> b(3000 * 4, complex(1, 0));
  auto B = fft::FFTBatch(b, 3000);
  EXPECT(dsputils::ComplexEqual(B[3000], complex(3000, 0)) && std::abs(B[3001]) < 1e-9,
         "FFTBatch Bluestein row 1");
  auto BM = fft::FFTBatchMulti(b, 3000, false, fft::Devices());
  EXPECT(BM == B, "FFTBatchMulti equals FFTBatch");
  std::cout << "checks " << checks << " failures " << failures << "\n";
  return failures ? 1 : 0;
}
