// dev_api.hip — the development build's entry points (include/gdsp_fft_dev.h):
// the three wavefront-shuffle / wave-resident kernels that were built, found
// parity-green and measured slower than the product kernels,
// callable on their own so their tests can keep them honest. Everything here
// goes through the public C ABI (plans, batched device FFTs) plus the tables
// each kernel needs, built on the host from the reference's definitions; no
// product source refers to this file (make DEV=1 only).
#include <math.h>

#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "dev.hpp"
#include "gdsp_fft.h"
#include "gdsp_fft_dev.h"

namespace gdsp {
namespace {

#define DCHK(expr)                                    \
  do {                                                \
    if ((expr) != hipSuccess) return GDSP_ERR_HIP;    \
  } while (0)

int64_t next_pow2(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

// T_n[k] = exp(-2 pi i k / n) in long double, rounded once (as the product's
// power-of-2 plan tables)
std::vector<cd> table(int64_t n) {
  std::vector<cd> h((size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    const long double a = -2.0L * 3.141592653589793238462643383279502884L * (long double)k /
                          (long double)n;
    h[(size_t)k] = {(double)cosl(a), (double)sinl(a)};
  }
  return h;
}

template <class T>
int upload(const std::vector<T> &h, T **d) {
  DCHK(hipMalloc((void **)d, h.size() * sizeof(T)));
  DCHK(hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return GDSP_OK;
}

// The chirp-z tables of the reference (bluestein.go:32-94) on M =
// NextPowerOf2(2n - 1), plus each rejected kernel's permuted copies.
struct Tabs {
  int64_t n = 0, m = 0;
  int q = 0;                              // wave kernel: waves per transform
  cd *chirp = nullptr, *tm = nullptr;     // conj(w_k); T_M
  cd *t2048 = nullptr, *wbase = nullptr, *bhatw = nullptr;  // wave kernel
  cd *bhats = nullptr;                    // shuffle kernel (M = 8192)
};

int build(int64_t n, Tabs &t) {
  t.n = n;
  t.m = next_pow2(2 * n - 1);
  const int64_t M = t.m;
  std::vector<cd> w((size_t)n), chirp((size_t)n), b((size_t)M, cd{0.0, 0.0});
  for (int64_t k = 0; k < n; ++k) {  // the reference's unreduced angle pi/n k^2
    double sn = 0.0, cs = 1.0;
    if (k) {
      const double ang = M_PI / (double)n * (double)(k * k);
      sn = sin(ang);
      cs = cos(ang);
    }
    w[(size_t)k] = {cs, sn};
    chirp[(size_t)k] = {cs, -sn};
  }
  for (int64_t i = 0; i < n; ++i) {
    b[(size_t)i] = w[(size_t)i];
    if (i) b[(size_t)(M - i)] = w[(size_t)i];
  }
  // bhat = FFT_M(b) / M with the engine's own power-of-2 transform
  gdsp_plan *pm = nullptr;
  int st = gdsp_plan_create(M, &pm);
  if (st != GDSP_OK) return st;
  cd *db = nullptr, *dbh = nullptr;
  if ((st = upload(b, &db)) != GDSP_OK) return st;
  DCHK(hipMalloc((void **)&dbh, (size_t)M * sizeof(cd)));
  if ((st = gdsp_fft_batch_device(pm, db, dbh, 1, 0, nullptr)) != GDSP_OK) return st;
  std::vector<cd> bh((size_t)M);
  DCHK(hipMemcpy(bh.data(), dbh, (size_t)M * sizeof(cd), hipMemcpyDeviceToHost));
  (void)hipFree(db);
  (void)hipFree(dbh);
  for (auto &v : bh) v = {v.x / (double)M, v.y / (double)M};
  if ((st = upload(chirp, &t.chirp)) != GDSP_OK) return st;
  if ((st = upload(table(M), &t.tm)) != GDSP_OK) return st;
  t.q = bluestein_wave_q(n, M);
  if (t.q) {
    const int Q = t.q;
    std::vector<cd> bw((size_t)M), wb((size_t)(Q * 65));
    const long double tau = 2.0L * 3.141592653589793238462643383279502884L;
    for (int q = 0; q < Q; ++q) {
      for (int64_t k = 0; k < 2048; ++k) bw[(size_t)(q * 2048 + k)] = bh[(size_t)(Q * k + q)];
      for (int j = 0; j <= 64; ++j) {
        const long double a = -tau * (long double)(q * j) / (long double)M;
        wb[(size_t)(q * 65 + j)] = {(double)cosl(a), (double)sinl(a)};
      }
    }
    if ((st = upload(bw, &t.bhatw)) != GDSP_OK) return st;
    if ((st = upload(wb, &t.wbase)) != GDSP_OK) return st;
    if ((st = upload(table(2048), &t.t2048)) != GDSP_OK) return st;
  }
  if (M == 8192 && 2 * n <= M) {
    std::vector<cd> bs((size_t)M);
    for (int r = 0; r < 32; ++r)
      for (int tt = 0; tt < 256; ++tt) bs[(size_t)(r * 256 + tt)] = bh[(size_t)bluestein_shfl_bin(tt, r)];
    if ((st = upload(bs, &t.bhats)) != GDSP_OK) return st;
  }
  return GDSP_OK;
}

std::mutex g_mu;
std::map<std::pair<int, int64_t>, Tabs> g_tabs;  // (device, n)

int tabs_for(int64_t n, const Tabs **out) {
  int dev = 0;
  DCHK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_tabs.find({dev, n});
  if (it == g_tabs.end()) {
    Tabs t;
    const int st = build(n, t);
    if (st != GDSP_OK) return st;
    it = g_tabs.emplace(std::make_pair(dev, n), t).first;
  }
  *out = &it->second;
  return GDSP_OK;
}

}  // namespace
}  // namespace gdsp

using gdsp::cd;

extern "C" {

int gdsp_dev_chirpz_wave_q(int64_t n) {
  if (n < 2) return 0;
  return gdsp::bluestein_wave_q(n, gdsp::next_pow2(2 * n - 1));
}

int gdsp_dev_fft_batch_chirpz_wave(int64_t n, const void *d_in, void *d_out, int64_t batch,
                                   int inverse, void *stream) {
  if (batch < 0 || !d_in || !d_out || !gdsp_dev_chirpz_wave_q(n)) return GDSP_ERR_INVALID;
  if (batch == 0) return GDSP_OK;
  const gdsp::Tabs *t = nullptr;
  const int st = gdsp::tabs_for(n, &t);
  if (st != GDSP_OK) return st;
  return gdsp::launch_bluestein_wave(t->q, inverse != 0, (const cd *)d_in, (cd *)d_out, n, batch,
                                     t->t2048, t->wbase, t->bhatw, t->chirp, 1.0 / (double)n,
                                     (hipStream_t)stream) == hipSuccess
             ? GDSP_OK
             : GDSP_ERR_HIP;
}

int gdsp_dev_fft_batch_chirpz_shfl(int64_t n, const void *d_in, void *d_out, int64_t batch,
                                   int inverse, void *stream) {
  if (batch < 0 || !d_in || !d_out || n < 2049 || n > 4096) return GDSP_ERR_INVALID;
  if (batch == 0) return GDSP_OK;
  const gdsp::Tabs *t = nullptr;
  const int st = gdsp::tabs_for(n, &t);
  if (st != GDSP_OK) return st;
  return gdsp::launch_bluestein_shfl(inverse != 0, (const cd *)d_in, (cd *)d_out, n, batch, t->tm,
                                     t->chirp, t->bhats, 1.0 / (double)n, (hipStream_t)stream) ==
                 hipSuccess
             ? GDSP_OK
             : GDSP_ERR_HIP;
}

// the half-overlap NFFT 4096 accumulation of gdsp_pwelch_accumulate_device
// on one of the rejected kernels (same worker geometry: 2048 workers)
static int pw4096_dev(hipError_t (*launch)(const double *, int64_t, int64_t, int64_t, int64_t,
                                           const double *, const cd *, double *, hipStream_t),
                      const double *d_x, int64_t n, int64_t seg_begin, int64_t seg_end,
                      const double *d_win, double *d_acc, void *stream) {
  if (!d_x || !d_win || !d_acc || seg_begin < 0 || seg_end < seg_begin ||
      (seg_end > seg_begin && (seg_end - 1) * 2048 + 4096 > n))
    return GDSP_ERR_INVALID;
  if (seg_end == seg_begin) return GDSP_OK;
  static cd *tw = nullptr;
  static std::mutex mu;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (!tw && gdsp::upload(gdsp::table(4096), &tw) != GDSP_OK) return GDSP_ERR_HIP;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t target = npairs < 2048 ? npairs : 2048;
  const int64_t ppw = (npairs + target - 1) / target;
  const int64_t nworkers = (npairs + ppw - 1) / ppw;
  double *part = nullptr, *red = nullptr;
  DCHK(hipMalloc((void **)&part, (size_t)nworkers * 4096 * sizeof(double)));
  DCHK(hipMalloc((void **)&red,
                 (size_t)gdsp::reduce_scratch_doubles(nworkers, 4096) * sizeof(double)));
  hipError_t e = launch(d_x, seg_begin, seg_end, ppw, nworkers, d_win, tw, part, s);
  if (e == hipSuccess) e = gdsp::launch_reduce_partials(part, nworkers, 4096, d_acc, red, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(part);
  (void)hipFree(red);
  return e == hipSuccess ? GDSP_OK : GDSP_ERR_HIP;
}

int gdsp_dev_pwelch4096_shfl_accumulate(const double *d_x, int64_t n, int64_t seg_begin,
                                        int64_t seg_end, const double *d_win, double *d_acc,
                                        void *stream) {
  return pw4096_dev(gdsp::launch_pwelch4096_shfl, d_x, n, seg_begin, seg_end, d_win, d_acc,
                    stream);
}

int gdsp_dev_pwelch4096_row3_accumulate(const double *d_x, int64_t n, int64_t seg_begin,
                                        int64_t seg_end, const double *d_win, double *d_acc,
                                        void *stream) {
  return pw4096_dev(gdsp::launch_pwelch4096_row3, d_x, n, seg_begin, seg_end, d_win, d_acc,
                    stream);
}

}  // extern "C"
