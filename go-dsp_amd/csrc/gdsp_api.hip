// gdsp_api.hip — the C ABI of libgdspfft (include/gdsp_fft.h): plan cache,
// per-thread streams, host-pointer entry points (what cgo binds) and
// device-pointer entry points (what the multi-GPU drivers call).
//
// Every transform runs on the GPU. There is no CPU compute path: without a
// HIP device the entry points return GDSP_ERR_NO_DEVICE.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "fft_device.hpp"
#include "gdsp_fft.h"
#include "launch.hpp"
#include "api_internal.hpp"

using gdsp::cd;

#define GDSP_VERSION "gdspfft 0.3.0 (gfx950)"

namespace {

thread_local std::string g_last_error;
int g_worker_pool_size = 0;  // fft.SetWorkerPoolSize mirror (no GPU meaning)

int fail(int st, const std::string &msg) {
  g_last_error = msg;
  return st;
}

#define HIPCHK(expr)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(GDSP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
  } while (0)

#define STCHK(expr)               \
  do {                            \
    int s_ = (expr);              \
    if (s_ != GDSP_OK) return s_; \
  } while (0)

bool is_pow2(int64_t x) { return (x & (x - 1)) == 0; }

int ilog2(int64_t x) {
  int r = 0;
  while (x > 1) {
    x >>= 1;
    ++r;
  }
  return r;
}

// dsputils.NextPowerOf2 (dsputils/dsputils.go:39-45): float Log2/Ceil/Pow.
int64_t next_pow2_ref(int64_t x) {
  if (is_pow2(x)) return x;
  return (int64_t)pow(2.0, ceil(log2((double)x)));
}

int current_device(int *dev) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(GDSP_ERR_NO_DEVICE, "no HIP device visible");
  if (hipGetDevice(dev) != hipSuccess) return fail(GDSP_ERR_NO_DEVICE, "hipGetDevice failed");
  return GDSP_OK;
}

// One non-blocking stream per (thread, device) for the host-pointer API.
hipStream_t thread_stream(int dev) {
  thread_local std::map<int, hipStream_t> streams;
  auto it = streams.find(dev);
  if (it != streams.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams[dev] = s;
  return s;
}

// The one-kernel transform exchanges real and imaginary halves in turn
// (half the LDS, so more workgroups per CU than with two buffers).
bool lds_split_default() { return true; }

std::atomic<unsigned> g_algo{GDSP_ALGO_DEFAULT};
constexpr unsigned kAlgoAll = GDSP_ALGO_GENERIC_MIXED | GDSP_ALGO_NO_CHIRPZ_PARTS |
                              GDSP_ALGO_CHIRPZ_POW2 | GDSP_ALGO_CHIRPZ_UNFUSED |
                              GDSP_ALGO_NO_RADER | GDSP_ALGO_NO_RACE;

// Scratch device memory: a grow-only buffer per (device, stream, use-site
// slot), allocated with hipMalloc. Reuse is ordered by the stream itself: a
// slot is only ever used by work queued on its stream, so a later call can
// overwrite it only after the earlier kernels on that stream ran. Growing a
// slot synchronises its stream before freeing the old buffer.
// (Stream-ordered hipMallocAsync/hipFreeAsync lost kernel output
// intermittently under the ROCm 7.2 runtime here — tests/cpp reproduced it —
// so the library does not use it.) Device-API callers must not drive one
// stream from two host threads at once.
enum Slot {
  SLOT_IN = 0, SLOT_OUT, SLOT_AUX, SLOT_AUX2, SLOT_GLOBAL, SLOT_GLOBAL_IN, SLOT_REAL,
  SLOT_BLU, SLOT_FFT2, SLOT_PW_PART, SLOT_PW_RED, SLOT_PW_BUF, SLOT_FS0, SLOT_FS1, SLOT_FS2,
  SLOT_FS3, SLOT_FFTN, SLOT_MX0, SLOT_MX1, SLOT_PARTS, SLOT_COUNT
};

struct Workspace {
  void *buf[SLOT_COUNT] = {};
  size_t cap[SLOT_COUNT] = {};
};

std::mutex g_ws_mu;
std::map<std::pair<int, hipStream_t>, Workspace> g_ws;

struct DevBuf {
  void *p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  int alloc(size_t bytes, hipStream_t st, Slot slot) {
    if (bytes == 0) bytes = 16;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(GDSP_ERR_NO_DEVICE, "hipGetDevice failed");
    std::lock_guard<std::mutex> lk(g_ws_mu);
    Workspace &w = g_ws[std::make_pair(dev, st)];
    if (w.cap[slot] < bytes) {
      if (w.buf[slot]) {
        HIPCHK(hipStreamSynchronize(st));  // queued users of the old buffer
        HIPCHK(hipFree(w.buf[slot]));
        w.buf[slot] = nullptr;
        w.cap[slot] = 0;
      }
      const size_t want = bytes + bytes / 4;  // headroom against regrowth
      hipError_t e = hipMalloc(&w.buf[slot], want);
      if (e != hipSuccess) {
        w.buf[slot] = nullptr;
        return fail(GDSP_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
      }
      w.cap[slot] = want;
    }
    p = w.buf[slot];
    return GDSP_OK;
  }
};

// Host <-> device copies through library-owned pinned staging buffers (two
// halves, double-buffered). The caller's memory is only touched by memcpy on
// the host, so pageable (Go / numpy) buffers never reach the HIP runtime and
// no pointer is retained after the call returns (cgo rule).
struct Staging {
  char *buf = nullptr;
  size_t half = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};  // a queued copy may still read / write the half
  ~Staging() {
    if (buf) (void)hipHostFree(buf);
    for (auto &e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

// 8 MiB halves: a 16 MiB vector (BenchmarkFFT's 2^20) already pipelines its
// host memcpy with the DMA of the previous half
constexpr size_t kStagingHalf = (size_t)8 << 20;

// memcpy between the caller's pageable memory and the pinned staging, split
// over a few host threads for large chunks (one thread copies ~10-20 GB/s,
// well below what PCIe moves)
void host_copy(void *dst, const void *src, size_t n) {
  constexpr size_t kPar = (size_t)2 << 20;
  const unsigned hw = std::thread::hardware_concurrency();
  const unsigned k = n < kPar ? 1 : std::min<unsigned>(4, hw ? hw : 1);
  if (k <= 1) {
    memcpy(dst, src, n);
    return;
  }
  const size_t part = (n / k + 63) & ~(size_t)63;
  std::thread th[3];
  size_t rest = n;  // this thread also copies [rest, n) if a thread could not start
  unsigned used = 0;
  for (unsigned i = 1; i < k && i * part < n; ++i) {
    const size_t off = i * part, c = std::min(part, n - off);
    try {
      th[used] = std::thread([=] { memcpy((char *)dst + off, (const char *)src + off, c); });
      ++used;
    } catch (...) {  // nothing may throw past the C ABI
      rest = off;
      break;
    }
  }
  memcpy(dst, src, std::min(part, n));
  if (rest < n) memcpy((char *)dst + rest, (const char *)src + rest, n - rest);
  for (unsigned i = 0; i < used; ++i) th[i].join();
}

int staging_get(Staging **out) {
  thread_local std::map<int, Staging> per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(GDSP_ERR_NO_DEVICE, "hipGetDevice failed");
  Staging &st = per_dev[dev];
  if (!st.buf) {
    HIPCHK(hipHostMalloc((void **)&st.buf, 2 * kStagingHalf, hipHostMallocDefault));
    st.half = kStagingHalf;
    for (auto &e : st.ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  *out = &st;
  return GDSP_OK;
}

// Host -> device through the staging halves. A half is refilled only after
// the copy that last used it has completed (its event); the copies themselves
// stay queued, and the stream orders them before the kernels and the
// device -> host copies that follow on the same stream.
int copy_h2d(void *dst, const void *src, size_t bytes, hipStream_t s) {
  Staging *st = nullptr;
  STCHK(staging_get(&st));
  int h = 0;
  for (size_t off = 0; off < bytes; off += st->half, h ^= 1) {
    const size_t c = bytes - off < st->half ? bytes - off : st->half;
    char *stg = st->buf + (size_t)h * st->half;
    if (st->pending[h]) {
      HIPCHK(hipEventSynchronize(st->ev[h]));
      st->pending[h] = false;
    }
    host_copy(stg, (const char *)src + off, c);
    HIPCHK(hipMemcpyAsync((char *)dst + off, stg, c, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(st->ev[h], s));
    st->pending[h] = true;
  }
  return GDSP_OK;
}

// Device -> host, double-buffered; returns once every chunk has landed in
// dst, so everything queued on s before it has completed too.
int copy_d2h(void *dst, const void *src, size_t bytes, hipStream_t s) {
  Staging *st = nullptr;
  STCHK(staging_get(&st));
  const size_t nchunk = (bytes + st->half - 1) / st->half;
  auto issue = [&](size_t i) -> int {
    const size_t off = i * st->half;
    const size_t c = bytes - off < st->half ? bytes - off : st->half;
    HIPCHK(hipMemcpyAsync(st->buf + (i & 1) * st->half, (const char *)src + off, c,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(st->ev[i & 1], s));
    st->pending[i & 1] = true;
    return GDSP_OK;
  };
  if (nchunk) STCHK(issue(0));
  for (size_t i = 0; i < nchunk; ++i) {
    if (i + 1 < nchunk) STCHK(issue(i + 1));
    HIPCHK(hipEventSynchronize(st->ev[i & 1]));
    st->pending[i & 1] = false;
    const size_t off = i * st->half;
    const size_t c = bytes - off < st->half ? bytes - off : st->half;
    host_copy((char *)dst + off, st->buf + (i & 1) * st->half, c);
  }
  return GDSP_OK;
}

// Mapped pinned host memory per (thread, device) for small host calls
// (input at 0, output at kZeroCopyOut): the kernels access it over the
// fabric, which for a few hundred KiB costs less than two copy launches.
constexpr size_t kZeroCopyOut = (size_t)512 << 10;
constexpr size_t kZeroCopyMax = (size_t)512 << 10;  // in + out bytes of one call
struct ZeroCopy {
  char *host = nullptr;
  void *dev = nullptr;
  ~ZeroCopy() {
    if (host) (void)hipHostFree(host);
  }
};

int zero_copy_get(ZeroCopy **out) {
  thread_local std::map<int, ZeroCopy> per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(GDSP_ERR_NO_DEVICE, "hipGetDevice failed");
  ZeroCopy &z = per_dev[dev];
  if (!z.host) {
    HIPCHK(hipHostMalloc((void **)&z.host, 2 * kZeroCopyOut, hipHostMallocMapped));
    hipError_t e = hipHostGetDevicePointer(&z.dev, z.host, 0);
    if (e != hipSuccess) {
      (void)hipHostFree(z.host);
      z.host = nullptr;
      return fail(GDSP_ERR_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    }
  }
  *out = &z;
  return GDSP_OK;
}

}  // namespace

enum PlanKind { KIND_TRIVIAL = 0, KIND_LDS = 1, KIND_GLOBAL = 2, KIND_BLUESTEIN = 3,
                KIND_BLUESTEIN_COMPOSED = 4, KIND_MIXED = 5, KIND_MIXED4 = 6, KIND_RADER = 7,
                KIND_RADER_PFA = 8 };

struct gdsp_plan {
  int device = 0;
  int64_t n = 0;
  int kind = KIND_TRIVIAL;
  int log2n = 0;
  cd *tw = nullptr;  // power of 2: T_n[k] = exp(-2 pi i k/n), n entries;
                     // mixed radix: the per-pass butterfly-major table
  gdsp::MixedDesc md{};
  gdsp::MixedDesc md_gen{};  // generic radix list (runtime-radix kernels)
  cd *tw_gen = nullptr;
  // the fused Pwelch's own compiled list where it differs from md's
  // (pwelch_fixed_radices; md_pw.n = 0: none)
  gdsp::MixedDesc md_pw{};
  cd *tw_pw = nullptr;
  gdsp::JitSpec *jit = nullptr;  // runtime-compiled specialisation of md (mixed_jit.hip)
  // mixed four-step (KIND_MIXED4): n = n1 * n2, one-kernel sub-plans, tw = T_n;
  // pow2col: n1 is a power of 2 in [16, 512], so the column DFT runs on
  // row-segment tiles; radixcol: n1 <= 25 is one radix, a column per thread
  // (either way 3 HBM passes instead of 5)
  int64_t n1 = 0, n2 = 0;
  bool pow2col = false, radixcol = false;
  // rowst: n2 a power of 2 in [16, 1024] and n1 a radixcol / mixcol column:
  // two passes, the rows' store carrying the transpose (rowfft_t_kernel)
  bool rowst = false;
  gdsp::JitRowT *rowt = nullptr;  // rowst with n2 smooth, not a power of 2: the rows' kernel
  // mixcol: n1 in [26, 1016] smooth, its column pass runtime-compiled
  gdsp::JitCol *mixcol = nullptr;
  gdsp_plan *p1 = nullptr, *p2 = nullptr;
  // Bluestein (fft/bluestein.go): M = NextPowerOf2(2n-1), chirp = conj(w),
  // bhat = FFT_M(b)/M
  int64_t m = 0;
  int log2m = 0;
  gdsp_plan *mplan = nullptr;
  cd *chirp = nullptr;
  cd *bhat = nullptr;
  // output-split chirp-z (bluestein_kernel PARTS): n in (8192, 16384] whose
  // NextPowerOf2(2n-1) = 32768 exceeds one kernel runs as `parts` fused
  // convolutions of M = 16384, each giving kpart outputs; bhat holds parts * M
  int parts = 1;
  // fused chirp-z on M = 16 RB 16 (chirpz6k.hip: the smallest such M >= 2n - 1,
  // 129 <= n <= 3200, where bluestein.go:70 pads to NextPowerOf2(2n - 1));
  // tw6k: its pass twiddle bases
  bool c6k = false;
  cd *tw6k = nullptr;
  // composed chirp-z without its fused transposes (GDSP_ALGO_CHIRPZ_UNFUSED)
  bool unfused = false;
  int64_t kpart = 0;
  // Rader (KIND_RADER, a prime n whose n - 1 has a radix list): the kernel,
  // m = n - 1 (the cyclic convolution's length), tw its per-pass twiddle
  // bases, bhat = FFT_m(b)/m, gpow[q] = g^q mod n, ginv[r] = g^-r mod n
  gdsp::JitRader *rader = nullptr;
  int *gpow = nullptr, *ginv = nullptr;
  // fused chirp-z on a smooth convolution length (KIND_BLUESTEIN, m = L):
  // bluestein_fixed_kernel for n, tw_blu its per-pass twiddle bases
  gdsp::JitBlu *blufix = nullptr;
  cd *tw_blu = nullptr, *bhat_blu = nullptr;
  int64_t m_blu = 0;
  gdsp::MixedDesc md_blu{};
  // prime-factor Rader (KIND_RADER_PFA, n = n1 * n2, n2 a prime with a Rader
  // plan p2 whose tables the kernel reads, gcd(n1, n2) = 1): rader is
  // rader_pfa_kernel for the cofactor n1, m = n2 - 1
};

namespace {

// recursive: building a Bluestein plan runs FFT_M(b), whose four-step path
// fetches sub-plans from this cache on the same thread
std::recursive_mutex g_plan_mu;
// keyed by (device, n, algorithm flags the plan was built under)
std::map<std::tuple<int, int64_t, unsigned>, gdsp_plan *> g_plans;
std::map<std::tuple<int, int64_t, unsigned>, gdsp_plan *> g_chirpz_plans;  // forced Bluestein

int exec_plan(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
              hipStream_t s);

// T_n[k] = exp(-2 pi i k/n), evaluated in long double and rounded once.
int upload_twiddles(int dev, int64_t n, cd **dst) {
  std::vector<cd> h((size_t)n);
  for (int64_t k = 0; k < n; ++k) {
    long double a = -2.0L * 3.141592653589793238462643383279502884L * (long double)k /
                    (long double)n;
    h[(size_t)k].x = (double)cosl(a);
    h[(size_t)k].y = (double)sinl(a);
  }
  HIPCHK(hipMalloc((void **)dst, (size_t)n * sizeof(cd)));
  STCHK(copy_h2d(*dst, h.data(), (size_t)n * sizeof(cd), thread_stream(dev)));
  // plans are shared by every stream and thread: the table must be complete
  HIPCHK(hipStreamSynchronize(thread_stream(dev)));
  return GDSP_OK;
}

int get_plan_locked(int dev, int64_t n, gdsp_plan **out);

// Radices of the mixed-radix kernel for n (fft_mixed.hip), or false when n is
// a power of 2, too long, or has a prime factor above 13 (-> Bluestein).
bool mixed_radices(int64_t n, std::vector<int> &rad, bool specs = true) {
  rad.clear();
  if (n < 2 || n > gdsp::kMixedSpecMax || is_pow2(n)) return false;
  if (n > gdsp::kMixedMax) {  // beyond the runtime-radix kernel: specialisations only
    int fr[16], fnp = 0;
    if (!specs || !gdsp::mixed_fixed_radices((int)n, fr, &fnp)) return false;
    rad.assign(fr, fr + fnp);
    return true;
  }
  int64_t m = n;
  int a = 0;
  while (m % 2 == 0) {
    m /= 2;
    ++a;
  }
  std::vector<int> odd;
  for (int q : {13, 11, 7, 5, 3})
    while (m % q == 0) {
      m /= q;
      odd.push_back(q);
    }
  if (m != 1) return false;
  int fr[16], fnp = 0;
  if (specs && gdsp::mixed_fixed_radices((int)n, fr, &fnp)) {
    rad.assign(fr, fr + fnp);
    return true;
  }
  while (a >= 4) {
    rad.push_back(16);
    a -= 4;
  }
  if (a) rad.push_back(1 << a);
  rad.insert(rad.end(), odd.begin(), odd.end());
  return rad.size() <= 12;
}

// Descriptor + per-pass twiddle bases W_{Ns*R}^k (k < Ns; the kernels
// raise them to the powers r = 1..R-1 in registers) of one radix list.
// geometry: check the thread count of the mixed-radix kernels' geometry (the
// fused chirp-z kernels, which only take the twiddle bases, have their own)
int make_mixed_desc(int dev, int64_t n, const std::vector<int> &rad, gdsp::MixedDesc &d,
                    cd **tw, bool geometry = true) {
  d.n = (int)n;
  d.npass = (int)rad.size();
  d.codes = 0;
  int need = 1;
  for (size_t q = 0; q < rad.size(); ++q) {
    d.codes |= (uint64_t)rad[q] << (5 * q);
    const int jmax = rad[q] > 16 ? 1 : 16 / rad[q], nb = (int)n / rad[q];
    need = std::max(need, (nb + jmax - 1) / jmax);
  }
  int t1 = 1;
  while (t1 < need) t1 <<= 1;
  if (t1 > 64) t1 = (need + 63) / 64 * 64;
  // (the runtime-radix kernels check t1 <= 512 themselves; a compiled or
  // runtime-compiled specialisation may use up to 1024 threads per transform)
  if (geometry && t1 > 1024) return fail(GDSP_ERR_UNSUPPORTED, "mixed-radix geometry");
  d.t1 = t1;
  d.tpw = std::max(1, std::min(256 / t1, gdsp::kMixedMax / (int)n));
  std::vector<cd> h;
  int64_t ns = rad[0];
  for (size_t q = 1; q < rad.size(); ++q) {
    const int R = rad[q];
    for (int64_t k = 0; k < ns; ++k) {
      const long double ang = -2.0L * 3.141592653589793238462643383279502884L * (long double)k /
                              (long double)(ns * R);
      h.push_back({(double)cosl(ang), (double)sinl(ang)});
    }
    ns *= R;
  }
  if (h.empty()) h.push_back({1.0, 0.0});
  HIPCHK(hipMalloc((void **)tw, h.size() * sizeof(cd)));
  STCHK(copy_h2d(*tw, h.data(), h.size() * sizeof(cd), thread_stream(dev)));
  HIPCHK(hipStreamSynchronize(thread_stream(dev)));
  return GDSP_OK;
}

int build_mixed(int dev, int64_t n, const std::vector<int> &rad, gdsp_plan *p) {
  p->kind = KIND_MIXED;
  STCHK(make_mixed_desc(dev, n, rad, p->md, &p->tw));
  {
    int pr[16], pnp = 0;
    if (gdsp::pwelch_fixed_radices((int)n, pr, &pnp))
      STCHK(make_mixed_desc(dev, n, std::vector<int>(pr, pr + pnp), p->md_pw, &p->tw_pw));
  }
  // the runtime-radix kernels (fused Pwelch) take the generic list: radices
  // <= 16, no composites (a compiled specialisation's list may hold them)
  std::vector<int> gen;
  if (!mixed_radices(n, gen, false)) {
    p->md_gen = gdsp::MixedDesc{};  // no runtime-radix list (n > kMixedMax)
    return GDSP_OK;
  }
  if (gen == rad) {
    p->md_gen = p->md;
    p->tw_gen = p->tw;
    return GDSP_OK;
  }
  return make_mixed_desc(dev, n, gen, p->md_gen, &p->tw_gen);
}

// Lengths one kernel transforms per row: powers of 2 up to the LDS limit,
// the mixed-radix set, and every other m <= 8192 through the fused chirp-z
// kernel (M = NextPowerOf2(2m - 1) <= 16384), so a length with a large prime
// factor but a smooth cofactor (8191 * 64) still gets a three-pass four-step
// instead of the composed chirp-z over 2n-point rows.
// Output parts of the split chirp-z for n (see gdsp_plan::parts): the fewest
// P <= 8 with n + ceil(n/P) - 1 <= 16384 where NextPowerOf2(2n-1) exceeds
// one kernel, else 0 (composed chirp-z). P = 8 (n <= 14563) measured 10.8
// against 11.5 ms for the composed chirp-z per 2^27 samples, P = 2 4x faster.
// The algorithm flags a plan is built under: read once by the outermost
// get_plan_locked of a thread (the cache key) and used by every decision of
// that build and of the sub-plans it fetches, so a concurrent
// gdsp_set_algorithm cannot leave a plan built under mixed flags in the
// cache (plans are built under g_plan_mu; the snapshot is per thread).
thread_local int t_build_depth = 0;
thread_local unsigned t_build_flags = 0;
unsigned plan_flags() { return gdsp::algo_flags(); }

int chirpz_parts(int64_t n) {
  const bool off = (plan_flags() & GDSP_ALGO_NO_CHIRPZ_PARTS) != 0;
  const int64_t mk = (int64_t)1 << gdsp::kMaxLdsLog2;
  if (off || next_pow2_ref(2 * n - 1) <= mk) return 0;
  for (int parts = 2; parts <= 8; ++parts)
    if (n + (n + parts - 1) / parts - 1 <= mk) return parts;
  return 0;
}

bool one_kernel_len(int64_t m) {
  if (m < 2) return false;
  if (chirpz_parts(m)) {
    // only a prime builds as the output-split chirp-z plan: a composite in
    // (8192, 14563] has a four-step split, which build_plan takes first
    bool prime = true;
    for (int64_t d = 2; d * d <= m && prime; ++d) prime = m % d != 0;
    if (prime) return true;
  }
  if (is_pow2(m)) return ilog2(m) <= gdsp::kMaxLdsLog2;
  std::vector<int> rad;
  if (mixed_radices(m, rad)) return true;
  int jr[5], jnp = 0;  // a runtime-compiled specialisation
  if (gdsp::jit_enabled() && gdsp::jit_radices((int)m, jr, &jnp)) return true;
  return next_pow2_ref(2 * m - 1) <= ((int64_t)1 << gdsp::kMaxLdsLog2);
}

// n = n1 * n2 with both factors one-kernel lengths, n1 <= n2 as balanced as
// possible (fewest, shortest transposes); false if none exists.
bool mixed4_split(int64_t n, int64_t &n1, int64_t &n2) {
  for (int64_t d = (int64_t)sqrtl((long double)n); d >= 2; --d) {
    if (n % d == 0 && one_kernel_len(d) && one_kernel_len(n / d)) {
      n1 = d;
      n2 = n / d;
      return true;
    }
  }
  return false;
}

// n = R * C with R a power of 2 in [16, 512] (column tiles) and C a
// one-kernel length; the largest such R (shortest rows) wins.
bool pow2col_split(int64_t n, int64_t &r, int64_t &c) {
  for (int64_t R = (int64_t)1 << gdsp::kColMaxLog2; R >= ((int64_t)1 << gdsp::kColMinLog2);
       R >>= 1) {
    if (n % R == 0 && one_kernel_len(n / R)) {
      r = R;
      c = n / R;
      return true;
    }
  }
  return false;
}

// n = L * C with L a single radix (<= 25, largest first) and C a one-kernel
// length.
bool radixcol_split(int64_t n, int64_t &l, int64_t &c) {
  for (int L : {25, 20, 16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2}) {
    if (gdsp::colradix_supported(L) && n % L == 0 && one_kernel_len(n / L)) {
      l = L;
      c = n / L;
      return true;
    }
  }
  return false;
}

// n = L * C with L in [26, 1016] a smooth non-power-of-2 length (the
// column pass, colfixed_kernel compiled for L's radix list) and C a
// one-kernel length; the smallest such L (widest column tiles) whose column
// kernel builds wins.
// the runtime-compiled column pass for the column length L of n = L * (n / L)
bool mixcol_try(int dev, int64_t n, int64_t L, gdsp_plan *p) {
  if (!gdsp::jit_enabled() || n % L || L < 26 || L > 1016 || is_pow2(L) || !one_kernel_len(L))
    return false;
  gdsp_plan *p1 = nullptr;
  if (get_plan_locked(dev, L, &p1) != GDSP_OK || p1->kind != KIND_MIXED) return false;
  int rad[16], np = p1->md.npass;
  if (np < 2 || np > 16) return false;
  for (int q = 0; q < np; ++q) rad[q] = (int)((p1->md.codes >> (5 * q)) & 31);
  gdsp::JitCol *col = gdsp::jit_col_build(dev, rad, np);
  if (!col) return false;
  p->mixcol = col;
  p->n1 = L;
  p->n2 = n / L;
  p->p1 = p1;
  return true;
}

bool mixcol_build(int dev, int64_t n, gdsp_plan *p) {
  if (!gdsp::jit_enabled()) return false;
  for (int64_t L = 26; L <= 1016; ++L) {
    if (n % L || is_pow2(L) || !one_kernel_len(n / L) || !one_kernel_len(L)) continue;
    if (mixcol_try(dev, n, L, p)) return true;
  }
  return false;
}

// n = L * 2^k, 2^k in [16, 1024], with a column pass for L (one radix <= 25:
// colradix_kernel; 26 <= L <= 1016 smooth: the runtime-compiled
// colfixed_kernel): two HBM passes, the columns and then the rows of 2^k
// with the transpose in their store (rowfft_t_kernel), instead of three.
// Rows of 256 first (256-B output segments), then shorter ones (longer
// segments, longer columns), then 512 and 1024.
bool pow2rows_build(int dev, int64_t n, gdsp_plan *p) {
  for (int k : {8, 7, 6, 5, 4, 9, 10}) {
    const int64_t C = (int64_t)1 << k;
    if (n % C) continue;
    const int64_t L = n / C;
    if (L < 2 || is_pow2(L)) continue;
    if (L <= 25 && gdsp::colradix_supported((int)L)) {
      p->radixcol = true;
      p->n1 = L;
      p->n2 = C;
    } else if (!mixcol_try(dev, n, L, p)) {
      continue;
    }
    p->rowst = true;
    return true;
  }
  return false;
}

// n = L * C with C <= 1024 a smooth one-kernel length (not a power of 2; its
// rows by the runtime-compiled rowt_fixed_kernel, the transpose in their
// store) and a column pass for L (a power of 2 in [16, 512], one radix <= 25
// or a runtime-compiled column length in [26, 1016]): two HBM passes where
// pow2rows_build finds no power-of-2 row length (10^6 = 1000 x 1000, 44100).
// Rows of 1000 (10 x 10 x 10) first where the columns are >= 64 points long,
// then the split closest to C = sqrt(n): per 2^27 samples (profiles/r04/
// mixed4_rows_ab.txt) 10^6, 600000, 200000, 100000, 50000 took 1.6-2.0 ms
// on rows of 1000 but up to 3.1 on the balanced split, while 44100 took
// 1.93-2.03 ms at C = 225 / 210 and 2.42 at 630 (2.34 in three passes), and
// 30000 1.78 at C = 150 and 2.50 at 1000.
bool mixrows_build(int dev, int64_t n, gdsp_plan *p) {
  if (!gdsp::jit_enabled()) return false;
  std::vector<int64_t> cands;
  for (int64_t C = 16; C <= 1024; ++C)
    if (n % C == 0 && !is_pow2(C)) cands.push_back(C);
  const long double r = sqrtl((long double)n);
  // the rows-of-1000 preference holds only where its columns are >= 64
  // points; every other candidate (short columns included: the single-radix
  // colradix_kernel takes L <= 25) is ordered by its distance from sqrt(n)
  auto pref = [n](int64_t c) { return c == 1000 && n / c >= 64; };
  std::stable_sort(cands.begin(), cands.end(), [r, pref](int64_t a, int64_t b) {
    if (pref(a) != pref(b)) return pref(a);
    return fabsl((long double)a - r) < fabsl((long double)b - r);
  });
  for (const int64_t C : cands) {
    if (!one_kernel_len(C)) continue;
    const int64_t L = n / C;
    const bool p2col = is_pow2(L) && L >= 16 && L <= 512;
    const bool rcol = !is_pow2(L) && L <= 25 && gdsp::colradix_supported((int)L);
    const bool mcol = !is_pow2(L) && L >= 26 && L <= 1016 && one_kernel_len(L);
    if (!p2col && !rcol && !mcol) continue;
    gdsp_plan *pc = nullptr;
    if (get_plan_locked(dev, C, &pc) != GDSP_OK || pc->kind != KIND_MIXED) continue;
    int rad[16], np = pc->md.npass;
    if (np < 1 || np > 16) continue;
    for (int q = 0; q < np; ++q) rad[q] = (int)((pc->md.codes >> (5 * q)) & 31);
    gdsp_plan save = *p;
    if (p2col) {
      p->pow2col = true;
      p->n1 = L;
      p->n2 = C;
      if (get_plan_locked(dev, L, &p->p1) != GDSP_OK) {
        *p = save;
        continue;
      }
    } else if (rcol) {
      p->radixcol = true;
      p->n1 = L;
      p->n2 = C;
    } else if (!mixcol_try(dev, n, L, p)) {
      continue;
    }
    gdsp::JitRowT *rt = gdsp::jit_rowt_build(dev, rad, np);
    if (!rt) {
      *p = save;  // (a built column kernel stays cached in the JIT module list)
      continue;
    }
    p->rowt = rt;
    p->rowst = true;
    return true;
  }
  return false;
}


bool fourstep2_applies(int ln);  // (exec_fourstep2 below)

bool is_prime64(int64_t n) {
  if (n < 2) return false;
  for (int64_t d = 2; d * d <= n; ++d)
    if (n % d == 0) return false;
  return true;
}

int64_t pow_mod(int64_t b, int64_t e, int64_t m) {
  int64_t r = 1 % m;
  b %= m;
  for (; e > 0; e >>= 1) {
    if (e & 1) r = r * b % m;
    b = b * b % m;
  }
  return r;
}

// smallest primitive root of the prime p
int64_t primitive_root(int64_t p) {
  std::vector<int64_t> f;
  int64_t m = p - 1;
  for (int64_t d = 2; d * d <= m; ++d)
    if (m % d == 0) {
      f.push_back(d);
      while (m % d == 0) m /= d;
    }
  if (m > 1) f.push_back(m);
  for (int64_t g = 2; g < p; ++g) {
    bool ok = true;
    for (int64_t q : f) ok = ok && pow_mod(g, (p - 1) / q, p) != 1;
    if (ok) return g;
  }
  return 0;
}

// Radix list of Rader's convolution length N = P - 1: the compiled
// specialisation's list where there is one, else the runtime-compiled
// choice (jit_radices); a power of 2 as radix-16 passes with the remainder
// last (FPass runs any radix dft_any has).
bool rader_radices(int64_t N, std::vector<int> &rad) {
  rad.clear();
  if (N < 2 || N > gdsp::kMixedSpecMax) return false;
  // (N = 3000: the specialisation's 25 15 8, 1.66 ms per 65 536 x 3001;
  // 8 15 25, 20 15 10, 10 10 3 10, 12 10 25 and 15 10 20 took 2.2-3.8 ms,
  // profiles/r05/rader_radix_ab.txt; the fused Pwelch's own four-pass lists
  // are slower here too: 3001 on 15 5 5 8 1.41-1.42 against 1.30-1.31 ms per
  // 2^27 samples, 4001 on 10 10 10 4 1.63 against 1.40-1.41,
  // scripts/archive/gpu_r05_raderpw.sh)
  if (is_pow2(N)) {
    int a = ilog2(N);
    while (a >= 4) {
      rad.push_back(16);
      a -= 4;
    }
    if (a) rad.push_back(1 << a);
    return true;
  }
  int fr[16], fnp = 0;
  if (gdsp::mixed_fixed_radices((int)N, fr, &fnp) || gdsp::jit_radices((int)N, fr, &fnp)) {
    rad.assign(fr, fr + fnp);
    return true;
  }
  return false;
}

// Rader's algorithm (rader_fixed_kernel, mixed_fixed.hpp) for a prime n >= 17
// whose n - 1 has a radix list: the DFT as a cyclic convolution of length
// n - 1 (two FFTs of n - 1 points in one kernel) instead of bluestein.go:68-94's
// chirp-z (FFTs of NextPowerOf2(2n - 1), or of a smaller smooth M, chirpz6k.hip).
// *built = false (and p untouched) where it does not apply or the kernel
// does not compile: the plan then takes the chirp-z below.
int rader_try(int dev, int64_t n, gdsp_plan *p, bool *built) {
  *built = false;
  if ((plan_flags() & GDSP_ALGO_NO_RADER) || !gdsp::jit_enabled() || n < 17 ||
      n > gdsp::kMixedSpecMax + 1 || !is_prime64(n))
    return GDSP_OK;
  const int64_t N = n - 1;
  std::vector<int> rad;
  if (!rader_radices(N, rad)) return GDSP_OK;
  // a radix-29 or -31 pass (dft_odd's long constant tables) costs more than
  // the chirp-z it would replace: 2729 (2728 = 8 11 31) 1.82 against 1.74 ms
  // per 2^27 samples (profiles/r05/rader_sweep.jsonl)
  for (int r : rad)
    if (r > 25) return GDSP_OK;
  // nor does a list needing more than 640 threads per transform (the largest
  // pass count over the butterflies a thread takes, as FixedGeo): 8191 (8190
  // = 15 13 7 6, 683 threads) 2.10-2.12 against 2.03-2.04 ms per 2^27
  // samples, 8009 (8008 = 13 11 7 8, 728 threads) ties (2.03-2.06 against
  // 2.08-2.17); 6007 (6006 = 13 11 7 6, 546 threads) gains 7 %
  {
    int t1 = 1;
    for (int r : rad) {
      const int64_t nb = N / r, jm = r > 16 ? 1 : 16 / r, need = (nb + jm - 1) / jm;
      if (need > t1) t1 = (int)need;
    }
    if (t1 > 640) return GDSP_OK;
  }
  gdsp::JitRader *j = gdsp::jit_rader_build(dev, rad.data(), (int)rad.size());
  if (!j) return GDSP_OK;
  gdsp_plan *pn = nullptr;  // FFT_N for bhat
  STCHK(get_plan_locked(dev, N, &pn));
  const int64_t g = primitive_root(n);
  if (!g) return fail(GDSP_ERR_INVALID, "no primitive root");
  std::vector<int> gp((size_t)N), gi((size_t)N);
  int64_t x = 1;
  for (int64_t q = 0; q < N; ++q) {
    gp[(size_t)q] = (int)x;
    x = x * g % n;
  }
  for (int64_t r = 0; r < N; ++r) gi[(size_t)r] = gp[(size_t)((N - r) % N)];
  // b[q] = W_n^ginv[q], the exponent reduced exactly, in long double
  std::vector<cd> b((size_t)N);
  for (int64_t q = 0; q < N; ++q) {
    const long double a =
        -2.0L * 3.141592653589793238462643383279502884L * (long double)gi[(size_t)q] / (long double)n;
    b[(size_t)q] = {(double)cosl(a), (double)sinl(a)};
  }
  // The tables are built into locals and given to p only when every step
  // succeeded; a failure frees them and leaves p untouched.
  hipStream_t s = thread_stream(dev);
  gdsp::MixedDesc d{};
  cd *tw = nullptr, *bh = nullptr, *db = nullptr;
  int *dgp = nullptr, *dgi = nullptr;
  auto release = [&] {
    if (tw) (void)hipFree(tw);
    if (bh) (void)hipFree(bh);
    if (db) (void)hipFree(db);
    if (dgp) (void)hipFree(dgp);
    if (dgi) (void)hipFree(dgi);
  };
  int st = make_mixed_desc(dev, N, rad, d, &tw);
  auto hip_ok = [&](hipError_t e) {
    if (st == GDSP_OK && e != hipSuccess) st = fail(GDSP_ERR_HIP, hipGetErrorString(e));
    return st == GDSP_OK;
  };
  if (st == GDSP_OK && hip_ok(hipMalloc((void **)&dgp, (size_t)N * sizeof(int))) &&
      hip_ok(hipMalloc((void **)&dgi, (size_t)N * sizeof(int))) &&
      hip_ok(hipMalloc((void **)&bh, (size_t)N * sizeof(cd))) &&
      hip_ok(hipMalloc((void **)&db, (size_t)N * sizeof(cd)))) {
    st = copy_h2d(dgp, gp.data(), (size_t)N * sizeof(int), s);
    if (st == GDSP_OK) st = copy_h2d(dgi, gi.data(), (size_t)N * sizeof(int), s);
    if (st == GDSP_OK) st = copy_h2d(db, b.data(), (size_t)N * sizeof(cd), s);
    // FFT_N(b) on the device with the engine itself, with the inverse's 1/N
    if (st == GDSP_OK) st = exec_plan(pn, db, bh, 1, false, gdsp::LOAD_COMPLEX, s);
    if (st == GDSP_OK) {
      hipError_t e = gdsp::launch_scale(bh, N, 1.0 / (double)N, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      hip_ok(e);
    }
  }
  if (st != GDSP_OK) {
    (void)hipStreamSynchronize(s);  // nothing in flight reads the tables any more
    release();
    return st;
  }
  (void)hipFree(db);
  p->kind = KIND_RADER;
  p->rader = j;
  p->tw = tw;
  p->md = d;
  p->m = N;
  p->gpow = dgp;
  p->ginv = dgi;
  p->bhat = bh;
  *built = true;
  return GDSP_OK;
}

// Plan-time race of two ways to run a batched transform of n, where the cost
// model cannot rank them (the prime-factor Rader kernel against the chirp-z
// plan it would replace; the smooth-L chirp-z against the power-of-2 one):
// ~2^23 samples of synthetic rows, each candidate launched three times,
// alternating, on the building thread's stream; *a_wins = a's fastest launch
// < margin x b's. Plans are built once per (device, n, flags), so this costs
// a few milliseconds once. Where the scratch cannot be had, a wins (the
// model's candidate); GDSP_ALGO_NO_RACE skips the race the same way.
using Runner = std::function<int(const cd *in, cd *out, int64_t batch, hipStream_t s)>;
int race(int dev, int64_t n, const Runner &a, const Runner &b, double margin, bool *a_wins) {
  *a_wins = true;
  if (plan_flags() & GDSP_ALGO_NO_RACE) return GDSP_OK;
  hipStream_t s = thread_stream(dev);
  const int64_t batch = std::max<int64_t>(1, ((int64_t)1 << 23) / n);
  const size_t bytes = (size_t)batch * (size_t)n * sizeof(cd);
  cd *in = nullptr, *out = nullptr;
  if (hipMalloc((void **)&in, bytes) != hipSuccess) return GDSP_OK;
  if (hipMalloc((void **)&out, bytes) != hipSuccess) {
    (void)hipFree(in);
    return GDSP_OK;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float best[2] = {1e30f, 1e30f};
  int st = GDSP_OK;
  hipError_t he = hipEventCreate(&e0);
  if (he == hipSuccess) he = hipEventCreate(&e1);
  if (he == hipSuccess)
    he = gdsp::launch_fill_uniform(reinterpret_cast<double *>(in), 2 * batch * n, 0x5EED, 0, s);
  if (he != hipSuccess) st = fail(GDSP_ERR_HIP, hipGetErrorString(he));
  const Runner *run[2] = {&a, &b};
  for (int c = 0; c < 2 && st == GDSP_OK; ++c) st = (*run[c])(in, out, batch, s);  // warm-up
  for (int it = 0; it < 3 && st == GDSP_OK; ++it)
    for (int c = 0; c < 2 && st == GDSP_OK; ++c) {
      he = hipEventRecord(e0, s);
      if (he == hipSuccess) st = (*run[c])(in, out, batch, s);
      if (st == GDSP_OK && he == hipSuccess) he = hipEventRecord(e1, s);
      if (st == GDSP_OK && he == hipSuccess) he = hipEventSynchronize(e1);
      float ms = 0.0f;
      if (st == GDSP_OK && he == hipSuccess) he = hipEventElapsedTime(&ms, e0, e1);
      if (he != hipSuccess && st == GDSP_OK) st = fail(GDSP_ERR_HIP, hipGetErrorString(he));
      if (st == GDSP_OK) best[c] = std::min(best[c], ms);
    }
  (void)hipStreamSynchronize(s);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(in);
  (void)hipFree(out);
  if (st == GDSP_OK) *a_wins = best[0] < margin * best[1];
  return st;
}

// The device tables a plan owns (not its cached sub-plans), for a plan built
// only to be raced and dropped.
void free_plan_tables(gdsp_plan *p) {
  for (cd *t : {p->tw, p->tw_gen == p->tw ? nullptr : p->tw_gen, p->tw_pw, p->chirp, p->bhat,
                p->tw6k, p->tw_blu, p->bhat_blu})
    if (t) (void)hipFree(t);
  if (p->gpow) (void)hipFree(p->gpow);
  if (p->ginv) (void)hipFree(p->ginv);
}

// skip: the kinds a plan built as a race's alternative leaves out
enum { SKIP_RADER = 1, SKIP_PFA = 2 };
int build_plan(int dev, int64_t n, gdsp_plan *p, bool chirpz = false, int skip = 0);

// Rader's plan for a prime n (kind 7, built by rader_try) against the chirp-z
// plan n gets without it, timed (race): kept where it is 3 % faster,
// otherwise p becomes that plan. Round 5 measured Rader 1.1-2.2x faster on a
// sample of primes (profiles/r05/rader_sweep.jsonl); the race covers the
// lists it did not sample (a radix-17/19/23 pass in n - 1's list: the
// round-6 kind-8 calibration lost on those, profiles/r06/pfa_calib.jsonl).
int rader_race(int dev, int64_t n, gdsp_plan *p) {
  if (plan_flags() & GDSP_ALGO_NO_RACE) return GDSP_OK;
  gdsp_plan *alt = new gdsp_plan();
  // (no alternative to race: Rader's plan stands)
  const bool have_alt = build_plan(dev, n, alt, false, SKIP_RADER | SKIP_PFA) == GDSP_OK;
  bool rader_wins = true;
  int st = GDSP_OK;
  if (have_alt) {
    Runner rader = [&](const cd *in, cd *out, int64_t batch, hipStream_t s) -> int {
      return exec_plan(p, in, out, batch, false, gdsp::LOAD_COMPLEX, s);
    };
    Runner other = [&](const cd *in, cd *out, int64_t batch, hipStream_t s) -> int {
      return exec_plan(alt, in, out, batch, false, gdsp::LOAD_COMPLEX, s);
    };
    st = race(dev, n, rader, other, 0.97, &rader_wins);
  }
  if (st == GDSP_OK && !rader_wins) {
    free_plan_tables(p);
    *p = *alt;
  } else {
    free_plan_tables(alt);
  }
  delete alt;
  return st;
}

// A composite n <= 8192 whose largest prime factor P > 31 has a Rader plan
// and whose cofactor M = n / P (gcd(M, P) = 1) has an in-register DFT:
// rader_pfa_kernel (mixed_fixed.hpp), Good-Thomas over M x P with the M
// DFT_P as Rader convolutions of length P - 1, one kernel, on the prime P's
// plan tables — where it beats the plan n gets without it (the race; the
// prime-factor kernel loses where the Rader list has a radix-17/19/23 pass
// or the cofactor is large: 38 of 150 sampled lengths at 0.59-0.99 x the
// chirp-z time, profiles/r06/pfa_calib.jsonl, and no cost model separated
// them). *built: p is complete (kind 8, or the alternative plan where that
// won); false (p untouched): not applicable, build_plan goes on as before.
int pfa_rader_try(int dev, int64_t n, gdsp_plan *p, bool *built) {
  *built = false;
  if ((plan_flags() & GDSP_ALGO_NO_RADER) || !gdsp::jit_enabled() || n > gdsp::kMixedSpecMax ||
      is_prime64(n))
    return GDSP_OK;
  int64_t P = 1, m = n;
  for (int64_t d = 2; d * d <= m; ++d)
    while (m % d == 0) {
      P = d;
      m /= d;
    }
  if (m > 1) P = m;  // the largest prime factor
  const int64_t M = n / P;
  if (P <= 31 || M % P == 0 || !gdsp::pfa_cofactor_supported((int)M)) return GDSP_OK;
  gdsp_plan *pp = nullptr;
  STCHK(get_plan_locked(dev, P, &pp));
  if (pp->kind != KIND_RADER) return GDSP_OK;
  int rad[16];
  const int np = pp->md.npass;
  if (np < 1 || np > 16) return GDSP_OK;
  for (int q = 0; q < np; ++q) rad[q] = (int)((pp->md.codes >> (5 * q)) & 31);
  gdsp::JitRader *j = gdsp::jit_rader_pfa_build(dev, (int)M, rad, np);
  if (!j) return GDSP_OK;
  if (!(plan_flags() & GDSP_ALGO_NO_RACE)) {
    const double scale = 1.0 / (double)n;
    Runner pfa = [&](const cd *in, cd *out, int64_t batch, hipStream_t s) -> int {
      HIPCHK(gdsp::jit_launch_rader(j, false, gdsp::LOAD_COMPLEX, in, out, batch, pp->tw,
                                    pp->bhat, pp->gpow, pp->ginv, scale, s));
      return GDSP_OK;
    };
    gdsp_plan *alt = new gdsp_plan();
    // (no alternative to race: the kind-8 plan stands)
    const bool have_alt = build_plan(dev, n, alt, false, SKIP_PFA) == GDSP_OK;
    bool pfa_wins = true;
    int st = GDSP_OK;
    if (have_alt) {
      Runner other = [&](const cd *in, cd *out, int64_t batch, hipStream_t s) -> int {
        return exec_plan(alt, in, out, batch, false, gdsp::LOAD_COMPLEX, s);
      };
      // the prime-factor kernel only where it is 3 % faster: near a tie the
      // alternative (the reference's algorithm) stays
      st = race(dev, n, pfa, other, 0.97, &pfa_wins);
    }
    if (st == GDSP_OK && !pfa_wins) {
      *p = *alt;  // the alternative plan, tables and all
      delete alt;
      *built = true;
      return GDSP_OK;
    }
    free_plan_tables(alt);
    delete alt;
    STCHK(st);
  }
  p->kind = KIND_RADER_PFA;
  p->rader = j;
  p->p2 = pp;
  p->n1 = M;
  p->n2 = P;
  p->m = P - 1;
  *built = true;
  return GDSP_OK;
}

// The fused chirp-z on a smooth convolution length L >= 2n - 1
// (bluestein_fixed_kernel), tried on a complete fused chirp-z plan p on M
// (a power of 2, or the M = 16 RB 16 kernel): L where the lane-cost
// model puts it below 0.85 of M's kernel (blufix_length: n just above a
// power of 2 — 4097 <= n <= 6144 on L <= 12288 instead of 16384, ...),
// built with its own tables (b on L, bhat = FFT_L(b) / L by the engine), and
// kept where it wins the race against p as it is (3 % margin). The same
// linear convolution, hence the same DFT. GDSP_ALGO_CHIRPZ_POW2 keeps the
// power of 2; the forced chirp-z plan keeps its M.
int blufix_try(int dev, int64_t n, gdsp_plan *p, const std::vector<cd> &w) {
  if (p->kind != KIND_BLUESTEIN || p->parts != 1 || (plan_flags() & GDSP_ALGO_CHIRPZ_POW2) ||
      !gdsp::jit_enabled())
    return GDSP_OK;
  std::vector<int> now;
  if (p->c6k) {
    int rad6[4];
    now.assign(rad6, rad6 + gdsp::chirpz6k_radices(p->m, rad6));
  } else {
    int a = p->log2m;
    for (; a >= 4; a -= 4) now.push_back(16);
    if (a) now.push_back(1 << a);
  }
  int rad[4], np = 0;
  const int L = gdsp::blufix_length(n, p->m, now.data(), (int)now.size(), rad, &np);
  if (!L) return GDSP_OK;
  gdsp::JitBlu *j = gdsp::jit_blu_build(dev, n, rad, np);
  if (!j) return GDSP_OK;
  gdsp_plan *lp = nullptr;  // FFT_L for bhat
  STCHK(get_plan_locked(dev, L, &lp));
  gdsp::MixedDesc d{};
  cd *tw = nullptr, *bh = nullptr, *db = nullptr;
  STCHK(make_mixed_desc(dev, L, std::vector<int>(rad, rad + np), d, &tw));
  std::vector<cd> b((size_t)L, cd{0.0, 0.0});
  for (int64_t i = 0; i < n; ++i) {  // bluestein.go:78-85 on L
    b[(size_t)i] = w[(size_t)i];
    if (i != 0) b[(size_t)(L - i)] = w[(size_t)i];
  }
  hipStream_t s = thread_stream(dev);
  int st = GDSP_OK;
  if (hipMalloc((void **)&bh, (size_t)L * sizeof(cd)) != hipSuccess ||
      hipMalloc((void **)&db, (size_t)L * sizeof(cd)) != hipSuccess)
    st = fail(GDSP_ERR_HIP, "hipMalloc (chirp-z tables)");
  if (st == GDSP_OK) st = copy_h2d(db, b.data(), (size_t)L * sizeof(cd), s);
  if (st == GDSP_OK) st = exec_plan(lp, db, bh, 1, false, gdsp::LOAD_COMPLEX, s);
  if (st == GDSP_OK) {
    hipError_t e = gdsp::launch_scale(bh, L, 1.0 / (double)L, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) st = fail(GDSP_ERR_HIP, hipGetErrorString(e));
  }
  if (db) (void)hipFree(db);
  bool wins = true;
  if (st == GDSP_OK) {
    const double scale = 1.0 / (double)n;
    Runner smooth = [&](const cd *in, cd *out, int64_t batch, hipStream_t q) -> int {
      HIPCHK(gdsp::jit_launch_blu(j, false, gdsp::LOAD_COMPLEX, in, out, batch, tw, p->chirp, bh,
                                  scale, q));
      return GDSP_OK;
    };
    Runner now_plan = [&](const cd *in, cd *out, int64_t batch, hipStream_t q) -> int {
      return exec_plan(p, in, out, batch, false, gdsp::LOAD_COMPLEX, q);
    };
    st = race(dev, n, smooth, now_plan, 0.97, &wins);
  }
  if (st != GDSP_OK || !wins) {
    (void)hipFree(tw);
    if (bh) (void)hipFree(bh);
    return st;
  }
  p->blufix = j;
  p->tw_blu = tw;
  p->bhat_blu = bh;
  p->m_blu = L;
  p->md_blu = d;
  return GDSP_OK;
}

// skip (SKIP_RADER, SKIP_PFA): without those kinds, for the alternative a
// race times them against (rader_race, pfa_rader_try)
int build_plan(int dev, int64_t n, gdsp_plan *p, bool chirpz, int skip) {
  p->device = dev;
  p->n = n;
  if (n <= 1) {
    p->kind = KIND_TRIVIAL;
    return GDSP_OK;
  }
  if (is_pow2(n) && !chirpz) {
    p->log2n = ilog2(n);
    p->kind = p->log2n <= gdsp::kMaxLdsLog2 ? KIND_LDS : KIND_GLOBAL;
    return upload_twiddles(dev, n, &p->tw);
  }
  std::vector<int> rad;
  int fr[16], fnp = 0;
  if (!chirpz && n <= gdsp::kMixedSpecMax && !gdsp::mixed_fixed_radices((int)n, fr, &fnp) &&
      gdsp::jit_enabled()) {
    // smooth length without a compiled specialisation: compile one (hipRTC);
    // if that fails it takes the runtime-radix kernel or Bluestein below
    int jr[5], jnp = 0;
    if (gdsp::jit_radices((int)n, jr, &jnp)) {
      if (gdsp::JitSpec *j = gdsp::jit_spec_build(dev, jr, jnp, (int)n)) {
        p->jit = j;
        return build_mixed(dev, n, std::vector<int>(jr, jr + jnp), p);
      }
    }
  }
  if (!chirpz && mixed_radices(n, rad)) return build_mixed(dev, n, rad, p);
  if (!chirpz && next_pow2_ref(2 * n - 1) > ((int64_t)1 << gdsp::kMaxLdsLog2) &&
      (pow2rows_build(dev, n, p) || mixrows_build(dev, n, p))) {
    p->kind = KIND_MIXED4;
    STCHK(get_plan_locked(dev, p->n2, &p->p2));
    return upload_twiddles(dev, n, &p->tw);
  }
  if (!chirpz && next_pow2_ref(2 * n - 1) > ((int64_t)1 << gdsp::kMaxLdsLog2) &&
      pow2col_split(n, p->n1, p->n2)) {
    // n = 2^a * C with 2^a in [16, 512] and C a one-kernel length: the
    // power-of-2 four-step structure (column tiles, rows of C, transpose)
    p->kind = KIND_MIXED4;
    p->pow2col = true;
    STCHK(get_plan_locked(dev, p->n1, &p->p1));
    STCHK(get_plan_locked(dev, p->n2, &p->p2));
    return upload_twiddles(dev, n, &p->tw);
  }
  if (!chirpz && next_pow2_ref(2 * n - 1) > ((int64_t)1 << gdsp::kMaxLdsLog2) &&
      radixcol_split(n, p->n1, p->n2)) {
    p->kind = KIND_MIXED4;
    p->radixcol = true;
    STCHK(get_plan_locked(dev, p->n2, &p->p2));
    return upload_twiddles(dev, n, &p->tw);
  }
  if (!chirpz && next_pow2_ref(2 * n - 1) > ((int64_t)1 << gdsp::kMaxLdsLog2) &&
      mixcol_build(dev, n, p)) {
    // the same three-launch structure with a runtime-compiled column pass
    p->kind = KIND_MIXED4;
    STCHK(get_plan_locked(dev, p->n2, &p->p2));
    return upload_twiddles(dev, n, &p->tw);
  }
  if (!chirpz && next_pow2_ref(2 * n - 1) > ((int64_t)1 << gdsp::kMaxLdsLog2) &&
      mixed4_split(n, p->n1, p->n2)) {
    // smooth n beyond one kernel, where Bluestein would be the composed
    // multi-pass chain: four-step over one-kernel factors (5 passes; 3-3.5x
    // faster than composed chirp-z at 10^4..10^6, while the fused chirp-z
    // kernel still wins for n <= 8192: 3.5 vs 6.3 ms at n = 5000)
    p->kind = KIND_MIXED4;
    STCHK(get_plan_locked(dev, p->n1, &p->p1));
    STCHK(get_plan_locked(dev, p->n2, &p->p2));
    return upload_twiddles(dev, n, &p->tw);
  }
  if (!chirpz) {
    bool built = false;
    if (!(skip & SKIP_RADER)) {
      STCHK(rader_try(dev, n, p, &built));
      if (built) return rader_race(dev, n, p);
    }
    if (!(skip & SKIP_PFA)) {
      STCHK(pfa_rader_try(dev, n, p, &built));
      if (built) return GDSP_OK;
    }
  }
  // Bluestein factors, bluestein.go:32-61: w_k = (cos, sin)(Pi/n * k*k),
  // k = 0 exactly 1 (angle not reduced, as the reference computes it).
  p->m = next_pow2_ref(2 * n - 1);
  p->log2m = ilog2(p->m);
  p->kind = p->log2m <= gdsp::kMaxLdsLog2 ? KIND_BLUESTEIN : KIND_BLUESTEIN_COMPOSED;
  if (p->kind == KIND_BLUESTEIN_COMPOSED && !chirpz && !p->mplan) {
    // Output-split chirp-z: X[k0 + k] for k < kpart needs a circular
    // convolution of length >= n + kpart - 1 only (bluestein.go:70 sizes it for
    // all n outputs, 2n - 1), so P parts of kpart = ceil(n/P) run on the
    // one-kernel M = 16384 wherever n + kpart - 1 <= 16384 with P <= 8
    // (n <= 14563); the composed chirp-z over 32768 moves ~8 HBM passes of M
    // per transform. GDSP_ALGO_NO_CHIRPZ_PARTS keeps the composed path.
    if (const int parts = chirpz_parts(n)) {
      p->m = (int64_t)1 << gdsp::kMaxLdsLog2;
      p->log2m = gdsp::kMaxLdsLog2;
      p->kind = KIND_BLUESTEIN;
      p->parts = parts;
      p->kpart = (n + parts - 1) / parts;
    }
  }
  p->unfused = (plan_flags() & GDSP_ALGO_CHIRPZ_UNFUSED) != 0;
  if (p->kind == KIND_BLUESTEIN_COMPOSED && !chirpz &&
      !(plan_flags() & GDSP_ALGO_CHIRPZ_POW2)) {
    // The composed chirp-z is HBM-bound, so its cost follows M: take the
    // smallest M >= 2n - 1 with a three-pass split (power-of-2 or
    // single-radix columns, one-kernel rows) instead of bluestein.go:70's
    // power of 2; the convolution, hence the DFT, is the same. Only where it
    // measured faster: M <= 0.55 of a power of 2 <= 2^16 (8209: 19.5 vs 22.1
    // ms, 16411: 19.4 vs 21.3; 10007, 65537, 100003 were slower), and only
    // where the power of 2 has no two-pass FFT (exec_fourstep2, 2^15..2^20):
    // against it the smooth M lost (16411 15.6 vs 9.9 ms per 2^27 samples
    // with the premultiply folded in; profiles/r04/fourstep2_ab.txt).
    // The forced chirp-z plan keeps the reference's M for the composed
    // chirp-z (the fused one at 1025..1536 / 2049..3072 takes M = 3072 / 6144
    // below).
    for (int64_t m = 2 * n - 1;
         p->m <= 65536 && !fourstep2_applies(ilog2(p->m)) && m <= (p->m * 11) / 20; ++m) {
      int64_t r = 0, c = 0;
      if (pow2col_split(m, r, c) || radixcol_split(m, r, c)) {
        gdsp_plan *mp = nullptr;
        if (get_plan_locked(dev, m, &mp) == GDSP_OK && mp->kind == KIND_MIXED4 &&
            (mp->pow2col || mp->radixcol)) {
          p->m = m;
          p->log2m = 0;
          p->mplan = mp;
        }
        break;
      }
    }
  }
  bool c6k_ok = !(plan_flags() & GDSP_ALGO_CHIRPZ_POW2);
  if (p->kind == KIND_BLUESTEIN && p->parts == 1 && gdsp::chirpz6k_m(n) && c6k_ok) {
    // 129 <= n <= 3200: bluestein.go:70 pads the convolution to
    // NextPowerOf2(2n - 1); the smallest M = 16 * RB * 16 >= 2n - 1 of the
    // kept RB gives the same linear convolution (and DFT) on up to 44 %
    // fewer points (chirpz6k.hip). GDSP_ALGO_CHIRPZ_POW2 keeps the power of 2.
    p->m = gdsp::chirpz6k_m(n);
    p->log2m = 0;
    p->c6k = true;
    gdsp::MixedDesc d6{};
    int rad6[4];
    const int np6 = gdsp::chirpz6k_radices(p->m, rad6);
    STCHK(make_mixed_desc(dev, p->m, std::vector<int>(rad6, rad6 + np6), d6, &p->tw6k, false));
  }
  if (!p->mplan) STCHK(get_plan_locked(dev, p->m, &p->mplan));
  std::vector<cd> w((size_t)n), chirp((size_t)n),
      b((size_t)p->m * (size_t)p->parts, cd{0.0, 0.0});
  for (int64_t k = 0; k < n; ++k) {
    double sn = 0.0, cs = 1.0;
    if (k != 0) {
      const double ang = M_PI / (double)n * (double)(k * k);
      sn = sin(ang);
      cs = cos(ang);
    }
    w[(size_t)k] = {cs, sn};
    chirp[(size_t)k] = {cs, -sn};
  }
  if (p->parts == 1) {
    for (int64_t i = 0; i < n; ++i) {  // bluestein.go:78-85
      b[(size_t)i] = w[(size_t)i];
      if (i != 0) b[(size_t)(p->m - i)] = w[(size_t)i];
    }
  } else {
    // part q: c[j mod M] = w_(k0 + j), j in [-(n-1), kpart-1], k0 = q kpart
    // (w_(-i) = w_i; indices k0 + j >= n feed no wanted output)
    for (int q = 0; q < p->parts; ++q) {
      cd *c = b.data() + (size_t)q * (size_t)p->m;
      const int64_t k0 = q * p->kpart;
      for (int64_t j = -(n - 1); j < p->kpart; ++j) {
        const int64_t i = k0 + j < 0 ? -(k0 + j) : k0 + j;
        if (i < n) c[(size_t)(j < 0 ? p->m + j : j)] = w[(size_t)i];
      }
    }
  }
  const size_t nb = (size_t)p->m * (size_t)p->parts;
  HIPCHK(hipMalloc((void **)&p->chirp, (size_t)n * sizeof(cd)));
  hipStream_t s = thread_stream(dev);
  STCHK(copy_h2d(p->chirp, chirp.data(), (size_t)n * sizeof(cd), s));
  HIPCHK(hipMalloc((void **)&p->bhat, nb * sizeof(cd)));
  cd *db = nullptr;
  HIPCHK(hipMalloc((void **)&db, nb * sizeof(cd)));
  STCHK(copy_h2d(db, b.data(), nb * sizeof(cd), s));
  // FFT_M(b) on the device with the engine itself, then fold the IFFT's 1/M
  int st = exec_plan(p->mplan, db, p->bhat, p->parts, false, gdsp::LOAD_COMPLEX, s);
  if (st == GDSP_OK) {
    hipError_t e = gdsp::launch_scale(p->bhat, (int64_t)nb, 1.0 / (double)p->m, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) st = fail(GDSP_ERR_HIP, hipGetErrorString(e));
  }
  (void)hipFree(db);
  STCHK(st);
  if (!chirpz) STCHK(blufix_try(dev, n, p, w));
  return GDSP_OK;
}

int get_plan_locked(int dev, int64_t n, gdsp_plan **out, bool chirpz = false) {
  auto &cache = chirpz ? g_chirpz_plans : g_plans;
  auto key = std::make_tuple(dev, n, plan_flags());
  auto it = cache.find(key);
  if (it != cache.end()) {
    *out = it->second;
    return GDSP_OK;
  }
  gdsp_plan *p = new gdsp_plan();
  struct Depth {  // leaves the snapshot on every exit, exceptions included
    explicit Depth(unsigned f) {
      if (t_build_depth++ == 0) t_build_flags = f;
    }
    ~Depth() { --t_build_depth; }
  };
  int st;
  {
    Depth d(std::get<2>(key));
    st = build_plan(dev, n, p, chirpz);
  }
  if (st != GDSP_OK) {
    delete p;  // device tables of a failed plan are leaked deliberately (rare)
    return st;
  }
  cache[key] = p;
  *out = p;
  return GDSP_OK;
}

int get_plan_locked(int dev, int64_t n, gdsp_plan **out) {
  return get_plan_locked(dev, n, out, false);
}

int get_plan(int64_t n, gdsp_plan **out, bool chirpz = false) {
  int dev = 0;
  STCHK(current_device(&dev));
  std::lock_guard<std::recursive_mutex> lk(g_plan_mu);
  return get_plan_locked(dev, n, out, chirpz);
}

// Large power of 2: radix-16 Stockham passes through HBM, last pass into out.
int exec_global(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
                hipStream_t s) {
  std::vector<int> radix;
  int rem = p->log2n;
  while (rem >= 4) {
    radix.push_back(16);
    rem -= 4;
  }
  if (rem) radix.push_back(1 << rem);
  const int np = (int)radix.size();
  const size_t bytes = (size_t)batch * (size_t)p->n * sizeof(cd);
  DevBuf scratch, inbuf;
  STCHK(scratch.alloc(bytes, s, SLOT_GLOBAL));
  const void *src = in;
  if (in == (const void *)out && ((np - 1) % 2 == 0)) {
    STCHK(inbuf.alloc(bytes, s, SLOT_GLOBAL_IN));
    HIPCHK(hipMemcpyAsync(inbuf.p, in, bytes, hipMemcpyDeviceToDevice, s));
    src = inbuf.p;
  }
  int log2ns = 0;
  for (int q = 0; q < np; ++q) {
    cd *dst = ((np - 1 - q) % 2 == 0) ? out : (cd *)scratch.p;
    HIPCHK(gdsp::launch_global_pass(radix[q], inv && q == 0, q == 0 ? load : gdsp::LOAD_COMPLEX,
                                    inv && q == np - 1, src, dst, p->tw, p->log2n, log2ns, batch,
                                    1.0 / (double)p->n, s));
    src = dst;
    log2ns += ilog2(radix[q]);
  }
  return GDSP_OK;
}

// Large power of 2, N = R*C (x as R rows x C columns, n = C*n1 + n2):
//   A  column DFT_R over n1 for every n2, times W_N^(n2*k1)  (tile kernel, into work)
//   B  row DFT_C over n2 for every k1, contiguous rows        (LDS kernel / recursion)
//   C  X[k1 + R*k2] = Y[k1][k2]: transpose R x C -> C x R      (into out)
// Three HBM round trips for N <= 2^22 (vs one per radix-16 pass), any batch.
int exec_plan_depth(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv,
                    int load, hipStream_t s, int depth);

void fourstep_split(int ln, int *lr, int *lc);

// 2^15 <= N <= 2^20: two HBM round trips instead of three. N = R*C with
// rows of C = 256 (512 at 2^18, 1024 from 2^19): the column pass as below,
// then the rows DFT_C with the transpose fused into their store
// (rowfft_t_kernel: a workgroup's TPW = 256 / (C / 16) rows leave as 64-256-B
// segments of X). Per 2^27 samples (profiles/r04/fourstep2_ab.txt): 2^15
// 2.10 -> 1.46 ms, 2^16 2.17 -> 1.55, 2^17 2.16 -> 1.57, 2^18 2.11 -> 1.60,
// 2^19 2.16 -> 1.88, 2^20 2.21 -> 1.90; BenchmarkFFT's one 2^20 transform
// 0.039 -> 0.031 ms.
bool fourstep2_applies(int ln) { return ln >= 15 && ln <= 20; }
int fourstep2_lc(int ln) { return ln >= 19 ? 10 : (ln >= 18 ? 9 : 8); }

int exec_fourstep2(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
                   hipStream_t s, int depth) {
  const int ln = p->log2n;
  const int lc = fourstep2_lc(ln), lr = ln - lc;
  gdsp_plan *pr = nullptr, *pcol = nullptr;
  STCHK(get_plan((int64_t)1 << lr, &pr));
  STCHK(get_plan((int64_t)1 << lc, &pcol));
  const int64_t N = p->n, R = (int64_t)1 << lr, C = (int64_t)1 << lc;
  DevBuf work;
  // (its own slot per recursion depth: as the rows of a longer four-step it
  // runs while the caller's work buffer, SLOT_FS0 + depth - 1, holds them)
  STCHK(work.alloc((size_t)batch * (size_t)N * sizeof(cd), s, (Slot)(SLOT_FS0 + depth)));
  cd *w = (cd *)work.p;
  const cd *src = (const cd *)in;
  if (load == gdsp::LOAD_REAL) {
    HIPCHK(gdsp::launch_real_to_complex((const double *)in, w, batch * N, s));
    src = w;
  }
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_colfft(lr, inv, 2, false, src + b0 * N, w + b0 * N, C, 1, 0, 1, 0, 1,
                               pr->tw, p->tw, ln, 1.0, nb, N, s));
  }
  HIPCHK(gdsp::launch_rowfft_t(lc, inv ? 1 : 0, w, out, batch * R, R, pcol->tw, 1.0 / (double)N,
                               s));
  return GDSP_OK;
}

int exec_fourstep(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
                  hipStream_t s, int depth) {
  const int ln = p->log2n;
  if (depth >= 4) return fail(GDSP_ERR_UNSUPPORTED, "transform too long");
  if (fourstep2_applies(ln)) return exec_fourstep2(p, in, out, batch, inv, load, s, depth);
  int lr, lc;
  fourstep_split(ln, &lr, &lc);
  // Few transforms: rows of 8192 leave the row pass at <= 256 workgroups, and
  // rows of 4096 (twice the rows, the column DFT twice as long) measured
  // 5-20 % faster per call at batch * 2^(ln-13) <= 256 (2^17..2^21 at batch 1:
  // 2^20 0.0275 -> 0.026 ms, 2^18 0.022 -> 0.0177; scripts/archive/dev/fs_split_ab.py,
  // profiles/r02/fs_split.jsonl); larger batches keep 8192.
  if (lc == 13 && lr + 1 <= gdsp::kColMaxLog2 && (batch << lr) <= 256) {
    lc = 12;
    lr += 1;
  }
  if (depth >= 4) return fail(GDSP_ERR_UNSUPPORTED, "transform too long");
  gdsp_plan *pr = nullptr, *pcol = nullptr;
  STCHK(get_plan((int64_t)1 << lr, &pr));
  STCHK(get_plan((int64_t)1 << lc, &pcol));
  const int64_t N = p->n, R = (int64_t)1 << lr, C = (int64_t)1 << lc;
  DevBuf work;
  STCHK(work.alloc((size_t)batch * (size_t)N * sizeof(cd), s, (Slot)(SLOT_FS0 + depth)));
  cd *w = (cd *)work.p;
  const cd *src = (const cd *)in;
  if (load == gdsp::LOAD_REAL) {
    HIPCHK(gdsp::launch_real_to_complex((const double *)in, w, batch * N, s));
    src = w;
  }
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_colfft(lr, inv, 2, false, src + b0 * N, w + b0 * N, C, 1, 0, 1, 0, 1,
                               pr->tw, p->tw, ln, 1.0, nb, N, s));
  }
  STCHK(exec_plan_depth(pcol, w, w, batch * R, false, gdsp::LOAD_COMPLEX, s, depth + 1));
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_transpose(w + b0 * N, out + b0 * N, R, C, s, nb, inv,
                                  1.0 / (double)N));
  }
  return GDSP_OK;
}

// Smooth non-power-of-2 n = N1*N2 beyond one kernel (x as N1 rows x N2
// columns, n = N2*n1 + n2, k = k1 + N1*k2), every step a one-kernel pass:
//   a  transpose x -> B (N2 x N1)                          (w1)
//   b  DFT_N1 along B's rows                               (in place)
//   c  transpose -> Y (N1 x N2), times W_N^(n2*k1)         (w2)
//   d  DFT_N2 along Y's rows                               (in place)
//   e  transpose -> X (N2 x N1), X[k1 + N1*k2] = Z[k1][k2] (out)
// Inverse: inverse sub-transforms (1/N1 * 1/N2 = 1/N) and conj(W).
// The reference runs these lengths through Bluestein (fft/bluestein.go).
// Column pass (conj in for an inverse) and rows of a three-pass mixed
// four-step plan, src -> w; the R x C -> C x R transpose is left to the caller.
int mixed4_col_rows(const gdsp_plan *p, const cd *src, cd *w, int64_t batch, bool inv,
                    hipStream_t s) {
  const int64_t N = p->n, N1 = p->n1, N2 = p->n2;
  const int lr = p->pow2col ? ilog2(N1) : 0;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    if (p->mixcol)
      HIPCHK(gdsp::jit_launch_col(p->mixcol, inv, src + b0 * N, w + b0 * N, N2, N, nb, p->p1->tw,
                                  p->tw, s));
    else if (p->radixcol)
      HIPCHK(gdsp::launch_colradix((int)N1, inv, src + b0 * N, w + b0 * N, N2, N, nb, p->tw, s));
    else
      HIPCHK(gdsp::launch_colfft(lr, inv, 2, false, src + b0 * N, w + b0 * N, N2, 1, 0, 1, 0, 1,
                                 p->p1->tw, p->tw, 0, 1.0, nb, N, s, N));
  }
  return exec_plan(p->p2, w, w, batch * N1, false, gdsp::LOAD_COMPLEX, s);
}

int exec_mixed4(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
                hipStream_t s) {
  const int64_t N = p->n, N1 = p->n1, N2 = p->n2;
  if (p->rowst) {
    // columns DFT_N1 times W_N^(col*k1) (conj in for an inverse), then rows
    // DFT_N2 (a power of 2) whose store carries the transpose (and conj +
    // 1/N for an inverse)
    DevBuf work;
    STCHK(work.alloc((size_t)batch * (size_t)N * sizeof(cd), s, SLOT_MX0));
    cd *w = (cd *)work.p;
    const cd *src = (const cd *)in;
    if (load == gdsp::LOAD_REAL) {
      HIPCHK(gdsp::launch_real_to_complex((const double *)in, w, batch * N, s));
      src = w;
    }
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
      const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
      if (p->mixcol)
        HIPCHK(gdsp::jit_launch_col(p->mixcol, inv, src + b0 * N, w + b0 * N, N2, N, nb, p->p1->tw,
                                    p->tw, s));
      else if (p->radixcol)
        HIPCHK(gdsp::launch_colradix((int)N1, inv, src + b0 * N, w + b0 * N, N2, N, nb, p->tw, s));
      else
        HIPCHK(gdsp::launch_colfft(ilog2(N1), inv, 2, false, src + b0 * N, w + b0 * N, N2, 1, 0, 1,
                                   0, 1, p->p1->tw, p->tw, 0, 1.0, nb, N, s, N));
    }
    if (p->rowt)
      HIPCHK(gdsp::jit_launch_rowt(p->rowt, inv, w, out, batch * N1, N1, p->p2->tw,
                                   1.0 / (double)N, s));
    else
      HIPCHK(gdsp::launch_rowfft_t(ilog2(N2), inv ? 1 : 0, w, out, batch * N1, N1, p->p2->tw,
                                   1.0 / (double)N, s));
    return GDSP_OK;
  }
  if (p->pow2col || p->radixcol || p->mixcol) {
    // as exec_fourstep with R = N1 (power of 2) and C = N2 (any one-kernel
    // length): column DFT_R on row-segment tiles times W_N^(col*k1) (table
    // index mod N), rows DFT_C, conj/scale-fused transpose R x C -> C x R
    DevBuf work;
    STCHK(work.alloc((size_t)batch * (size_t)N * sizeof(cd), s, SLOT_MX0));
    cd *w = (cd *)work.p;
    const cd *src = (const cd *)in;
    if (load == gdsp::LOAD_REAL) {
      HIPCHK(gdsp::launch_real_to_complex((const double *)in, w, batch * N, s));
      src = w;
    }
    STCHK(mixed4_col_rows(p, src, w, batch, inv, s));
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
      const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
      HIPCHK(gdsp::launch_transpose(w + b0 * N, out + b0 * N, N1, N2, s, nb, inv,
                                    1.0 / (double)N));
    }
    return GDSP_OK;
  }
  const size_t bytes = (size_t)batch * (size_t)N * sizeof(cd);
  DevBuf b1, b2;
  STCHK(b1.alloc(bytes, s, SLOT_MX0));
  STCHK(b2.alloc(bytes, s, SLOT_MX1));
  cd *w1 = (cd *)b1.p, *w2 = (cd *)b2.p;
  const cd *src = (const cd *)in;
  if (load == gdsp::LOAD_REAL) {
    HIPCHK(gdsp::launch_real_to_complex((const double *)in, w2, batch * N, s));
    src = w2;
  }
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_transpose(src + b0 * N, w1 + b0 * N, N1, N2, s, nb));
  }
  STCHK(exec_plan(p->p1, w1, w1, batch * N2, inv, gdsp::LOAD_COMPLEX, s));
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_transpose(w1 + b0 * N, w2 + b0 * N, N2, N1, s, nb, false, 1.0, p->tw, N,
                                  inv));
  }
  STCHK(exec_plan(p->p2, w2, w2, batch * N1, inv, gdsp::LOAD_COMPLEX, s));
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
    HIPCHK(gdsp::launch_transpose(w2 + b0 * N, out + b0 * N, N1, N2, s, nb));
  }
  return GDSP_OK;
}

// log2 of the column and row lengths exec_fourstep uses for a 2^ln FFT
void fourstep_split(int ln, int *lr, int *lc) {
  if (ln - 13 >= gdsp::kColMinLog2 && ln - 13 <= gdsp::kColMaxLog2) {
    *lc = 13;
    *lr = ln - 13;
  } else if (ln - 13 < gdsp::kColMinLog2) {
    *lr = gdsp::kColMinLog2;
    *lc = ln - *lr;
  } else {
    *lr = gdsp::kColMaxLog2;
    *lc = ln - *lr;  // rows longer than 8192 recurse
  }
}

int exec_bluestein_composed(const gdsp_plan *p, const cd *in, cd *out, int64_t batch, bool inv,
                            hipStream_t s) {
  DevBuf a;
  STCHK(a.alloc((size_t)batch * (size_t)p->m * sizeof(cd), s, SLOT_BLU));
  cd *da = (cd *)a.p;
  const bool two_pass =
      !p->unfused && p->mplan->kind == KIND_GLOBAL && fourstep2_applies(p->log2m);
  // (the two-pass form folds the premultiply into its first column pass)
  if (!two_pass) HIPCHK(gdsp::launch_chirp_premul(in, da, p->n, p->m, batch, p->chirp, inv, s));
  const gdsp_plan *mp = p->mplan;
  if (!p->unfused && mp->kind == KIND_MIXED4 && (mp->pow2col || mp->radixcol || mp->mixcol)) {
    // smooth M (a three-pass mixed four-step): the same two fused transposes
    const int64_t M = p->m;
    DevBuf work;
    STCHK(work.alloc((size_t)batch * (size_t)M * sizeof(cd), s, SLOT_MX0));
    cd *w = (cd *)work.p;
    for (int pass = 1; pass <= 2; ++pass) {
      STCHK(mixed4_col_rows(mp, da, w, batch, false, s));
      for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        if (pass == 1)
          HIPCHK(gdsp::launch_transpose_blu(w + b0 * M, da + b0 * M, mp->n1, mp->n2, nb, 1, p->n,
                                            p->bhat, false, 1.0, s));
        else
          HIPCHK(gdsp::launch_transpose_blu(w + b0 * M, out + b0 * p->n, mp->n1, mp->n2, nb, 2,
                                            p->n, p->chirp, inv, 1.0 / (double)p->n, s));
      }
    }
    return GDSP_OK;
  }
  if (two_pass) {
    // 2^15 <= M <= 2^20: both FFT_M as the two-pass four-step, the
    // premultiply in the first column pass's loads (colfft_chirp_kernel: x
    // read once, the zero padding never), the b-hat and output steps in the
    // rows' transposed store (rowfft_t_kernel modes 2 and 3): 2 + 2 passes
    // over M instead of 1 + 3 + 3
    const int lc2 = fourstep2_lc(p->log2m), lr2 = p->log2m - lc2;
    const int64_t M = p->m, R = (int64_t)1 << lr2, C = (int64_t)1 << lc2;
    gdsp_plan *pr = nullptr, *pcol = nullptr;
    STCHK(get_plan(R, &pr));
    STCHK(get_plan(C, &pcol));
    DevBuf work;
    STCHK(work.alloc((size_t)batch * (size_t)M * sizeof(cd), s, SLOT_FS0));
    cd *w = (cd *)work.p;
    for (int pass = 1; pass <= 2; ++pass) {
      for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        if (pass == 1)
          HIPCHK(gdsp::launch_colfft_chirp(lr2, inv, in + b0 * p->n, w + b0 * M, C, p->n, p->chirp,
                                           pr->tw, p->mplan->tw, nb, s));
        else
          HIPCHK(gdsp::launch_colfft(lr2, false, 2, false, da + b0 * M, w + b0 * M, C, 1, 0, 1, 0,
                                     1, pr->tw, p->mplan->tw, p->log2m, 1.0, nb, M, s));
      }
      if (pass == 1)
        HIPCHK(gdsp::launch_rowfft_t(lc2, 2, w, da, batch * R, R, pcol->tw, 1.0, s, p->bhat,
                                     p->n, false));
      else
        HIPCHK(gdsp::launch_rowfft_t(lc2, 3, w, out, batch * R, R, pcol->tw,
                                     1.0 / (double)p->n, s, p->chirp, p->n, inv));
    }
    return GDSP_OK;
  }
  int lr = 0, lc = 0;
  fourstep_split(p->log2m, &lr, &lc);
  if (!p->unfused && lc <= 13 && p->mplan->kind == KIND_GLOBAL) {
    // both FFT_M as exec_fourstep's column tiles + rows, each final
    // transpose carrying the chirp-z step after it: conj(A * bhat) into da,
    // then conj(r) * chirp into out (two passes over M fewer)
    const int64_t M = p->m, R = (int64_t)1 << lr, C = (int64_t)1 << lc;
    gdsp_plan *pr = nullptr, *pcol = nullptr;
    STCHK(get_plan(R, &pr));
    STCHK(get_plan(C, &pcol));
    DevBuf work;
    STCHK(work.alloc((size_t)batch * (size_t)M * sizeof(cd), s, SLOT_FS0));
    cd *w = (cd *)work.p;
    for (int pass = 1; pass <= 2; ++pass) {
      for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        HIPCHK(gdsp::launch_colfft(lr, false, 2, false, da + b0 * M, w + b0 * M, C, 1, 0, 1, 0, 1,
                                   pr->tw, p->mplan->tw, p->log2m, 1.0, nb, M, s));
      }
      STCHK(exec_plan_depth(pcol, w, w, batch * R, false, gdsp::LOAD_COMPLEX, s, 1));
      for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        if (pass == 1)
          HIPCHK(gdsp::launch_transpose_blu(w + b0 * M, da + b0 * M, R, C, nb, 1, p->n, p->bhat,
                                            false, 1.0, s));
        else
          HIPCHK(gdsp::launch_transpose_blu(w + b0 * M, out + b0 * p->n, R, C, nb, 2, p->n,
                                            p->chirp, inv, 1.0 / (double)p->n, s));
      }
    }
    return GDSP_OK;
  }
  STCHK(exec_plan(p->mplan, da, da, batch, false, gdsp::LOAD_COMPLEX, s));
  HIPCHK(gdsp::launch_bhat_mul_conj(da, p->m, batch, p->bhat, s));
  STCHK(exec_plan(p->mplan, da, da, batch, false, gdsp::LOAD_COMPLEX, s));
  HIPCHK(gdsp::launch_chirp_postmul(da, out, p->n, p->m, batch, p->chirp, inv,
                                    1.0 / (double)p->n, s));
  return GDSP_OK;
}

// Batched transform of `batch` rows of n on device buffers. load = LOAD_REAL
// reads float64 rows (fft.FFTReal); in == out is allowed.
int exec_plan(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv, int load,
              hipStream_t s) {
  return exec_plan_depth(p, in, out, batch, inv, load, s, 0);
}

int exec_plan_depth(const gdsp_plan *p, const void *in, cd *out, int64_t batch, bool inv,
                    int load, hipStream_t s, int depth) {
  if (batch <= 0) return GDSP_OK;
  const double scale = 1.0 / (double)(p->n > 0 ? p->n : 1);
  switch (p->kind) {
    case KIND_TRIVIAL: {
      if (p->n == 0) return GDSP_OK;
      if (load == gdsp::LOAD_REAL) {
        HIPCHK(gdsp::launch_real_to_complex((const double *)in, out, batch, s));
      } else if (in != (const void *)out) {
        HIPCHK(hipMemcpyAsync(out, in, (size_t)batch * sizeof(cd), hipMemcpyDeviceToDevice, s));
      }
      return GDSP_OK;
    }
    case KIND_MIXED:
      if (p->jit)
        HIPCHK(gdsp::jit_launch_fft(p->jit, inv, load, in, out, batch, p->tw, scale, s));
      else
        HIPCHK(gdsp::launch_fft_mixed(p->md, inv, load, in, out, batch, p->tw, scale, s));
      return GDSP_OK;
    case KIND_MIXED4:
      return exec_mixed4(p, in, out, batch, inv, load, s);
    case KIND_RADER:
      HIPCHK(gdsp::jit_launch_rader(p->rader, inv, load, in, out, batch, p->tw, p->bhat, p->gpow,
                                    p->ginv, scale, s));
      return GDSP_OK;
    case KIND_RADER_PFA: {
      const gdsp_plan *q = p->p2;  // the prime factor's Rader tables
      HIPCHK(gdsp::jit_launch_rader(p->rader, inv, load, in, out, batch, q->tw, q->bhat, q->gpow,
                                    q->ginv, scale, s));
      return GDSP_OK;
    }
    case KIND_LDS:
      HIPCHK(gdsp::launch_fft_lds(p->log2n, inv, load, lds_split_default(), in, out, batch, p->tw,
                                  scale, s));
      return GDSP_OK;
    case KIND_GLOBAL:
      if (p->log2n <= 13 + 3 * gdsp::kColMaxLog2)
        return exec_fourstep(p, in, out, batch, inv, load, s, depth);
      return exec_global(p, in, out, batch, inv, load, s);
    case KIND_BLUESTEIN:
    case KIND_BLUESTEIN_COMPOSED: {
      if (p->kind == KIND_BLUESTEIN && p->blufix) {
        HIPCHK(gdsp::jit_launch_blu(p->blufix, inv, load, in, out, batch, p->tw_blu, p->chirp,
                                    p->bhat_blu, scale, s));
        return GDSP_OK;
      }
      if (p->kind == KIND_BLUESTEIN && p->c6k) {
        // real input read by the kernel itself (no complex copy first)
        HIPCHK(gdsp::launch_chirpz6k(p->m, inv, load, in, out, p->n, batch, p->tw6k, p->chirp,
                                     p->bhat, scale, s));
        return GDSP_OK;
      }
      const cd *src = (const cd *)in;
      DevBuf tmp;
      if (load == gdsp::LOAD_REAL) {
        STCHK(tmp.alloc((size_t)batch * (size_t)p->n * sizeof(cd), s, SLOT_REAL));
        HIPCHK(gdsp::launch_real_to_complex((const double *)in, (cd *)tmp.p, batch * p->n, s));
        src = (const cd *)tmp.p;
      }
      if (p->kind == KIND_BLUESTEIN && p->parts > 1) {
        // the parts of a row run in different workgroups, so a part may
        // write the row before another has read it: in place (the four-step
        // rows, or a caller's in == out) goes through a copy of the input
        DevBuf cp;
        if ((const void *)src == (const void *)out) {
          const size_t bytes = (size_t)batch * (size_t)p->n * sizeof(cd);
          STCHK(cp.alloc(bytes, s, SLOT_PARTS));
          HIPCHK(hipMemcpyAsync(cp.p, src, bytes, hipMemcpyDeviceToDevice, s));
          src = (const cd *)cp.p;
        }
        HIPCHK(gdsp::launch_bluestein_parts(p->log2m, inv, src, out, p->n, batch, p->parts,
                                            p->kpart, p->mplan->tw, p->chirp, p->bhat, scale,
                                            s));
        return GDSP_OK;
      }
      if (p->kind == KIND_BLUESTEIN) {
        HIPCHK(gdsp::launch_bluestein(p->log2m, inv, src, out, p->n, batch, p->mplan->tw, p->chirp,
                                      p->bhat, scale, s));
        return GDSP_OK;
      }
      return exec_bluestein_composed(p, src, out, batch, inv, s);
    }
  }
  return fail(GDSP_ERR_INVALID, "bad plan kind");
}

// Host-pointer batched transform: H2D, exec, D2H, synchronise.
int host_batch(const void *x, size_t in_elem_bytes, double *out, int64_t n, int64_t batch,
               bool inv, int load) {
  if (n < 0 || batch < 0) return fail(GDSP_ERR_INVALID, "negative size");
  if (batch == 0) return GDSP_OK;
  if (n == 0) {
    if (inv) return fail(GDSP_ERR_EMPTY, "IFFT of an empty slice (index out of range)");
    return GDSP_OK;
  }
  if (!x || !out) return fail(GDSP_ERR_INVALID, "NULL pointer");
  gdsp_plan *p = nullptr;
  STCHK(get_plan(n, &p));
  hipStream_t s = thread_stream(p->device);
  if (!s) return fail(GDSP_ERR_HIP, "stream creation failed");
  const size_t in_bytes = (size_t)batch * (size_t)n * in_elem_bytes;
  const size_t out_bytes = (size_t)batch * (size_t)n * sizeof(cd);
  if (in_bytes + out_bytes <= kZeroCopyMax) {
    // small calls: the kernels read and write mapped pinned host memory
    // directly — one launch and one synchronisation instead of two copies
    ZeroCopy *zc = nullptr;
    STCHK(zero_copy_get(&zc));
    memcpy(zc->host, x, in_bytes);
    char *dbase = (char *)zc->dev;
    const int st = exec_plan(p, dbase, (cd *)(dbase + kZeroCopyOut), batch, inv, load, s);
    // drain even on failure: kernels already queued may still touch the
    // mapped buffer the next call on this thread refills
    const hipError_t se = hipStreamSynchronize(s);
    if (st != GDSP_OK) return st;
    if (se != hipSuccess)
      return fail(GDSP_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
    memcpy(out, zc->host + kZeroCopyOut, out_bytes);
    return GDSP_OK;
  }
  DevBuf din, dout;
  STCHK(din.alloc(in_bytes, s, SLOT_IN));
  STCHK(dout.alloc(out_bytes, s, SLOT_OUT));
  STCHK(copy_h2d(din.p, x, in_bytes, s));
  const int st = exec_plan(p, din.p, (cd *)dout.p, batch, inv, load, s);
  if (st != GDSP_OK) {
    (void)hipStreamSynchronize(s);  // queued copies still read the staging halves
    return st;
  }
  STCHK(copy_d2h(out, dout.p, out_bytes, s));  // returns after the stream drained
  return GDSP_OK;
}

void hann_table(int64_t L, double *r) {  // window/window.go:62-76
  if (L <= 0) return;
  if (L == 1) {
    r[0] = 1;
    return;
  }
  const int64_t N = L - 1;
  const double coef = 2 * M_PI / (double)N;
  for (int64_t i = 0; i <= N; ++i) r[i] = 0.5 * (1 - cos(coef * (double)i));
}

int segment_count(int64_t lx, int64_t size, int64_t noverlap, int64_t *count) {
  const int64_t stride = size - noverlap;  // spectral/spectral.go:22-33
  if (lx == size) {
    *count = 1;
  } else if (lx > size) {
    if (stride == 0) return fail(GDSP_ERR_DIVIDE_BY_ZERO, "integer divide by zero");
    *count = (lx - size) / stride + 1;
    if (*count < 0) return fail(GDSP_ERR_INVALID, "makeslice: len out of range");
  } else {
    *count = 0;
  }
  return GDSP_OK;
}

}  // namespace

// Configuration (launch.hpp): the deployment knobs, the development build's
// experiment switches and the algorithm flags.
namespace gdsp {
const char *knob(Knob k) {
  static const char *const names[] = {"GDSP_DEVICES",   "GDSP_MULTI_MIN_BYTES", "GDSP_JIT",
                                      "GDSP_JIT_INCLUDE", "GDSP_JIT_CACHE",     "GDSP_JIT_VERBOSE",
                                      "XDG_CACHE_HOME",  "HOME"};
  return (int)k >= 0 && (int)k < (int)(sizeof names / sizeof names[0]) ? getenv(names[k]) : nullptr;
}
// Inside a plan build (t_build_depth > 0) every reader — mixed_fixed_radices,
// pwelch_fixed_radices, jit_enabled, ... — sees the flags snapshot the plan is
// cached under (plan_flags), so a concurrent gdsp_set_algorithm cannot give
// one plan parts chosen under different flags.
unsigned algo_flags() {
  return t_build_depth > 0 ? t_build_flags : g_algo.load(std::memory_order_relaxed);
}
}  // namespace gdsp

// Forwarders for the multi-device layer (api_internal.hpp, multi.hip).
namespace gdsp_api {
int set_error(int st, const std::string &msg) { return fail(st, msg); }
hipStream_t stream_for(int dev) { return thread_stream(dev); }
int scratch(size_t bytes, hipStream_t s, ScratchSlot slot, void **p) {
  static const Slot map[] = {SLOT_IN, SLOT_AUX, SLOT_AUX2};
  DevBuf b;
  STCHK(b.alloc(bytes, s, map[slot]));
  *p = b.p;
  return GDSP_OK;
}
int h2d(void *dst, const void *src, size_t bytes, hipStream_t s) {
  return copy_h2d(dst, src, bytes, s);
}
int d2h(void *dst, const void *src, size_t bytes, hipStream_t s) {
  return copy_d2h(dst, src, bytes, s);
}
int batch_on_current_device(const void *x, size_t in_elem_bytes, double *out, int64_t n,
                            int64_t batch, bool inv, int load) {
  return host_batch(x, in_elem_bytes, out, n, batch, inv, load);
}
void hann(int64_t L, double *out) { hann_table(L, out); }
int segments(int64_t lx, int64_t size, int64_t noverlap, int64_t *count) {
  return segment_count(lx, size, noverlap, count);
}
}  // namespace gdsp_api

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

const char *gdsp_status_string(int st) {
  switch (st) {
    case GDSP_OK: return "ok";
    case GDSP_ERR_INVALID: return "invalid argument";
    case GDSP_ERR_UNEQUAL: return "arrays not of equal size";
    case GDSP_ERR_EMPTY: return "empty input array";
    case GDSP_ERR_RAGGED: return "ragged input array";
    case GDSP_ERR_DIVIDE_BY_ZERO: return "integer divide by zero";
    case GDSP_ERR_NO_DEVICE: return "no HIP device";
    case GDSP_ERR_HIP: return "HIP runtime error";
    case GDSP_ERR_NOMEM: return "out of memory";
    case GDSP_ERR_UNSUPPORTED: return "unsupported size";
  }
  return "unknown status";
}

const char *gdsp_last_error(void) { return g_last_error.c_str(); }
const char *gdsp_version(void) { return GDSP_VERSION; }

int gdsp_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int gdsp_set_algorithm(unsigned flags) {
  if (flags & ~kAlgoAll) return fail(GDSP_ERR_INVALID, "unknown algorithm flag");
  g_algo.store(flags);
  return GDSP_OK;
}

unsigned gdsp_get_algorithm(void) { return g_algo.load(); }

int gdsp_fft(const double *x, double *out, int64_t n) {
  return host_batch(x, sizeof(cd), out, n, 1, false, gdsp::LOAD_COMPLEX);
}

int gdsp_ifft(const double *x, double *out, int64_t n) {
  return host_batch(x, sizeof(cd), out, n, 1, true, gdsp::LOAD_COMPLEX);
}

int gdsp_fft_real(const double *x, double *out, int64_t n) {
  return host_batch(x, sizeof(double), out, n, 1, false, gdsp::LOAD_REAL);
}

int gdsp_ifft_real(const double *x, double *out, int64_t n) {
  if (n < 0) return fail(GDSP_ERR_INVALID, "negative size");
  if (n == 0) return fail(GDSP_ERR_EMPTY, "IFFT of an empty slice (index out of range)");
  std::vector<double> c((size_t)(2 * n), 0.0);  // dsputils.ToComplex
  for (int64_t i = 0; i < n; ++i) c[(size_t)(2 * i)] = x[i];
  return host_batch(c.data(), sizeof(cd), out, n, 1, true, gdsp::LOAD_COMPLEX);
}

// Large batches are split over the library's device set (gdsp_set_devices;
// multi.hip): parallelism stays inside the call, as in radix2.go:89-151.
int gdsp_fft_batch(const double *x, double *out, int64_t n, int64_t batch, int inverse) {
  if (n > 0 && gdsp_api::multi_wanted((size_t)n * (size_t)batch * sizeof(cd), batch))
    return gdsp_api::fft_batch_multi(x, sizeof(cd), out, n, batch, inverse != 0,
                                     gdsp::LOAD_COMPLEX, nullptr, 0);
  return host_batch(x, sizeof(cd), out, n, batch, inverse != 0, gdsp::LOAD_COMPLEX);
}

int gdsp_fft_real_batch(const double *x, double *out, int64_t n, int64_t batch) {
  if (n > 0 && gdsp_api::multi_wanted((size_t)n * (size_t)batch * sizeof(double), batch))
    return gdsp_api::fft_batch_multi(x, sizeof(double), out, n, batch, false, gdsp::LOAD_REAL,
                                     nullptr, 0);
  return host_batch(x, sizeof(double), out, n, batch, false, gdsp::LOAD_REAL);
}

int gdsp_convolve(const double *x, const double *y, double *out, int64_t n) {
  // fft.Convolve, fft/fft.go:55-69: IFFT(FFT(x) * FFT(y))
  if (n < 0) return fail(GDSP_ERR_INVALID, "negative size");
  if (n == 0) return fail(GDSP_ERR_EMPTY, "IFFT of an empty slice (index out of range)");
  if (!x || !y || !out) return fail(GDSP_ERR_INVALID, "NULL pointer");
  gdsp_plan *p = nullptr;
  STCHK(get_plan(n, &p));
  hipStream_t s = thread_stream(p->device);
  const size_t bytes = (size_t)n * sizeof(cd);
  DevBuf d;
  STCHK(d.alloc(3 * bytes, s, SLOT_IN));
  cd *dx = (cd *)d.p, *dy = dx + n, *dz = dy + n;
  STCHK(copy_h2d(dx, x, bytes, s));
  STCHK(copy_h2d(dy, y, bytes, s));
  STCHK(exec_plan(p, dx, dx, 2, false, gdsp::LOAD_COMPLEX, s));  // both rows at once
  HIPCHK(gdsp::launch_pointwise_mul(dx, dy, dz, n, s));
  STCHK(exec_plan(p, dz, dz, 1, true, gdsp::LOAD_COMPLEX, s));
  STCHK(copy_d2h(out, dz, bytes, s));
  return GDSP_OK;
}

int gdsp_fft2_device(const void *d_in, void *d_out, int64_t rows, int64_t cols, int inverse,
                     void *d_work, void *stream) {
  // fft/fft.go:123-154: column pass (length rows, batch cols), then row pass
  if (rows <= 0) return fail(GDSP_ERR_EMPTY, "empty input array");
  if (cols < 0) return fail(GDSP_ERR_INVALID, "negative size");
  // computeFFT2's row pass calls IFFT on each empty row, which panics
  // (fft/fft.go:40, :149-151); FFT of an empty row returns it unchanged
  if (cols == 0)
    return inverse ? fail(GDSP_ERR_EMPTY, "IFFT of an empty slice (index out of range)") : GDSP_OK;
  hipStream_t s = (hipStream_t)stream;  // NULL = the null stream (HIP convention)
  int dev = 0;
  STCHK(current_device(&dev));
  gdsp_plan *pr = nullptr, *pc = nullptr;
  STCHK(get_plan(rows, &pr));
  STCHK(get_plan(cols, &pc));
  DevBuf w;
  cd *work = (cd *)d_work;
  if (!work) {
    STCHK(w.alloc((size_t)rows * (size_t)cols * sizeof(cd), s, SLOT_FFT2));
    work = (cd *)w.p;
  }
  const bool inv = inverse != 0;
  const int lr = ilog2(rows);
  if (is_pow2(rows) && lr >= gdsp::kColMinLog2 && lr <= 2 * gdsp::kColMaxLog2) {
    // row pass (contiguous rows, any length) -> work; column pass on
    // row-segment tiles: one kernel for rows <= 512, otherwise the four-step
    // split rows = R1*R2 (A in place on work, B from work into out)
    STCHK(exec_plan(pc, d_in, work, rows, inv, gdsp::LOAD_COMPLEX, s));
    const double sc = 1.0 / (double)rows;
    if (lr <= gdsp::kColMaxLog2) {
      HIPCHK(gdsp::launch_colfft(lr, inv, 0, inv, work, (cd *)d_out, cols, 1, 0, 1, 0, 1,
                                 pr->tw, nullptr, lr, sc, 1, 0, s));
    } else {
      const int l1 = lr / 2, l2 = lr - l1;  // R1 <= R2
      gdsp_plan *p1 = nullptr, *p2 = nullptr;
      STCHK(get_plan((int64_t)1 << l1, &p1));
      STCHK(get_plan((int64_t)1 << l2, &p2));
      const int64_t R1 = (int64_t)1 << l1, R2 = (int64_t)1 << l2;
      HIPCHK(gdsp::launch_colfft(l1, inv, 1, false, work, work, cols, R2, 1, R2, 1, R2, p1->tw,
                                 pr->tw, lr, 1.0, 1, 0, s));
      HIPCHK(gdsp::launch_colfft(l2, false, 0, inv, work, (cd *)d_out, cols, R1, R2, 1, 1, R1,
                                 p2->tw, nullptr, lr, sc, 1, 0, s));
    }
    return GDSP_OK;
  }
  HIPCHK(gdsp::launch_transpose((const cd *)d_in, work, rows, cols, s));
  STCHK(exec_plan(pr, work, work, cols, inv, gdsp::LOAD_COMPLEX, s));
  HIPCHK(gdsp::launch_transpose(work, (cd *)d_out, cols, rows, s));
  STCHK(exec_plan(pc, d_out, (cd *)d_out, rows, inv, gdsp::LOAD_COMPLEX, s));
  return GDSP_OK;
}

// One axis of computeFFTN (fft/fft.go:172-185): the 1-D transform of the
// `outer` x `inner` lines of length L, read from src (cur itself, or the
// caller's input for the first axis), result in cur; other is scratch.
static int fft_axis(const cd *src, cd *cur, cd *other, int64_t L, int64_t inner, int64_t outer,
                    bool inv, hipStream_t s) {
  gdsp_plan *pl = nullptr;
  STCHK(get_plan(L, &pl));
  if (inner == 1) {
    STCHK(exec_plan(pl, src, cur, outer, inv, gdsp::LOAD_COMPLEX, s));
    return GDSP_OK;
  }
  const int lL = ilog2(L);
  const double sc = 1.0 / (double)L;
  if (is_pow2(L) && lL >= gdsp::kColMinLog2 && lL <= 2 * gdsp::kColMaxLog2) {
    const int l1 = lL <= gdsp::kColMaxLog2 ? lL : lL / 2, l2 = lL - l1;
    gdsp_plan *p1 = nullptr, *p2 = nullptr;
    STCHK(get_plan((int64_t)1 << l1, &p1));
    if (l2) STCHK(get_plan((int64_t)1 << l2, &p2));
    const int64_t R1 = (int64_t)1 << l1, R2 = (int64_t)1 << l2;
    for (int64_t o0 = 0; o0 < outer; o0 += 65535) {
      const int64_t nb = outer - o0 < 65535 ? outer - o0 : 65535;
      const cd *s0 = src + o0 * L * inner;
      cd *c0 = cur + o0 * L * inner, *t0 = other + o0 * L * inner;
      if (!l2) {
        HIPCHK(gdsp::launch_colfft(lL, inv, 0, inv, s0, c0, inner, 1, 0, 1, 0, 1, pl->tw,
                                   nullptr, lL, sc, nb, L * inner, s));
      } else {
        // A: src -> other, B: other -> cur (the result lands in cur, and
        // the caller's input is never written)
        HIPCHK(gdsp::launch_colfft(l1, inv, 1, false, s0, t0, inner, R2, 1, R2, 1, R2, p1->tw,
                                   pl->tw, lL, 1.0, nb, L * inner, s));
        HIPCHK(gdsp::launch_colfft(l2, false, 0, inv, t0, c0, inner, R1, R2, 1, 1, R1, p2->tw,
                                   nullptr, lL, sc, nb, L * inner, s));
      }
    }
    return GDSP_OK;
  }
  for (int64_t o0 = 0; o0 < outer; o0 += 65535) {
    const int64_t nb = outer - o0 < 65535 ? outer - o0 : 65535;
    HIPCHK(gdsp::launch_transpose(src + o0 * L * inner, other + o0 * L * inner, L, inner, s, nb));
  }
  STCHK(exec_plan(pl, other, other, outer * inner, inv, gdsp::LOAD_COMPLEX, s));
  for (int64_t o0 = 0; o0 < outer; o0 += 65535) {
    const int64_t nb = outer - o0 < 65535 ? outer - o0 : 65535;
    HIPCHK(gdsp::launch_transpose(other + o0 * L * inner, cur + o0 * L * inner, inner, L, s, nb));
  }
  return GDSP_OK;
}

// fft.FFTN / IFFTN (fft/fft.go:157-192): the 1-D transform along every line
// of dimension 0, then 1, ... of a row-major array. Per axis (length L,
// `inner` elements after it, `outer` before): contiguous lines (inner = 1) go
// to the batched row kernels; strided power-of-2 lines to the column-tile
// kernels batched over `outer` (one pass for L <= 512, the four-step split
// above); anything else through a batched transpose, the row kernels and a
// transpose back. axis >= 0 transforms that axis only.
static int fftn_device(const cd *in, cd *out, const int64_t *dims, int ndims, bool inv,
                       hipStream_t s, int axis = -1) {
  if (ndims < 1 || !dims) return fail(GDSP_ERR_INVALID, "no dimensions");
  if (axis >= ndims) return fail(GDSP_ERR_INVALID, "axis out of range");
  int64_t total = 1;
  for (int i = 0; i < ndims; ++i) {
    if (dims[i] < 1) return fail(GDSP_ERR_INVALID, "invalid dimensions");  // matrix.go:43
    total *= dims[i];
  }
  DevBuf work;
  STCHK(work.alloc((size_t)total * sizeof(cd), s, SLOT_FFTN));
  cd *cur = out, *other = (cd *)work.p;
  const cd *src = in;  // the first transformed axis reads the input directly
  int64_t inner = total;
  for (int d = 0; d < ndims; ++d) {
    const int64_t L = dims[d];
    inner /= L;
    const int64_t outer = total / (L * inner);
    if ((axis >= 0 && d != axis) || L == 1) continue;
    STCHK(fft_axis(src, cur, other, L, inner, outer, inv, s));
    src = cur;
  }
  if (src != out)
    HIPCHK(hipMemcpyAsync(out, src, (size_t)total * sizeof(cd), hipMemcpyDeviceToDevice, s));
  return GDSP_OK;
}

static int fft2_host(const double *x, bool real_in, double *out, int64_t rows, int64_t cols,
                     int inverse) {
  if (rows <= 0) return fail(GDSP_ERR_EMPTY, "empty input array");
  if (cols < 0) return fail(GDSP_ERR_INVALID, "negative size");
  // computeFFT2's row pass calls IFFT on each empty row, which panics
  // (fft/fft.go:40, :149-151); FFT of an empty row returns it unchanged
  if (cols == 0)
    return inverse ? fail(GDSP_ERR_EMPTY, "IFFT of an empty slice (index out of range)") : GDSP_OK;
  int dev = 0;
  STCHK(current_device(&dev));
  hipStream_t s = thread_stream(dev);
  const size_t cnt = (size_t)rows * (size_t)cols;
  DevBuf din, dout;
  STCHK(din.alloc(cnt * sizeof(cd), s, SLOT_IN));
  STCHK(dout.alloc(cnt * sizeof(cd), s, SLOT_OUT));
  if (real_in) {
    DevBuf dr;
    STCHK(dr.alloc(cnt * sizeof(double), s, SLOT_AUX));
    STCHK(copy_h2d(dr.p, x, cnt * sizeof(double), s));
    HIPCHK(gdsp::launch_real_to_complex((const double *)dr.p, (cd *)din.p, (int64_t)cnt, s));
  } else {
    STCHK(copy_h2d(din.p, x, cnt * sizeof(cd), s));
  }
  STCHK(gdsp_fft2_device(din.p, dout.p, rows, cols, inverse, nullptr, (void *)s));
  STCHK(copy_d2h(out, dout.p, cnt * sizeof(cd), s));
  return GDSP_OK;
}

int gdsp_fft2(const double *x, double *out, int64_t rows, int64_t cols, int inverse) {
  return fft2_host(x, false, out, rows, cols, inverse);
}

int gdsp_fft2_real(const double *x, double *out, int64_t rows, int64_t cols, int inverse) {
  return fft2_host(x, true, out, rows, cols, inverse);
}

int gdsp_fft_axis_device(const void *d_in, void *d_out, const int64_t *dims, int ndims,
                         int axis, int inverse, void *stream) {
  if (axis < 0) return fail(GDSP_ERR_INVALID, "axis out of range");
  int dev = 0;
  STCHK(current_device(&dev));
  return fftn_device((const cd *)d_in, (cd *)d_out, dims, ndims, inverse != 0,
                     (hipStream_t)stream, axis);
}

int gdsp_fftn_device(const void *d_in, void *d_out, const int64_t *dims, int ndims, int inverse,
                     void *stream) {
  int dev = 0;
  STCHK(current_device(&dev));
  return fftn_device((const cd *)d_in, (cd *)d_out, dims, ndims, inverse != 0,
                     (hipStream_t)stream);
}

int gdsp_fftn(const double *x, double *out, const int64_t *dims, int ndims, int inverse) {
  if (ndims < 1 || !dims || !x || !out) return fail(GDSP_ERR_INVALID, "bad argument");
  int64_t total = 1;
  for (int i = 0; i < ndims; ++i) {
    if (dims[i] < 1) return fail(GDSP_ERR_INVALID, "invalid dimensions");
    total *= dims[i];
  }
  int dev = 0;
  STCHK(current_device(&dev));
  hipStream_t s = thread_stream(dev);
  const size_t bytes = (size_t)total * sizeof(cd);
  DevBuf din, dout;
  STCHK(din.alloc(bytes, s, SLOT_IN));
  STCHK(dout.alloc(bytes, s, SLOT_OUT));
  STCHK(copy_h2d(din.p, x, bytes, s));
  STCHK(fftn_device((const cd *)din.p, (cd *)dout.p, dims, ndims, inverse != 0, s));
  STCHK(copy_d2h(out, dout.p, bytes, s));
  return GDSP_OK;
}

int gdsp_ensure_plan(int64_t n) {
  if (n < 0) return fail(GDSP_ERR_INVALID, "negative size");
  gdsp_plan *p = nullptr;
  return get_plan(n, &p);
}

void gdsp_set_worker_pool_size(int n) { g_worker_pool_size = n < 0 ? 0 : n; }
int gdsp_worker_pool_size(void) { return g_worker_pool_size; }

int gdsp_segment_count(int64_t lx, int64_t size, int64_t noverlap, int64_t *count) {
  if (!count) return fail(GDSP_ERR_INVALID, "NULL pointer");
  return segment_count(lx, size, noverlap, count);
}

int gdsp_window_hann(int64_t L, double *out) {
  if (L < 0) return fail(GDSP_ERR_INVALID, "negative size");
  hann_table(L, out);
  return GDSP_OK;
}

int gdsp_plan_create(int64_t n, gdsp_plan **plan) {
  if (n < 0 || !plan) return fail(GDSP_ERR_INVALID, "bad argument");
  return get_plan(n, plan);
}

int gdsp_plan_create_chirpz(int64_t n, gdsp_plan **plan) {
  if (n < 2 || !plan) return fail(GDSP_ERR_INVALID, "bad argument");
  return get_plan(n, plan, true);
}

int gdsp_plan_destroy(gdsp_plan *) { return GDSP_OK; }

int gdsp_plan_kind(const gdsp_plan *plan) { return plan ? plan->kind : -1; }
int gdsp_plan_parts(const gdsp_plan *plan) { return plan ? plan->parts : 0; }

int gdsp_plan_radices(const gdsp_plan *plan, int *rad, int cap) {
  if (!plan || cap < 0 || (cap > 0 && !rad)) return fail(GDSP_ERR_INVALID, "bad argument");
  const gdsp::MixedDesc *d = nullptr;
  if (plan->kind == KIND_MIXED || plan->kind == KIND_RADER) d = &plan->md;
  else if (plan->blufix) d = &plan->md_blu;
  else if (plan->kind == KIND_RADER_PFA && plan->p2) d = &plan->p2->md;
  if (!d) return 0;
  for (int q = 0; q < d->npass && q < cap; ++q) rad[q] = (int)((d->codes >> (5 * q)) & 31);
  return d->npass;
}

int gdsp_plan_info(const gdsp_plan *plan, int64_t *n, int64_t *m, int64_t *n1, int64_t *n2,
                   int *runtime_compiled) {
  if (!plan) return fail(GDSP_ERR_INVALID, "NULL plan");
  if (n) *n = plan->n;
  if (m) *m = plan->blufix ? plan->m_blu : plan->m;
  if (n1) *n1 = plan->n1;
  if (n2) *n2 = plan->n2;
  if (runtime_compiled)
    *runtime_compiled = (plan->jit || plan->mixcol || plan->rader || plan->blufix) ? 1 : 0;
  return GDSP_OK;
}

int gdsp_fft_batch_device(const gdsp_plan *plan, const void *d_in, void *d_out, int64_t batch,
                          int inverse, void *stream) {
  if (!plan || batch < 0) return fail(GDSP_ERR_INVALID, "bad argument");
  if (plan->n == 0 && inverse) return fail(GDSP_ERR_EMPTY, "IFFT of an empty slice");
  return exec_plan(plan, d_in, (cd *)d_out, batch, inverse != 0, gdsp::LOAD_COMPLEX,
                   (hipStream_t)stream);
}

int gdsp_fft_real_batch_device(const gdsp_plan *plan, const double *d_in, void *d_out,
                               int64_t batch, int inverse, void *stream) {
  if (!plan || batch < 0) return fail(GDSP_ERR_INVALID, "bad argument");
  if (plan->n == 0 && inverse) return fail(GDSP_ERR_EMPTY, "IFFT of an empty slice");
  const size_t in_bytes = (size_t)batch * (size_t)plan->n * sizeof(double);
  const char *i0 = (const char *)d_in, *o0 = (const char *)d_out;
  if (batch > 0 && plan->n > 0 && i0 < o0 + 2 * in_bytes && o0 < i0 + in_bytes)
    return fail(GDSP_ERR_INVALID, "real input overlaps the complex output");
  hipStream_t s = (hipStream_t)stream;
  if (inverse && batch > 0 && plan->n > 0) {
    // IFFTReal (fft.go:30-32 = IFFT(ToComplex(x))): the kernels read real rows
    // in the forward direction only, so widen into d_out and transform there
    HIPCHK(gdsp::launch_real_to_complex(d_in, (cd *)d_out, batch * plan->n, s));
    return exec_plan(plan, d_out, (cd *)d_out, batch, true, gdsp::LOAD_COMPLEX, s);
  }
  return exec_plan(plan, d_in, (cd *)d_out, batch, inverse != 0, gdsp::LOAD_REAL, s);
}

int gdsp_pwelch_accumulate_device(const double *d_x, int64_t n, int64_t nfft, int64_t pad,
                                  int64_t noverlap, int64_t seg_begin, int64_t seg_end,
                                  const double *d_win_seg, double *d_acc, void *stream) {
  if (nfft <= 0 || pad <= 0 || seg_begin < 0 || seg_end < seg_begin)
    return fail(GDSP_ERR_INVALID, "bad Pwelch geometry");
  if (seg_end == seg_begin) return GDSP_OK;
  const int64_t stride = nfft - noverlap;
  if ((seg_end - 1) * stride + nfft > n && seg_end > 1)
    return fail(GDSP_ERR_INVALID, "segments exceed the signal");
  const int64_t flen = pad > nfft ? pad : nfft;
  hipStream_t s = (hipStream_t)stream;  // NULL = the null stream
  gdsp_plan *p = nullptr;
  STCHK(get_plan(flen, &p));
  const int64_t nseg = seg_end - seg_begin;
  // The fused kernels address a pair's (or a wave's group of pairs') samples
  // with 32-bit offsets from one base; a very negative Noverlap (spectral.go:
  // 22-43 allows it) spreads the segments beyond that, so strides above 2^22
  // samples take the materialised path, which indexes in 64 bits.
  const bool fused = stride <= ((int64_t)1 << 22);
  if (fused && p->kind == KIND_LDS && gdsp::pwelch_wave_applies(p->log2n)) {
    // 64 <= F <= 1024: wave-resident transforms, no workgroup barriers
    // (pwelch_wave.hip), every wave a persistent worker over pair groups;
    // F = 2048: two-wave workgroups
    const bool half = 2 * noverlap == nfft && flen == nfft;
    int64_t gpw = 0, nblk = 0, nrows = 0;
    gdsp::pwelch_wave_geometry(p->log2n, half, nseg, &gpw, &nblk, &nrows);
    DevBuf part, red;
    STCHK(part.alloc((size_t)nrows * (size_t)flen * sizeof(double), s, SLOT_PW_PART));
    STCHK(red.alloc((size_t)gdsp::reduce_scratch_doubles(nrows, flen) * sizeof(double), s,
                    SLOT_PW_RED));
    HIPCHK(gdsp::launch_pwelch_wave(p->log2n, half, d_x, nfft, stride, seg_begin, seg_end, gpw,
                                    nblk, d_win_seg, p->tw, (double *)part.p, s));
    HIPCHK(gdsp::launch_reduce_partials((const double *)part.p, nrows, flen, d_acc,
                                        (double *)red.p, s));
    return GDSP_OK;
  }
  if (fused && p->kind == KIND_LDS && p->log2n >= 4) {
    // fused path: packed segment pairs, persistent workers over contiguous
    // pair ranges (the 50 % overlap of consecutive pairs is re-read from L2)
    const int64_t npairs = (nseg + 1) / 2;
    // workers per workgroup slot: 512 / 1024 / 4096 measured 2.86 / 2.81 /
    // 2.77 against 2.76 ms for 2048 (BASELINE configs[4])
    constexpr int64_t wmul = 2048;
    int64_t target = wmul * (int64_t)gdsp::pwelch_workers_per_block(p->log2n);
    if (target > npairs) target = npairs;
    const int64_t ppw = (npairs + target - 1) / target;
    const int64_t nworkers = (npairs + ppw - 1) / ppw;
    DevBuf part, red;
    STCHK(part.alloc((size_t)nworkers * (size_t)flen * sizeof(double), s, SLOT_PW_PART));
    STCHK(red.alloc((size_t)gdsp::reduce_scratch_doubles(nworkers, flen) * sizeof(double), s,
                    SLOT_PW_RED));
    if (2 * noverlap == nfft && flen == nfft && p->log2n >= 5) {
      // half overlap: each sample loaded once, window in LDS
      HIPCHK(gdsp::launch_pwelch_half(p->log2n, d_x, seg_begin, seg_end, ppw, nworkers, d_win_seg,
                                      p->tw, (double *)part.p, s));
    } else if (p->log2n == 12 && flen == nfft) {
      // any other overlap at 4096: the row kernel's structure without the carry
      HIPCHK(gdsp::launch_pwelch_rowg4096(d_x, stride, seg_begin, seg_end, ppw, nworkers,
                                          d_win_seg, p->tw, (double *)part.p, s));
    } else {
      HIPCHK(gdsp::launch_pwelch(p->log2n, d_x, nfft, stride, seg_begin, seg_end, ppw, nworkers,
                                 d_win_seg, p->tw, (double *)part.p, s));
    }
    HIPCHK(gdsp::launch_reduce_partials((const double *)part.p, nworkers, flen, d_acc,
                                        (double *)red.p, s));
    return GDSP_OK;
  }
  // the fused Pwelch on a compiled or runtime-compiled specialisation, on the
  // Pwelch's own list where it has one (md_pw); 0 workers per block where its
  // kernel cannot stage a pair this far apart (negative Noverlap)
  const bool own = p->md_pw.n > 0 && !p->jit;
  const gdsp::MixedDesc &pmd = own ? p->md_pw : p->md;
  const int wpb_fixed =
      !fused || p->kind != KIND_MIXED ? 0
      : p->jit                        ? gdsp::jit_pw_tpw(p->jit, stride + nfft)
                                      : gdsp::pwelch_fixed_workers_per_block(pmd, stride + nfft);
  if (wpb_fixed > 0 && !(gdsp::algo_flags() & GDSP_ALGO_GENERIC_MIXED)) {
    // fused path on a compiled specialisation (e.g. NFFT 1000, 3000)
    const cd *ptw = own ? p->tw_pw : p->tw;
    const int64_t npairs = (nseg + 1) / 2;
    const int wpb = wpb_fixed;
    int64_t target = 2048 * (int64_t)wpb;
    if (target > npairs) target = npairs;
    const int64_t ppw = (npairs + target - 1) / target;
    const int64_t nworkers = (npairs + ppw - 1) / ppw;
    DevBuf part, red;
    STCHK(part.alloc((size_t)nworkers * (size_t)flen * sizeof(double), s, SLOT_PW_PART));
    STCHK(red.alloc((size_t)gdsp::reduce_scratch_doubles(nworkers, flen) * sizeof(double), s,
                    SLOT_PW_RED));
    if (p->jit)
      HIPCHK(gdsp::jit_launch_pwelch(p->jit, d_x, nfft, stride, seg_begin, seg_end, ppw, nworkers,
                                     d_win_seg, p->tw, (double *)part.p, s));
    else
      HIPCHK(gdsp::launch_pwelch_fixed(pmd, d_x, nfft, stride, seg_begin, seg_end, ppw,
                                       nworkers, d_win_seg, ptw, (double *)part.p, s));
    HIPCHK(gdsp::launch_reduce_partials((const double *)part.p, nworkers, flen, d_acc,
                                        (double *)red.p, s));
    return GDSP_OK;
  }
  if (fused && p->kind == KIND_MIXED && p->md_gen.npass >= 2) {
    // fused mixed-radix path (smooth NFFT / Pad up to 4096)
    const int64_t npairs = (nseg + 1) / 2;
    int64_t target = 2048;
    if (target > npairs) target = npairs;
    const int64_t ppw = (npairs + target - 1) / target;
    const int64_t nworkers = (npairs + ppw - 1) / ppw;
    DevBuf part, red;
    STCHK(part.alloc((size_t)nworkers * (size_t)flen * sizeof(double), s, SLOT_PW_PART));
    STCHK(red.alloc((size_t)gdsp::reduce_scratch_doubles(nworkers, flen) * sizeof(double), s,
                    SLOT_PW_RED));
    HIPCHK(gdsp::launch_pwelch_mixed(p->md_gen, d_x, nfft, stride, seg_begin, seg_end, ppw,
                                     nworkers, d_win_seg, p->tw_gen, (double *)part.p, s));
    HIPCHK(gdsp::launch_reduce_partials((const double *)part.p, nworkers, flen, d_acc,
                                        (double *)red.p, s));
    return GDSP_OK;
  }
  // materialised path (lengths without a fused kernel): packed segment pairs
  // as complex rows, the batched FFT of the plan, per-bin partial power sums,
  // deterministic reduction into acc
  const int64_t nrows_all = (nseg + 1) / 2;
  int64_t rows = ((int64_t)1 << 25) / flen;  // 512 MiB of rows per chunk
  constexpr int64_t kRpp = 64;
  if (rows < 1) rows = 1;
  if (rows > 65535 * kRpp) rows = 65535 * kRpp;  // partial-sum grid limit
  if (rows > nrows_all) rows = nrows_all;
  const int64_t parts = (rows + kRpp - 1) / kRpp;
  DevBuf buf, part, red;
  STCHK(buf.alloc((size_t)rows * (size_t)flen * sizeof(cd), s, SLOT_PW_BUF));
  STCHK(part.alloc((size_t)parts * (size_t)flen * sizeof(double), s, SLOT_PW_PART));
  STCHK(red.alloc((size_t)gdsp::reduce_scratch_doubles(parts, flen) * sizeof(double), s,
                  SLOT_PW_RED));
  for (int64_t r0 = 0; r0 < nrows_all; r0 += rows) {
    const int64_t nr = (nrows_all - r0) < rows ? (nrows_all - r0) : rows;
    HIPCHK(gdsp::launch_segments_to_complex(d_x, nfft, flen, stride, seg_begin + 2 * r0, seg_end,
                                            nr, d_win_seg, (cd *)buf.p, s));
    STCHK(exec_plan(p, buf.p, (cd *)buf.p, nr, false, gdsp::LOAD_COMPLEX, s));
    HIPCHK(gdsp::launch_power_partials((const cd *)buf.p, nr, flen, kRpp, (double *)part.p, s));
    HIPCHK(gdsp::launch_reduce_partials((const double *)part.p, (nr + kRpp - 1) / kRpp, flen,
                                        d_acc, (double *)red.p, s));
  }
  return GDSP_OK;
}

int gdsp_pwelch_finalize(const double *acc, int64_t flen, int64_t nsegs, int64_t nfft,
                         int64_t pad, const double *win_nfft, double fs, int scale_off,
                         double *pxx, double *freqs) {
  // spectral/pwelch.go:113-142
  if (flen <= 0 || nfft <= 0 || pad <= 0 || !pxx || !freqs)
    return fail(GDSP_ERR_INVALID, "bad argument");
  const int64_t lp = pad / 2 + 1;
  std::vector<double> hw;
  if (!win_nfft) {
    hw.resize((size_t)nfft);
    hann_table(nfft, hw.data());
    win_nfft = hw.data();
  }
  double norm = 0;
  for (int64_t i = 0; i < nfft; ++i) norm += win_nfft[i] * win_nfft[i];
  if (!scale_off) norm *= fs;
  for (int64_t j = 0; j < lp; ++j) {
    double d = 0.0;
    if (nsegs > 0) {
      d = 0.5 * (acc[j] + acc[(flen - j) % flen]) / (double)nsegs;
      if (j > 0 && j < lp - 1) d *= 2;
    }
    pxx[j] = d / norm;
  }
  const double coef = fs / (double)pad;
  for (int64_t j = 0; j < lp; ++j) freqs[j] = (double)j * coef;
  return GDSP_OK;
}

int gdsp_pwelch(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                int64_t noverlap, const double *win_seg, const double *win_nfft, int scale_off,
                double *pxx, double *freqs, int64_t *lp_out) {
  // spectral/pwelch.go:74-145
  if (!lp_out) return fail(GDSP_ERR_INVALID, "NULL pointer");
  *lp_out = 0;
  if (n < 0) return fail(GDSP_ERR_INVALID, "negative size");
  if (n == 0) return GDSP_OK;
  if (nfft == 0) nfft = 256;
  if (pad == 0) pad = nfft;
  if (nfft < 0 || pad < 0) return fail(GDSP_ERR_INVALID, "negative NFFT/Pad");
  const int64_t lx = n < nfft ? nfft : n;  // dsputils.ZeroPadF(x, nfft)
  int64_t nsegs = 0;
  STCHK(segment_count(lx, nfft, noverlap, &nsegs));
  const int64_t flen = pad > nfft ? pad : nfft;
  const int64_t lp = pad / 2 + 1;
  std::vector<double> hseg, hnfft;
  if (!win_seg) {
    hseg.resize((size_t)flen);
    hann_table(flen, hseg.data());
    win_seg = hseg.data();
  }
  if (!win_nfft) {
    hnfft.resize((size_t)nfft);
    hann_table(nfft, hnfft.data());
    win_nfft = hnfft.data();
  }
  if (nsegs >= 2 && gdsp_api::multi_wanted((size_t)n * sizeof(double), nsegs))
    return gdsp_api::pwelch_multi(x, n, fs, nfft, pad, noverlap, win_seg, win_nfft, scale_off, pxx,
                                  freqs, lp_out, nullptr, 0);
  std::vector<double> acc((size_t)flen, 0.0);
  if (nsegs > 0) {
    int dev = 0;
    STCHK(current_device(&dev));
    hipStream_t s = thread_stream(dev);
    DevBuf dx, dw, dacc;
    STCHK(dx.alloc((size_t)lx * sizeof(double), s, SLOT_IN));
    STCHK(dw.alloc((size_t)flen * sizeof(double), s, SLOT_AUX));
    STCHK(dacc.alloc((size_t)flen * sizeof(double), s, SLOT_AUX2));
    if (lx > n) HIPCHK(hipMemsetAsync(dx.p, 0, (size_t)lx * sizeof(double), s));
    STCHK(copy_h2d(dx.p, x, (size_t)n * sizeof(double), s));
    STCHK(copy_h2d(dw.p, win_seg, (size_t)flen * sizeof(double), s));
    HIPCHK(hipMemsetAsync(dacc.p, 0, (size_t)flen * sizeof(double), s));
    STCHK(gdsp_pwelch_accumulate_device((const double *)dx.p, lx, nfft, pad, noverlap, 0, nsegs,
                                        (const double *)dw.p, (double *)dacc.p, s));
    STCHK(copy_d2h(acc.data(), dacc.p, (size_t)flen * sizeof(double), s));
  }
  STCHK(gdsp_pwelch_finalize(acc.data(), flen, nsegs, nfft, pad, win_nfft, fs, scale_off, pxx,
                             freqs));
  *lp_out = lp;
  return GDSP_OK;
}

static bool wav_format_ok(int audio_format, int bits) {
  return (audio_format == 1 && (bits == 8 || bits == 16)) || audio_format == 3;
}

static int64_t wav_sample_bytes(int audio_format, int bits) {
  return audio_format == 3 ? 4 : bits / 8;
}

int gdsp_wav_read_floats_device(const void *d_in, int64_t count, int audio_format,
                                int bits_per_sample, void *d_out, int out_f64, void *stream) {
  if (count < 0 || (count && (!d_in || !d_out))) return fail(GDSP_ERR_INVALID, "bad argument");
  if (!wav_format_ok(audio_format, bits_per_sample))
    return fail(GDSP_ERR_UNSUPPORTED, audio_format == 1 ? "wav: unknown bits per sample"
                                                        : "wav: unknown audio format");
  if (count == 0) return GDSP_OK;
  int dev = 0;
  STCHK(current_device(&dev));
  HIPCHK(gdsp::launch_wav_decode(d_in, count, audio_format, bits_per_sample, d_out, out_f64 != 0,
                                 (hipStream_t)stream));
  return GDSP_OK;
}

int gdsp_wav_read_floats(const void *in, int64_t count, int audio_format, int bits_per_sample,
                         void *out, int out_f64) {
  if (count < 0 || (count && (!in || !out))) return fail(GDSP_ERR_INVALID, "bad argument");
  if (!wav_format_ok(audio_format, bits_per_sample))
    return fail(GDSP_ERR_UNSUPPORTED, audio_format == 1 ? "wav: unknown bits per sample"
                                                        : "wav: unknown audio format");
  if (count == 0) return GDSP_OK;
  int dev = 0;
  STCHK(current_device(&dev));
  hipStream_t s = thread_stream(dev);
  if (!s) return fail(GDSP_ERR_HIP, "stream creation failed");
  const size_t in_bytes = (size_t)count * (size_t)wav_sample_bytes(audio_format, bits_per_sample);
  const size_t out_bytes = (size_t)count * (out_f64 ? 8 : 4);
  DevBuf din, dout;
  STCHK(din.alloc(in_bytes, s, SLOT_IN));
  STCHK(dout.alloc(out_bytes, s, SLOT_OUT));
  STCHK(copy_h2d(din.p, in, in_bytes, s));
  HIPCHK(gdsp::launch_wav_decode(din.p, count, audio_format, bits_per_sample, dout.p,
                                 out_f64 != 0, s));
  STCHK(copy_d2h(out, dout.p, out_bytes, s));  // returns after the stream drained
  return GDSP_OK;
}

int gdsp_fill_uniform_device(double *d_out, int64_t count, uint64_t seed, uint64_t offset,
                             void *stream) {
  if (count < 0 || (!d_out && count)) return fail(GDSP_ERR_INVALID, "bad argument");
  int dev = 0;
  STCHK(current_device(&dev));
  HIPCHK(gdsp::launch_fill_uniform(d_out, count, seed, offset, (hipStream_t)stream));
  return GDSP_OK;
}

}  // extern "C"
