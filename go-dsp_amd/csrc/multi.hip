// multi.hip — the multi-GPU layer of libgdspfft, behind the C ABI.
//
// The reference keeps all parallelism inside the library call: radix2FFT
// spreads a transform's butterflies over a goroutine pool
// (fft/radix2.go:89-151) and Pwelch folds every segment into one Pxx inside
// one loop (spectral/pwelch.go:107-122). The drop-in keeps that shape across
// the GPUs of a node, so a Go caller of fft.FFTBatch / spectral.Pwelch uses
// every GPU without a torch.distributed job:
//
//  - a batched FFT splits its rows into contiguous shards, one per device,
//    each run by a persistent host worker thread (its own stream and pinned
//    staging) through the single-device host path. Rows are independent:
//    no collective.
//  - Pwelch gives device i the segments [S*i/D, S*(i+1)/D) and the samples
//    they read ([lo*stride, (hi-1)*stride + nfft): its slice plus an
//    (nfft - stride)-sample halo); each device accumulates its per-bin power
//    sums; one in-process RCCL reduce (sum, float64, flen values) over a
//    ncclCommInitAll clique combines them on the first device, and the host
//    finalises Pxx (gdsp_pwelch_finalize). The summation order differs from
//    the reference's one segment at a time only at roundoff (non-negative
//    terms).
//
// RCCL is loaded with dlopen on the first multi-device Pwelch, so the
// library itself does not depend on it.
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>  // types and prototypes only; symbols resolved by dlopen

#include "api_internal.hpp"
#include "gdsp_fft.h"
#include "launch.hpp"

namespace {

using gdsp_api::set_error;

#define MHIPCHK(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return set_error(GDSP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define MSTCHK(expr)              \
  do {                            \
    int s_ = (expr);              \
    if (s_ != GDSP_OK) return s_; \
  } while (0)

// ---- device set -------------------------------------------------------------

std::mutex g_set_mu;
std::vector<int> g_set;  // empty: the calling thread's current device (or GDSP_DEVICES)
bool g_set_env_read = false;

// call counters for tests and diagnostics (gdsp_multi_stats)
std::atomic<int64_t> g_batch_calls{0}, g_pwelch_calls{0}, g_rccl_reduces{0}, g_host_reduces{0};

int visible_devices() {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

// A device may be listed more than once: its shards then run side by side
// on separate worker streams of that device (and a Pwelch over such a set
// combines its accumulators on the host, since an RCCL clique needs
// distinct devices).
int validate(const int *devices, int ndev, int count, std::vector<int> &out) {
  out.clear();
  for (int i = 0; i < ndev; ++i) {
    const int d = devices[i];
    if (d < 0 || d >= count)
      return set_error(GDSP_ERR_INVALID, "device " + std::to_string(d) + " not visible (" +
                                             std::to_string(count) + " devices)");
    out.push_back(d);
  }
  return GDSP_OK;
}

// GDSP_DEVICES="0,2,3" or "all": the initial device set of a process
// (deployment knob). Unset, a call uses the calling thread's current device.
void read_env_locked(int count) {
  if (g_set_env_read) return;
  g_set_env_read = true;
  const char *e = gdsp::knob(gdsp::KNOB_DEVICES);
  if (!e || !*e) return;
  std::vector<int> ids;
  if (strcmp(e, "all") == 0) {
    for (int d = 0; d < count; ++d) ids.push_back(d);
  } else {
    for (const char *p = e; *p;) {
      char *end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p) break;
      ids.push_back((int)v);
      p = *end == ',' ? end + 1 : end;
    }
  }
  std::vector<int> ok;
  if (validate(ids.data(), (int)ids.size(), count, ok) == GDSP_OK) g_set = ok;
}

// The devices of a call: the explicit list, else the library's set, else
// the calling thread's current device.
int resolve(const int *devices, int ndev, std::vector<int> &out, bool *configured = nullptr) {
  const int count = visible_devices();
  if (configured) *configured = false;
  if (count <= 0) return set_error(GDSP_ERR_NO_DEVICE, "no HIP device visible");
  if (ndev < 0) return set_error(GDSP_ERR_INVALID, "negative device count");
  if (devices && ndev > 0) return validate(devices, ndev, count, out);
  {
    std::lock_guard<std::mutex> lk(g_set_mu);
    read_env_locked(count);
    if (!g_set.empty()) {
      out = g_set;
      if (configured) *configured = true;
      return GDSP_OK;
    }
  }
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return set_error(GDSP_ERR_NO_DEVICE, "hipGetDevice failed");
  out.assign(1, cur);
  return GDSP_OK;
}

// ---- persistent per-shard host workers ----------------------------------------

// One persistent worker per (device, occurrence): the k-th time a device
// appears in a call's device list, that shard runs on worker (device, k).
// Workers persist, so their thread-local streams and pinned staging buffers
// are built once. A call holds the workers it uses for its whole duration
// (accumulate, collective, copy back), taken in one global order, so calls on
// disjoint device sets run concurrently and calls sharing a device queue.
class Pool {
 public:
  static Pool &get() {
    static Pool *p = new Pool;  // never destroyed: idle workers end with the process
    return *p;
  }

  // f(i) for shard i of devs (on worker (devs[i], occurrence)), concurrently;
  // the first failing shard's status and message become the caller's. When
  // every shard succeeded, after() runs on the calling thread while the call
  // still holds its workers (the collective step: no other call can touch
  // their streams or this device set's RCCL clique in between).
  int run(const std::vector<int> &devs, const std::function<int(int)> &f,
          const std::function<int()> &after = nullptr) {
    const int n = (int)devs.size();
    std::vector<W *> ws((size_t)n, nullptr);
    {
      std::lock_guard<std::mutex> lk(map_mu_);
      std::map<int, int> seen;
      for (int i = 0; i < n; ++i) {
        const std::pair<int, int> key(devs[i], seen[devs[i]]++);
        auto it = ws_.find(key);
        if (it == ws_.end()) {
          std::unique_ptr<W> w(new W);
          W *wp = w.get();
          try {
            wp->th = std::thread([wp] { loop(wp); });
            wp->th.detach();
          } catch (...) {
            return set_error(GDSP_ERR_NOMEM, "cannot start a device worker thread");
          }
          wp->key = key;
          it = ws_.emplace(key, std::move(w)).first;
        }
        ws[(size_t)i] = it->second.get();
      }
    }
    // the workers' call locks in one global order (map order = key order)
    std::vector<W *> order(ws);
    std::sort(order.begin(), order.end(), [](W *a, W *b) { return a->key < b->key; });
    std::vector<std::unique_lock<std::mutex>> held;
    held.reserve(order.size());
    for (W *w : order) held.emplace_back(w->call_mu);
    for (int i = 0; i < n; ++i) {
      W *w = ws[(size_t)i];
      std::lock_guard<std::mutex> lk(w->mu);
      w->f = &f;
      w->idx = i;
      w->busy = true;
      w->cv.notify_all();
    }
    int st = GDSP_OK;
    std::string msg;
    for (int i = 0; i < n; ++i) {
      W *w = ws[(size_t)i];
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [w] { return !w->busy; });
      if (st == GDSP_OK && w->st != GDSP_OK) {
        st = w->st;
        msg = w->msg;
      }
    }
    if (st != GDSP_OK) return set_error(st, msg);
    if (!after) return GDSP_OK;
    try {
      return after();
    } catch (...) {  // nothing may throw past the C ABI
      return set_error(GDSP_ERR_NOMEM, "exception in a multi-device call");
    }
  }

 private:
  struct W {
    std::pair<int, int> key;
    std::thread th;
    std::mutex call_mu;  // held by the call using this worker
    std::mutex mu;
    std::condition_variable cv;
    const std::function<int(int)> *f = nullptr;
    int idx = 0;
    bool busy = false;
    int st = GDSP_OK;
    std::string msg;
  };

  static void loop(W *w) {
    for (;;) {
      std::unique_lock<std::mutex> lk(w->mu);
      w->cv.wait(lk, [w] { return w->busy; });
      const std::function<int(int)> *f = w->f;
      const int idx = w->idx;
      lk.unlock();
      int st;
      try {
        st = (*f)(idx);
      } catch (...) {  // nothing may throw past the C ABI
        st = set_error(GDSP_ERR_NOMEM, "exception in a device worker");
      }
      const std::string msg = st == GDSP_OK ? std::string() : std::string(gdsp_last_error());
      lk.lock();
      w->st = st;
      w->msg = msg;
      w->busy = false;
      w->cv.notify_all();
    }
  }

  std::mutex map_mu_;
  std::map<std::pair<int, int>, std::unique_ptr<W>> ws_;
};

// ---- RCCL (dlopen) ----------------------------------------------------------------

struct Rccl {
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  std::string why;  // empty when loaded
};

const Rccl &rccl() {
  static Rccl r = [] {
    Rccl x;
    // the already-loaded copy first (torch maps librccl.so.1 itself)
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char *e = dlerror();
      x.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return x;
    }
    x.init_all = (decltype(x.init_all))dlsym(h, "ncclCommInitAll");
    x.reduce = (decltype(x.reduce))dlsym(h, "ncclReduce");
    x.group_start = (decltype(x.group_start))dlsym(h, "ncclGroupStart");
    x.group_end = (decltype(x.group_end))dlsym(h, "ncclGroupEnd");
    x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
    x.comm_abort = (decltype(x.comm_abort))dlsym(h, "ncclCommAbort");
    if (!x.init_all || !x.reduce || !x.group_start || !x.group_end || !x.error_string ||
        !x.comm_abort)
      x.why = "librccl.so.1 lacks an ncclCommInitAll/ncclReduce/ncclGroup*/ncclCommAbort symbol";
    return x;
  }();
  return r;
}

int nccl_fail(const Rccl &r, ncclResult_t e, const char *what) {
  return set_error(GDSP_ERR_HIP, std::string(what) + ": " + r.error_string(e));
}

// One clique per device list, built once (ncclCommInitAll) and kept until
// a collective on it fails (drop_comms).
std::mutex g_comms_mu;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;
// device lists whose clique ncclCommInitAll refused, with its message: the
// next kRefusedRetry calls on the same set go straight to the host sum
// instead of paying the failed setup again; the call after them
// tries ncclCommInitAll once more, so a transient failure does not disable
// RCCL for that set for the life of the process
struct Refusal {
  std::string why;
  int skips = 0;
};
constexpr int kRefusedRetry = 64;
std::map<std::vector<int>, Refusal> g_comms_refused;

// true: take the host sum this call (counted toward the retry)
bool clique_refused(const std::vector<int> &devs) {
  std::lock_guard<std::mutex> lk(g_comms_mu);
  auto bad = g_comms_refused.find(devs);
  if (bad == g_comms_refused.end()) return false;
  if (bad->second.skips++ < kRefusedRetry) return true;
  g_comms_refused.erase(bad);  // this call tries ncclCommInitAll again
  return false;
}

int comms_for(const std::vector<int> &devs, std::vector<ncclComm_t> **out) {
  auto &mu = g_comms_mu;
  auto &cache = g_comms;
  const Rccl &r = rccl();
  if (!r.why.empty()) return set_error(GDSP_ERR_UNSUPPORTED, r.why);
  std::lock_guard<std::mutex> lk(mu);
  auto bad = g_comms_refused.find(devs);
  if (bad != g_comms_refused.end()) return set_error(GDSP_ERR_UNSUPPORTED, bad->second.why);
  auto it = cache.find(devs);
  if (it == cache.end()) {
    std::vector<ncclComm_t> c(devs.size());
    const ncclResult_t e = r.init_all(c.data(), (int)devs.size(), devs.data());
    if (e != ncclSuccess) {
      const int st = nccl_fail(r, e, "ncclCommInitAll");
      g_comms_refused[devs] = Refusal{std::string(gdsp_last_error()), 0};
      return st;
    }
    it = cache.emplace(devs, std::move(c)).first;
  }
  *out = &it->second;
  return GDSP_OK;
}

// After a failed collective: abort every communicator of the clique (so no
// rank is left inside it) and forget it; the next call builds a new one.
void drop_comms(const std::vector<int> &devs) {
  const Rccl &r = rccl();
  std::lock_guard<std::mutex> lk(g_comms_mu);
  auto it = g_comms.find(devs);
  if (it == g_comms.end()) return;
  for (ncclComm_t c : it->second) (void)r.comm_abort(c);
  g_comms.erase(it);
}

// ---- shard geometry ----------------------------------------------------------------

void shard(int64_t total, int parts, int i, int64_t *lo, int64_t *hi) {
  // exact in 128 bits for any int64 total (total * (i+1) may overflow 64)
  *lo = (int64_t)((__int128)total * i / parts);
  *hi = (int64_t)((__int128)total * (i + 1) / parts);
}

void pwelch_shard(int64_t nsegs, int64_t nfft, int64_t noverlap, int parts, int i,
                  int64_t *seg_lo, int64_t *seg_hi, int64_t *x_lo, int64_t *x_hi) {
  shard(nsegs, parts, i, seg_lo, seg_hi);
  const int64_t stride = nfft - noverlap;
  if (*seg_hi > *seg_lo) {
    *x_lo = *seg_lo * stride;
    *x_hi = (*seg_hi - 1) * stride + nfft;
  } else {
    *x_lo = *x_hi = 0;
  }
}

int64_t multi_min_bytes() {
  static const int64_t v = [] {
    const char *e = gdsp::knob(gdsp::KNOB_MULTI_MIN_BYTES);
    const int64_t v = e ? (int64_t)strtoll(e, nullptr, 10) : 0;
    return v > 0 ? v : ((int64_t)64 << 20);
  }();
  return v;
}

}  // namespace

namespace gdsp_api {

// Automatic routing of the plain host entries is opt-in: only a configured
// set (gdsp_set_devices or GDSP_DEVICES) of more than one entry splits a
// call; by default every call stays on the caller's current device, so a
// one-rank-per-GPU job never fans out onto its neighbours' GPUs.
bool multi_wanted(size_t bytes, int64_t units) {
  if (units < 2 || (int64_t)bytes < multi_min_bytes()) return false;
  std::vector<int> devs;
  bool configured = false;
  if (resolve(nullptr, 0, devs, &configured) != GDSP_OK) return false;
  return configured && devs.size() > 1;
}

int fft_batch_multi(const void *x, size_t in_elem_bytes, double *out, int64_t n, int64_t batch,
                    bool inv, int load, const int *devices, int ndev) {
  if (n < 0 || batch < 0) return set_error(GDSP_ERR_INVALID, "negative size");
  std::vector<int> devs;
  MSTCHK(resolve(devices, ndev, devs));
  if (batch == 0 || n == 0) return batch_on_current_device(x, in_elem_bytes, out, n, batch, inv, load);
  if (!x || !out) return set_error(GDSP_ERR_INVALID, "NULL pointer");
  const int parts = (int)std::min<int64_t>((int64_t)devs.size(), batch);
  ++g_batch_calls;
  const std::vector<int> used(devs.begin(), devs.begin() + parts);
  return Pool::get().run(used, [&](int i) -> int {
    int64_t lo, hi;
    shard(batch, parts, i, &lo, &hi);
    MHIPCHK(hipSetDevice(devs[i]));
    const size_t row_in = (size_t)n * in_elem_bytes, row_out = (size_t)n * 2;
    return batch_on_current_device((const char *)x + (size_t)lo * row_in, in_elem_bytes,
                                   out + (size_t)lo * row_out, n, hi - lo, inv, load);
  });
}

// Device buffer owned by one call (the accumulators the reduce reads: never
// a worker's shared scratch, which the next call would reuse), freed on its
// own device.
struct CallBuf {
  void *p = nullptr;
  int dev = -1;
  ~CallBuf() {
    if (!p) return;
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(dev);
    (void)hipFree(p);
    if (cur >= 0) (void)hipSetDevice(cur);
  }
};

int pwelch_multi(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                 int64_t noverlap, const double *win_seg, const double *win_nfft, int scale_off,
                 double *pxx, double *freqs, int64_t *lp_out, const int *devices, int ndev) {
  // spectral/pwelch.go:74-145, segments sharded over devices
  if (!lp_out) return set_error(GDSP_ERR_INVALID, "NULL pointer");
  *lp_out = 0;
  if (n < 0) return set_error(GDSP_ERR_INVALID, "negative size");
  std::vector<int> devs;
  MSTCHK(resolve(devices, ndev, devs));
  if (n == 0) return GDSP_OK;
  if (nfft == 0) nfft = 256;
  if (pad == 0) pad = nfft;
  if (nfft < 0 || pad < 0) return set_error(GDSP_ERR_INVALID, "negative NFFT/Pad");
  if (!x || !pxx || !freqs) return set_error(GDSP_ERR_INVALID, "NULL pointer");
  const int64_t lx = n < nfft ? nfft : n;  // dsputils.ZeroPadF(x, nfft)
  int64_t nsegs = 0;
  MSTCHK(segments(lx, nfft, noverlap, &nsegs));
  const int64_t flen = pad > nfft ? pad : nfft;
  const int64_t lp = pad / 2 + 1;
  std::vector<double> hseg, hnfft;
  if (!win_seg) {
    hseg.resize((size_t)flen);
    hann(flen, hseg.data());
    win_seg = hseg.data();
  }
  if (!win_nfft) {
    hnfft.resize((size_t)nfft);
    hann(nfft, hnfft.data());
    win_nfft = hnfft.data();
  }
  std::vector<double> acc((size_t)flen, 0.0);
  if (nsegs > 0) {
    // the caller's current device is restored on every return path
    struct DeviceGuard {
      int dev = -1;
      DeviceGuard() { (void)hipGetDevice(&dev); }
      ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
      }
    } guard;
    const int D = (int)devs.size();
    // RCCL over a clique of the (distinct) devices; a set that repeats a
    // device, or a process without a usable librccl, sums the D
    // accumulators (flen float64 each) on the host in device order instead
    std::vector<int> sorted(devs);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const bool use_rccl = distinct && rccl().why.empty() && !clique_refused(devs);
    bool reduced_by_rccl = false;
    std::vector<std::vector<double>> part((size_t)D);
    std::vector<CallBuf> dacc((size_t)D);
    std::vector<hipStream_t> streams((size_t)D, nullptr);
    ++g_pwelch_calls;
    // Phase 1, on the workers: every shard accumulates into its own
    // call-owned device buffer (a failing shard reports its own status and
    // message; the others return GDSP_OK and their work is dropped).
    auto accumulate = [&](int i) -> int {
      MHIPCHK(hipSetDevice(devs[i]));
      hipStream_t s = stream_for(devs[i]);
      if (!s) return set_error(GDSP_ERR_HIP, "stream creation failed");
      streams[(size_t)i] = s;
      int64_t seg_lo, seg_hi, x_lo, x_hi;
      pwelch_shard(nsegs, nfft, noverlap, D, i, &seg_lo, &seg_hi, &x_lo, &x_hi);
      void *dx = nullptr, *dw = nullptr;
      const int64_t len = x_hi - x_lo;
      CallBuf &a = dacc[(size_t)i];
      a.dev = devs[i];
      MHIPCHK(hipMalloc(&a.p, (size_t)flen * sizeof(double)));
      MSTCHK(scratch((size_t)(len > 0 ? len : 1) * sizeof(double), s, SCRATCH_SIGNAL, &dx));
      MSTCHK(scratch((size_t)flen * sizeof(double), s, SCRATCH_WINDOW, &dw));
      MHIPCHK(hipMemsetAsync(a.p, 0, (size_t)flen * sizeof(double), s));
      if (len > 0) {
        const int64_t have = (x_hi < n ? x_hi : n) - x_lo;  // past n: ZeroPadF's zeros
        if (have < len) MHIPCHK(hipMemsetAsync(dx, 0, (size_t)len * sizeof(double), s));
        if (have > 0) MSTCHK(h2d(dx, x + x_lo, (size_t)have * sizeof(double), s));
        MSTCHK(h2d(dw, win_seg, (size_t)flen * sizeof(double), s));
        MSTCHK(gdsp_pwelch_accumulate_device((const double *)dx, len, nfft, pad, noverlap, 0,
                                             seg_hi - seg_lo, (const double *)dw,
                                             (double *)a.p, s));
      }
      if (use_rccl) return GDSP_OK;  // the reduce reads it on the same stream
      part[(size_t)i].resize((size_t)flen);
      return d2h(part[(size_t)i].data(), a.p, (size_t)flen * sizeof(double), s);
    };
    // Phase 2, on the calling thread once every shard succeeded, still inside
    // the pool's call: one grouped RCCL reduce over the clique (a single
    // thread driving several devices must group its calls), each rank on the
    // stream that produced its accumulator; root 0 receives the sum. A failed
    // group aborts the clique, so no rank stays inside the collective.
    auto reduce = [&]() -> int {
      const Rccl &r = rccl();
      std::vector<ncclComm_t> *comms = nullptr;
      const std::string prev_error(gdsp_last_error());
      if (comms_for(devs, &comms) != GDSP_OK) {
        // no clique for this set (ncclCommInitAll refused it; cached, so the
        // next call on this set skips RCCL): the accumulators come back to
        // the host and are summed there, and the call succeeds without
        // leaving the refusal as its last error
        for (int i = 0; i < D; ++i) {
          MHIPCHK(hipSetDevice(devs[i]));
          part[(size_t)i].resize((size_t)flen);
          MSTCHK(d2h(part[(size_t)i].data(), dacc[(size_t)i].p, (size_t)flen * sizeof(double),
                     streams[(size_t)i]));
        }
        return set_error(GDSP_OK, prev_error);
      }
      ncclResult_t e = r.group_start();
      if (e != ncclSuccess) return nccl_fail(r, e, "ncclGroupStart");
      ncclResult_t first = ncclSuccess;
      for (int i = 0; i < D && first == ncclSuccess; ++i) {
        if (hipSetDevice(devs[i]) != hipSuccess) {
          first = ncclUnhandledCudaError;
          break;
        }
        double *da = (double *)dacc[(size_t)i].p;
        first = r.reduce(da, da, (size_t)flen, ncclFloat64, ncclSum, 0, (*comms)[i],
                         streams[(size_t)i]);
      }
      e = r.group_end();
      if (first == ncclSuccess) first = e;
      if (first != ncclSuccess) {
        const int st = nccl_fail(r, first, "ncclReduce (grouped)");
        drop_comms(devs);
        return st;
      }
      MHIPCHK(hipSetDevice(devs[0]));
      part[0].resize((size_t)flen);
      MSTCHK(d2h(part[0].data(), dacc[0].p, (size_t)flen * sizeof(double), streams[0]));
      for (int i = 1; i < D; ++i) {
        MHIPCHK(hipSetDevice(devs[i]));
        MHIPCHK(hipStreamSynchronize(streams[(size_t)i]));
      }
      reduced_by_rccl = true;
      return GDSP_OK;
    };
    // one Pool::run holds the call's workers for the whole call (accumulate,
    // reduce, copy back): a concurrent call on an overlapping device set
    // queues behind it and never shares its accumulators, streams or clique;
    // one on a disjoint set runs beside it
    MSTCHK(Pool::get().run(devs, accumulate, use_rccl ? std::function<int()>(reduce) : nullptr));
    if (reduced_by_rccl) {
      acc.swap(part[0]);
      ++g_rccl_reduces;
    } else {
      for (int i = 0; i < D; ++i)
        for (int64_t k = 0; k < flen; ++k) acc[(size_t)k] += part[i][(size_t)k];
      ++g_host_reduces;
    }
  }
  MSTCHK(gdsp_pwelch_finalize(acc.data(), flen, nsegs, nfft, pad, win_nfft, fs, scale_off, pxx,
                              freqs));
  *lp_out = lp;
  return GDSP_OK;
}

}  // namespace gdsp_api

// ============================================================================
// C ABI (include/gdsp_fft.h, "multi-device")
// ============================================================================
extern "C" {

int gdsp_set_devices(const int *devices, int ndev) {
  if (ndev < 0 || (ndev > 0 && !devices)) return set_error(GDSP_ERR_INVALID, "bad device list");
  const int count = visible_devices();
  if (count <= 0) return set_error(GDSP_ERR_NO_DEVICE, "no HIP device visible");
  std::vector<int> v;
  MSTCHK(validate(devices, ndev, count, v));
  std::lock_guard<std::mutex> lk(g_set_mu);
  g_set_env_read = true;  // an explicit set overrides GDSP_DEVICES
  g_set = v;
  return GDSP_OK;
}

int gdsp_get_devices(int *devices, int cap) {
  std::vector<int> v;
  if (resolve(nullptr, 0, v) != GDSP_OK) return 0;
  for (int i = 0; i < cap && i < (int)v.size(); ++i) devices[i] = v[i];
  return (int)v.size();
}

int gdsp_multi_stats(int64_t *batch_calls, int64_t *pwelch_calls, int64_t *rccl_reduces,
                     int64_t *host_reduces) {
  if (batch_calls) *batch_calls = g_batch_calls.load();
  if (pwelch_calls) *pwelch_calls = g_pwelch_calls.load();
  if (rccl_reduces) *rccl_reduces = g_rccl_reduces.load();
  if (host_reduces) *host_reduces = g_host_reduces.load();
  return GDSP_OK;
}

int gdsp_batch_shard(int64_t batch, int ndev, int i, int64_t *lo, int64_t *hi) {
  if (batch < 0 || ndev <= 0 || i < 0 || i >= ndev || !lo || !hi)
    return set_error(GDSP_ERR_INVALID, "bad argument");
  shard(batch, ndev, i, lo, hi);
  return GDSP_OK;
}

int gdsp_pwelch_shard(int64_t nsegs, int64_t nfft, int64_t noverlap, int ndev, int i,
                      int64_t *seg_lo, int64_t *seg_hi, int64_t *x_lo, int64_t *x_hi) {
  if (nsegs < 0 || nfft <= 0 || noverlap < 0 || noverlap >= nfft || ndev <= 0 || i < 0 ||
      i >= ndev || !seg_lo || !seg_hi || !x_lo || !x_hi)
    return set_error(GDSP_ERR_INVALID, "bad argument");
  pwelch_shard(nsegs, nfft, noverlap, ndev, i, seg_lo, seg_hi, x_lo, x_hi);
  return GDSP_OK;
}

int gdsp_fft_batch_multi(const double *x, double *out, int64_t n, int64_t batch, int inverse,
                         const int *devices, int ndev) {
  return gdsp_api::fft_batch_multi(x, 2 * sizeof(double), out, n, batch, inverse != 0,
                                   gdsp::LOAD_COMPLEX, devices, ndev);
}

int gdsp_pwelch_multi(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                      int64_t noverlap, const double *win_seg, const double *win_nfft,
                      int scale_off, double *pxx, double *freqs, int64_t *lp_out,
                      const int *devices, int ndev) {
  return gdsp_api::pwelch_multi(x, n, fs, nfft, pad, noverlap, win_seg, win_nfft, scale_off, pxx,
                                freqs, lp_out, devices, ndev);
}

}  // extern "C"
