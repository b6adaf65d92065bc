// mixed_jit.hip — runtime-compiled mixed-radix specialisations (hipRTC).
//
// The compiled specialisations (fft_specs*.hip) inline every pass of a fixed
// radix list and run at 4.8-6 TB/s; a smooth length without one would take
// the runtime-radix kernel (2.5-4 TB/s, n <= 4096) or Bluestein (n > 4096).
// At plan creation such a length gets a radix list chosen like the compiled
// ones (as few passes as radices <= 25 allow, full waves, a power-of-2 radix
// last; at most 512 threads per transform where a list allows it, else up to
// 1024), and the same kernel templates (mixed_fixed.hpp) are compiled for it
// with hipRTC: the batched transform (forward, inverse, real input) and the
// fused Pwelch kernel, ~0.3-1.7 s once per length. Any failure (no hipRTC,
// a compile error) leaves the plan on the runtime-radix kernel or Bluestein,
// so this is a speed path only; failures are counted and the last one is
// reported by gdsp_jit_stats. GDSP_JIT=0 disables it.
//
// Deployment: the headers the compiler needs are embedded in the library
// (embed_headers.py at build time), so no source tree has to ship with it
// (GDSP_JIT_INCLUDE=<dir> compiles against headers on disk instead). Built
// code objects are kept in an on-disk cache keyed by the embedded headers'
// hash, the GPU architecture, the compiler options and the kernel names
// (GDSP_JIT_CACHE=<dir>, default $XDG_CACHE_HOME/gdspfft or
// ~/.cache/gdspfft; GDSP_JIT_CACHE=off disables it), so a second process
// creating the same plan loads it instead of compiling.
#include <dlfcn.h>
#include <errno.h>
#include <sys/stat.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "gdsp_fft.h"
#include "jit_headers.inc"
#include "launch.hpp"

namespace gdsp {

struct JitSpec {
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr, real = nullptr, pw = nullptr;
  int n = 0, wg = 0, tpw = 0;
  int pw_stage = 0;  // the fused Pwelch's LDS-DMA stage in doubles (PwfDma::STG), 0: none
};

struct JitCol {  // colfixed_kernel for one column length
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr;
  int l = 0, w = 0, wg = 0;
};
struct JitRowT {  // rowt_fixed_kernel for one row length (forward, conj + scale out)
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, cso = nullptr;
  int n = 0, w = 0, wg = 0;
};
struct JitRader {  // rader_fixed_kernel for one prime P = N + 1
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr, real = nullptr;
  int p = 0, wg = 0, tpw = 0;
};

namespace {

// the radices dft_any has (mixed_core.hpp); 17 .. 31 only here (31 is also
// the largest a 5-bit MixedDesc code holds)
constexpr int kRadices[] = {31, 29, 25, 23, 20, 19, 17, 16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2};

// FixedGeo (mixed_fixed.hpp) on the host: threads per transform, transforms
// per workgroup
void fixed_geo(const int *rad, int np, int *t1, int *tpw) {
  int n = 1;
  for (int q = 0; q < np; ++q) n *= rad[q];
  int m = 1;
  for (int q = 0; q < np; ++q) {
    const int nb = n / rad[q], jm = rad[q] > 16 ? 1 : 16 / rad[q], need = (nb + jm - 1) / jm;
    if (need > m) m = need;
  }
  const int slots = (n + 7) & ~7;
  int t = 256 / m > 1 ? 256 / m : 1;
  while (t > 1 && t * slots * 16 > 65536) --t;
  *t1 = m;
  *tpw = t;
}

struct Choice {
  int rad[5], np = 0;
  double eff = 0;
  bool pow2last = false, wide = false;  // wide: more than 512 threads per transform
  double cost = 0;                      // lane_cost
};

// F64 instructions per point of dft_any<R> (mixed_core.hpp, counted by hand;
// odd primes by dft_odd's 3 (R - 1) + H (4 H + 4), H = (R - 1) / 2)
double dft_cost(int r) {
  switch (r) {
    case 2: return 2.0;
    case 4: return 4.0;
    case 6: return 8.0;
    case 8: return 6.5;
    case 9: return 11.1;
    case 10: return 10.8;
    case 12: return 10.7;
    case 15: return 14.0;
    case 16: return 9.4;
    case 20: return 13.6;
    case 25: return 17.0;
    default: {
      const int h = (r - 1) / 2;
      return (3.0 * (r - 1) + h * (4.0 * h + 4.0)) / r;
    }
  }
}

// Cost model of a list's passes (tools/spec_candidates.py): each pass's DFT
// plus twiddle chain per point, over the share of the transform's T1
// threads its butterflies keep busy. A pass with few butterflies (a radix-25
// first pass of 80 beside a radix-5 pass of 400) idles most lanes of the
// compute-bound kernels (the fused Pwelch above all).
double lane_cost(const int *rad, int np, int t1) {
  int n = 1;
  for (int q = 0; q < np; ++q) n *= rad[q];
  double c = 0;
  for (int q = 0; q < np; ++q) {
    const int nb = n / rad[q], jj = (nb + t1 - 1) / t1;
    const double use = (double)nb / ((double)jj * t1);
    c += (dft_cost(rad[q]) + (q ? 8.0 * (rad[q] - 1) / rad[q] : 0.0)) / use;
  }
  return c;
}

bool better(const Choice &a, const Choice &b) {  // a before b?
  if (a.wide != b.wide) return !a.wide;
  if (a.np != b.np) return a.np < b.np;
  if (a.eff != b.eff) return a.eff > b.eff;
  if (a.pow2last != b.pow2last) return a.pow2last;
  return a.rad[0] > b.rad[0];
}

// best: by better(); cheap: the lowest lane_cost among the lists of this
// depth (narrow ones first)
void search(int n, int depth, int maxdepth, Choice &cur, Choice &best, Choice &cheap) {
  if (depth == maxdepth) {
    if (n != 1) return;
    int t1 = 0, tpw = 0;
    fixed_geo(cur.rad, depth, &t1, &tpw);
    if (t1 > 1024) return;
    const int wg = t1 * tpw, waves = (wg + 63) / 64;
    Choice c = cur;
    c.np = depth;
    c.wide = t1 > 512;
    c.eff = (double)wg / (waves * 64);
    const int last = cur.rad[depth - 1];
    c.pow2last = (last & (last - 1)) == 0;
    c.cost = lane_cost(cur.rad, depth, t1);
    if (best.np == 0 || better(c, best)) best = c;
    if (cheap.np == 0 || c.wide < cheap.wide ||
        (c.wide == cheap.wide && c.cost < cheap.cost))
      cheap = c;
    return;
  }
  for (int r : kRadices) {
    if (n % r) continue;
    cur.rad[depth] = r;
    search(n / r, depth + 1, maxdepth, cur, best, cheap);
  }
}

// GDSP_JIT_INCLUDE: compile against headers on disk (empty: the embedded ones)
std::string include_dir() {
  const char *e = knob(KNOB_JIT_INCLUDE);
  return e ? e : "";
}

// ---- statistics (gdsp_jit_stats) ----------------------------------------------
std::atomic<int64_t> g_built{0}, g_cached{0}, g_failed{0};
std::mutex g_fail_mu;
std::string g_last_failure;

void record_failure(const std::string &what, const std::string &why) {
  ++g_failed;
  std::lock_guard<std::mutex> lk(g_fail_mu);
  g_last_failure = what + ": " + why;
}

// ---- on-disk code-object cache -------------------------------------------------
uint64_t fnv1a(const std::string &s, uint64_t h) {
  for (unsigned char c : s) h = (h ^ c) * 0x100000001B3ULL;
  return h;
}

std::string cache_dir() {
  const char *e = knob(KNOB_JIT_CACHE);
  if (e && (!strcmp(e, "off") || !strcmp(e, "0"))) return "";
  std::string d;
  if (e && *e) d = e;
  else if (const char *x = knob(KNOB_XDG_CACHE_HOME)) d = std::string(x) + "/gdspfft";
  else if (const char *h = knob(KNOB_HOME)) d = std::string(h) + "/.cache/gdspfft";
  else d = "/tmp/gdspfft-" + std::to_string((long)getuid());
  return d;
}

// The cache directory (created 0700) is used only when it is a real
// directory owned by this user that nobody else can write: code objects
// loaded from it run on the GPU, so another local user must not be able to
// plant them (e.g. by pre-creating /tmp/gdspfft-<uid>).
bool make_dirs(const std::string &d) {
  for (size_t p = 1; p <= d.size(); ++p) {
    if (p == d.size() || d[p] == '/') {
      const std::string sub = d.substr(0, p);
      if (mkdir(sub.c_str(), p == d.size() ? 0700 : 0755) != 0 && errno != EEXIST) return false;
    }
  }
  return true;
}

bool cache_dir_trusted(const std::string &d) {
  struct stat st;
  if (lstat(d.c_str(), &st) != 0) return false;
  return S_ISDIR(st.st_mode) && st.st_uid == getuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

// cache file: "GDSPJIT1\n", the lowered (mangled) name of each kernel, then
// the code object; written to a temporary name and renamed into place
bool cache_load(const std::string &path, size_t nnames, std::vector<std::string> &lowered,
                std::vector<char> &code) {
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) return false;
  bool ok = false;
  char magic[9] = {};
  if (fread(magic, 1, 9, f) == 9 && !memcmp(magic, "GDSPJIT1\n", 9)) {
    lowered.clear();
    ok = true;
    for (size_t q = 0; ok && q < nnames; ++q) {
      uint32_t len = 0;
      ok = fread(&len, 4, 1, f) == 1 && len < 4096;
      std::string nm(len, '\0');
      ok = ok && fread(&nm[0], 1, len, f) == len;
      lowered.push_back(nm);
    }
    uint64_t cs = 0;
    ok = ok && fread(&cs, 8, 1, f) == 1 && cs > 0 && cs < ((uint64_t)1 << 30);
    if (ok) {
      code.resize(cs);
      ok = fread(code.data(), 1, cs, f) == cs;
    }
  }
  fclose(f);
  return ok;
}

void cache_store(const std::string &dir, const std::string &path,
                 const std::vector<std::string> &lowered, const std::vector<char> &code) {
  if (!make_dirs(dir)) return;
  const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
  FILE *f = fopen(tmp.c_str(), "wb");
  if (!f) return;
  bool ok = fwrite("GDSPJIT1\n", 1, 9, f) == 9;
  for (const auto &nm : lowered) {
    const uint32_t len = (uint32_t)nm.size();
    ok = ok && fwrite(&len, 4, 1, f) == 1 && fwrite(nm.data(), 1, len, f) == len;
  }
  const uint64_t cs = code.size();
  ok = ok && fwrite(&cs, 8, 1, f) == 1 && fwrite(code.data(), 1, cs, f) == cs;
  ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path.c_str()) != 0) unlink(tmp.c_str());
}

bool load_functions(const std::vector<char> &code, const std::vector<std::string> &lowered,
                    hipModule_t *mod, std::vector<hipFunction_t> &fs) {
  *mod = nullptr;
  if (hipModuleLoadData(mod, code.data()) != hipSuccess) {
    *mod = nullptr;
    return false;
  }
  fs.assign(lowered.size(), nullptr);
  for (size_t q = 0; q < lowered.size(); ++q) {
    if (hipModuleGetFunction(&fs[q], *mod, lowered[q].c_str()) != hipSuccess) {
      (void)hipModuleUnload(*mod);
      *mod = nullptr;
      return false;
    }
  }
  return true;
}

bool verbose() {
  static const bool v = knob(KNOB_JIT_VERBOSE) != nullptr;
  return v;
}

}  // namespace

bool jit_enabled() {
  static const bool on = [] {
    const char *e = knob(KNOB_JIT);
    return !(e && e[0] == '0');
  }();
  // GDSP_ALGO_GENERIC_MIXED (the runtime-radix kernel) turns it off too
  return on && !(algo_flags() & GDSP_ALGO_GENERIC_MIXED);
}

bool jit_radices(int n, int *rad, int *npass) {
  if (n < 2 || n > kMixedSpecMax || (n & (n - 1)) == 0) return false;
  Choice cur, best;
  Choice cheap[6];
  for (int k = 2; k <= 4; ++k) search(n, 0, k, cur, best, cheap[k]);
  // five passes only where no shorter list exists (2 * 7^4 = 4802, 2 * 3^4
  // * 7^2 = 7938, ...: chirp-z otherwise)
  if (best.np == 0) search(n, 0, 5, cur, best, cheap[5]);
  if (best.np == 0) return false;
  // the cheapest list of as many passes, where the model expects it at least
  // 15 % faster (its ranking is not reliable closer than that: round 5's
  // A/B of the compiled lists, profiles/r05/radix_lists_ab.txt)
  const Choice &ch = cheap[best.np];
  if (ch.np == best.np && ch.wide == best.wide && ch.cost < 0.85 * best.cost) best = ch;
  for (int q = 0; q < best.np; ++q) rad[q] = best.rad[q];
  *npass = best.np;
  return true;
}

// The convolution length of the smooth-L chirp-z (bluestein_fixed_kernel) for
// n, if one beats the current fused chirp-z's M by the lane-cost model:
// among L in [2n - 1, M), with a list of 2-4 passes of radices <= 16 (the
// cheap DFTs; 25 / 20 / odd primes above 13 cost 14-34 FP64 operations per
// point) within 1024 threads per transform, the L of the lowest L x
// lane_cost; taken only where that is below 0.85 of the current kernel's
// (M x lane_cost of its list: radix-16 passes for a power of 2, 16 x RB x 16
// or 16 x R1 x R2 x 16 for the chirpz6k.hip kernels).
int blufix_length(int64_t n, int64_t m_now, const int *rad_now, int np_now, int *rad, int *np) {
  if (n < 2 || 2 * n - 1 > 16384 || m_now <= 2 * n - 1) return 0;
  int t_now = 0, tpw_now = 0;
  fixed_geo(rad_now, np_now, &t_now, &tpw_now);
  double best = 0.85 * (double)m_now * lane_cost(rad_now, np_now, t_now);
  int bl = 0;
  static const int small[] = {16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2};
  for (int64_t L = 2 * n - 1; L < m_now && L <= 16384; ++L) {
    int64_t f = L;
    for (int q : {2, 3, 5, 7, 11, 13})
      while (f % q == 0) f /= q;
    if (f != 1 || (L & (L - 1)) == 0) continue;
    // every list of 2-4 radices <= 16 for L: the lowest L x lane_cost
    int cur[4];
    auto rec = [&](auto &&self, int64_t left, int depth) -> void {
      if (left == 1) {
        if (depth < 2) return;
        int t1 = 0, tpw = 0;
        fixed_geo(cur, depth, &t1, &tpw);
        if (t1 > 1024) return;
        const double c = (double)L * lane_cost(cur, depth, t1);
        if (c < best) {
          best = c;
          bl = (int)L;
          for (int q = 0; q < depth; ++q) rad[q] = cur[q];
          *np = depth;
        }
        return;
      }
      if (depth == 4) return;
      for (int r : small)
        if (left % r == 0) {
          cur[depth] = r;
          self(self, left / r, depth + 1);
        }
    };
    rec(rec, L, 0);
  }
  return bl;
}

struct JitBlu {  // bluestein_fixed_kernel for one n on one L
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr, real = nullptr;
  int n = 0, wg = 0, tpw = 0;
};

namespace {

// Compile `names` (kernel template instances of mixed_fixed.hpp) for device
// dev into one module; fs[q] = the kernel of names[q]. Loaded from the
// on-disk cache when an entry for the same headers, architecture, options
// and names exists. false on any failure (counted, gdsp_jit_stats).
bool compile_module(int dev, const std::vector<std::string> &names, const std::string &what,
                    hipModule_t *mod, std::vector<hipFunction_t> &fs) {
  hipDeviceProp_t prop;
  *mod = nullptr;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    record_failure(what, "hipGetDeviceProperties failed");
    return false;
  }
  const std::string arch = std::string("--offload-arch=") + prop.gcnArchName;
  const std::string incdir = include_dir();
  const std::string inc = "-I" + (incdir.empty() ? std::string(".") : incdir);
  const char *opts[] = {arch.c_str(), "-O3", "-std=c++17", inc.c_str()};
  // cache key: everything the code object depends on — the library and
  // runtime-compiler versions, the headers (embedded, or the files in
  // GDSP_JIT_INCLUDE by content), architecture, options and names
  int rtc_major = 0, rtc_minor = 0;
  (void)hiprtcVersion(&rtc_major, &rtc_minor);
  uint64_t key = fnv1a(gdsp_version(), gdsp_jit_embed::kHash);
  key = fnv1a("hiprtc " + std::to_string(rtc_major) + "." + std::to_string(rtc_minor), key);
  key = fnv1a(arch + "|" + incdir + "|-O3 -std=c++17", key);
  if (!incdir.empty()) {
    for (int h = 0; h < gdsp_jit_embed::kCount; ++h) {
      std::string text;
      if (FILE *f = fopen((incdir + "/" + gdsp_jit_embed::kNames[h]).c_str(), "rb")) {
        char buf[65536];
        size_t got;
        while ((got = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, got);
        fclose(f);
      }
      key = fnv1a(std::string(gdsp_jit_embed::kNames[h]) + "\n" + text, key);
    }
  }
  for (const auto &nm : names) key = fnv1a(nm + ";", key);
  std::string cdir = cache_dir();
  if (!cdir.empty() && !(make_dirs(cdir) && cache_dir_trusted(cdir))) {
    if (verbose()) fprintf(stderr, "gdsp: hipRTC cache %s not used (not a private directory)\n",
                           cdir.c_str());
    cdir.clear();
  }
  char hex[17];
  snprintf(hex, sizeof hex, "%016llx", (unsigned long long)key);
  const std::string cpath = cdir.empty() ? "" : cdir + "/" + hex + ".co";
  std::vector<std::string> lowered;
  std::vector<char> code;
  if (!cpath.empty() && cache_load(cpath, names.size(), lowered, code) &&
      load_functions(code, lowered, mod, fs)) {
    ++g_cached;
    if (verbose()) fprintf(stderr, "gdsp: hipRTC %s: loaded from %s\n", what.c_str(), cpath.c_str());
    return true;
  }
  const char *src = "#include \"mixed_fixed.hpp\"\n";
  hiprtcProgram prog;
  // embedded headers unless GDSP_JIT_INCLUDE points at a directory
  const int nh = incdir.empty() ? gdsp_jit_embed::kCount : 0;
  if (hiprtcCreateProgram(&prog, src, "gdsp_jit.hip", nh, nh ? gdsp_jit_embed::kTexts : nullptr,
                          nh ? gdsp_jit_embed::kNames : nullptr) != HIPRTC_SUCCESS) {
    record_failure(what, "hiprtcCreateProgram failed");
    return false;
  }
  for (const auto &nm : names) hiprtcAddNameExpression(prog, nm.c_str());
  bool ok = false;
  std::string why;
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc == HIPRTC_SUCCESS) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.assign(cs, 0);
    hiprtcGetCode(prog, code.data());
    lowered.clear();
    ok = cs > 0;
    for (size_t q = 0; ok && q < names.size(); ++q) {
      const char *low = nullptr;
      ok = hiprtcGetLoweredName(prog, names[q].c_str(), &low) == HIPRTC_SUCCESS && low;
      if (ok) lowered.push_back(low);
    }
    ok = ok && load_functions(code, lowered, mod, fs);
    if (!ok) why = "the compiled module did not load";
    if (ok && !cpath.empty()) cache_store(cdir, cpath, lowered, code);
  } else {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    why = std::string(hiprtcGetErrorString(rc)) + ": " + log.substr(0, 2000);
    if (verbose())
      fprintf(stderr, "gdsp: hipRTC %s failed (%s; %s %s):\n%s\n", what.c_str(),
              hiprtcGetErrorString(rc), arch.c_str(), inc.c_str(), log.c_str());
  }
  hiprtcDestroyProgram(&prog);
  if (ok) ++g_built;
  else record_failure(what, why);
  if (verbose()) fprintf(stderr, "gdsp: hipRTC %s: %s\n", what.c_str(), ok ? "built" : "not built");
  return ok;
}

std::string radix_list(const int *rad, int np) {
  std::string list;
  for (int q = 0; q < np; ++q) list += ", " + std::to_string(rad[q]);
  return list;
}

}  // namespace

JitSpec *jit_spec_build(int dev, const int *rad, int np, int n) {
  if (!jit_enabled()) return nullptr;
  const std::string list = radix_list(rad, np);
  const bool split = n > 4096, swz = rad[0] % 2 == 0;  // as spec_launch / launch_fixed
  const std::string sp = split ? "true" : "false", sw = swz ? "true" : "false";
  const std::vector<std::string> names = {
      "&gdsp::fft_mixed_fixed_kernel<false, 0, " + sp + ", " + sw + list + ">",
      "&gdsp::fft_mixed_fixed_kernel<true, 0, " + sp + ", " + sw + list + ">",
      "&gdsp::fft_mixed_fixed_kernel<false, 1, " + sp + ", " + sw + list + ">",
      "&gdsp::pwelch_fixed_kernel<" + sw + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "specialisation for n = " + std::to_string(n) + " (" +
                                      list.substr(2) + ")",
                      &mod, fs))
    return nullptr;
  JitSpec *j = new JitSpec;
  j->mod = mod;
  j->n = n;
  j->fwd = fs[0];
  j->inv = fs[1];
  j->real = fs[2];
  j->pw = fs[3];
  int t1 = 0;
  fixed_geo(rad, np, &t1, &j->tpw);
  j->wg = t1 * j->tpw;
  {
    // PwfDma (mixed_fixed.hpp) on the host: a radix-25 first pass, one
    // transform per workgroup, N <= 4096, exchange + stage + twiddle bases
    // within 80 KiB
    const int slots = (n + 7) & ~7, stg = (2 * slots + 127) / 128 * 128;
    int twn = 0, ns = 1;
    for (int q = 0; q + 1 < np; ++q) twn += (ns *= rad[q]);
    if (rad[0] == 25 && j->tpw == 1 && n <= 4096 && 8 * (slots + stg) + 16 * twn <= 81920)
      j->pw_stage = stg;
  }
  return j;
}

JitCol *jit_col_build(int dev, const int *rad, int np) {
  if (!jit_enabled() || np < 2) return nullptr;
  int L = 1;
  for (int q = 0; q < np; ++q) L *= rad[q];
  int t1 = 0, tpw = 0;
  fixed_geo(rad, np, &t1, &tpw);
  // columns per workgroup: the widest power of 2 <= 64 whose LDS (column
  // stride SL = slots + 1, odd) fits 80 KiB (two workgroups per CU), within
  // 1024 threads. The exchanges go as real / imaginary halves (SPLIT), which
  // doubles the width the LDS allows. Per 2^27 samples, 16 complex-exchange
  // columns -> this: 390625 3.15 -> 2.73 ms, 3^13 3.18 -> 2.98, 10^6 2.80
  // both
  const int sl = ((L + 7) & ~7) + 1;
  const int lds_max = 81920;
  const bool split = true;
  const int bytes = 8;
  int w = 64;
  while (w > 1 && (w * sl * bytes > lds_max || w * t1 > 1024)) w >>= 1;
  if (w * sl * bytes > 163840 || w * t1 > 1024) return nullptr;
  const std::string list = radix_list(rad, np), sw = rad[0] % 2 == 0 ? "true" : "false";
  const std::string ws = std::to_string(w) + (split ? ", true" : ", false");
  const std::vector<std::string> names = {
      "&gdsp::colfixed_kernel<" + ws + ", false, " + sw + list + ">",
      "&gdsp::colfixed_kernel<" + ws + ", true, " + sw + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "column pass for L = " + std::to_string(L) + " (" +
                                      list.substr(2) + "), " + ws + " columns",
                      &mod, fs))
    return nullptr;
  JitCol *j = new JitCol;
  j->mod = mod;
  j->fwd = fs[0];
  j->inv = fs[1];
  j->l = L;
  j->w = w;
  j->wg = w * t1;
  return j;
}

JitRowT *jit_rowt_build(int dev, const int *rad, int np) {
  if (!jit_enabled() || np < 1) return nullptr;
  int n = 1;
  for (int q = 0; q < np; ++q) n *= rad[q];
  int t1 = 0, tpw = 0;
  fixed_geo(rad, np, &t1, &tpw);
  // rows per workgroup: the widest of 16, 8, 4 within 1024 threads and 80 KiB
  // of LDS (two workgroups per CU): the exchange (W rows of n-double halves)
  // or the transposed staging (n x (W + 1) doubles), whichever is larger
  const int sl = (n + 7) & ~7;
  int w = 16;
  while (w >= 4 && (w * t1 > 1024 || 8 * std::max(w * sl, n * (w + 1)) > 81920)) w >>= 1;
  if (w < 4) return nullptr;
  const std::string list = radix_list(rad, np), sw = rad[0] % 2 == 0 ? "true" : "false";
  const std::string ws = std::to_string(w);
  const std::vector<std::string> names = {
      "&gdsp::rowt_fixed_kernel<" + ws + ", false, " + sw + list + ">",
      "&gdsp::rowt_fixed_kernel<" + ws + ", true, " + sw + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "transposed rows for C = " + std::to_string(n) + " (" +
                                      list.substr(2) + "), " + ws + " rows",
                      &mod, fs))
    return nullptr;
  JitRowT *j = new JitRowT;
  j->mod = mod;
  j->fwd = fs[0];
  j->cso = fs[1];
  j->n = n;
  j->w = w;
  j->wg = w * t1;
  return j;
}

JitRader *jit_rader_build(int dev, const int *rad, int np) {
  if (!jit_enabled() || np < 1) return nullptr;
  int n = 1;
  for (int q = 0; q < np; ++q) n *= rad[q];
  int t1 = 0, tpw = 0;
  fixed_geo(rad, np, &t1, &tpw);
  if (t1 > 1024) return nullptr;
  // RaderGeo (mixed_fixed.hpp) on the host: the staging holds the P = N + 1
  // samples, as complex slots or (N > 4096) real / imaginary halves
  const bool split = n > 4096;
  const int slots = (n + 1 + 7) & ~7, dpt = split ? slots : 2 * slots;
  tpw = 256 / t1 > 1 ? 256 / t1 : 1;
  while (tpw > 1 && tpw * dpt * 8 > 65536) --tpw;
  const std::string list = radix_list(rad, np), sw = rad[0] % 2 == 0 ? "true" : "false";
  const std::vector<std::string> names = {
      "&gdsp::rader_fixed_kernel<false, 0, " + sw + list + ">",
      "&gdsp::rader_fixed_kernel<true, 0, " + sw + list + ">",
      "&gdsp::rader_fixed_kernel<false, 1, " + sw + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "Rader kernel for P = " + std::to_string(n + 1) + " (N = " +
                                      list.substr(2) + ")",
                      &mod, fs))
    return nullptr;
  JitRader *j = new JitRader;
  j->mod = mod;
  j->fwd = fs[0];
  j->inv = fs[1];
  j->real = fs[2];
  j->p = n + 1;
  j->tpw = tpw;
  j->wg = t1 * tpw;
  return j;
}

namespace {
// dft_native / pfa_split (mixed_fixed.hpp) on the host
bool host_dft_native(int r) {
  static const int nat[] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 17, 19, 20, 23, 25, 29, 31, 32};
  return std::find(std::begin(nat), std::end(nat), r) != std::end(nat);
}
int host_gcd(int a, int b) { return b ? host_gcd(b, a % b) : a; }
}  // namespace

bool pfa_cofactor_supported(int m) {
  if (m < 2) return false;
  if (host_dft_native(m)) return true;
  for (int r1 = 2; r1 < m; ++r1)
    if (m % r1 == 0 && host_gcd(r1, m / r1) == 1 && host_dft_native(r1) && host_dft_native(m / r1))
      return true;
  return false;
}

JitRader *jit_rader_pfa_build(int dev, int m, const int *rad, int np) {
  if (!jit_enabled() || np < 1 || !pfa_cofactor_supported(m)) return nullptr;
  int n = 1;
  for (int q = 0; q < np; ++q) n *= rad[q];
  if (n > 4096) return nullptr;
  int t1 = 0, tpw = 0;
  fixed_geo(rad, np, &t1, &tpw);
  // PfaGeo (mixed_fixed.hpp) on the host: M sub-transforms of T1 threads per
  // row, rows per workgroup within 256 threads and 40 KiB of row slots
  const int p = n + 1, nn = m * p, subs = (n + 7) & ~7;
  const int rsl = std::max(m * subs, nn), rt = m * t1;
  tpw = 256 / rt > 1 ? 256 / rt : 1;
  while (tpw > 1 && tpw * (rsl + m) * 16 > 40960) --tpw;
  const int wg = tpw * rt;
  const int ncol = tpw * p, ca = (ncol + wg - 1) / wg;
  const long lds = 16L * tpw * (rsl + m);
  // one workgroup of at most 1024 threads within the CU's LDS, and the
  // stage-A columns' M-point values of a thread within 32 complex128 registers
  if (wg > 1024 || lds > 163840 || ca * m > 32) return nullptr;
  const std::string list = radix_list(rad, np), sw = rad[0] % 2 == 0 ? "true" : "false";
  const std::string ms = ", " + std::to_string(m);
  const std::vector<std::string> names = {
      "&gdsp::rader_pfa_kernel<false, 0, " + sw + ms + list + ">",
      "&gdsp::rader_pfa_kernel<true, 0, " + sw + ms + list + ">",
      "&gdsp::rader_pfa_kernel<false, 1, " + sw + ms + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "prime-factor Rader kernel for n = " + std::to_string(nn) +
                                      " = " + std::to_string(m) + " x " + std::to_string(p) +
                                      " (N = " + list.substr(2) + ")",
                      &mod, fs))
    return nullptr;
  JitRader *j = new JitRader;
  j->mod = mod;
  j->fwd = fs[0];
  j->inv = fs[1];
  j->real = fs[2];
  j->p = nn;
  j->tpw = tpw;
  j->wg = wg;
  return j;
}

JitBlu *jit_blu_build(int dev, int64_t n, const int *rad, int np) {
  if (!jit_enabled() || np < 1) return nullptr;
  int L = 1;
  for (int q = 0; q < np; ++q) L *= rad[q];
  int t1 = 0, tpw = 0;
  fixed_geo(rad, np, &t1, &tpw);
  const bool split = L > 4096;  // as FixedGeo's exchange in spec_launch
  if (t1 > 1024 || 2 * n - 1 > L) return nullptr;
  const std::string list = radix_list(rad, np), sw = rad[0] % 2 == 0 ? "true" : "false";
  const std::string sp = split ? "true" : "false", ns = ", " + std::to_string(n);
  const std::vector<std::string> names = {
      "&gdsp::bluestein_fixed_kernel<false, 0, " + sp + ", " + sw + ns + list + ">",
      "&gdsp::bluestein_fixed_kernel<true, 0, " + sp + ", " + sw + ns + list + ">",
      "&gdsp::bluestein_fixed_kernel<false, 1, " + sp + ", " + sw + ns + list + ">"};
  hipModule_t mod = nullptr;
  std::vector<hipFunction_t> fs;
  if (!compile_module(dev, names, "chirp-z kernel for n = " + std::to_string(n) + " on L = " +
                                      std::to_string(L) + " (" + list.substr(2) + ")",
                      &mod, fs))
    return nullptr;
  JitBlu *j = new JitBlu;
  j->mod = mod;
  j->fwd = fs[0];
  j->inv = fs[1];
  j->real = fs[2];
  j->n = (int)n;
  j->tpw = tpw;
  j->wg = t1 * tpw;
  return j;
}

hipError_t jit_launch_blu(const JitBlu *j, bool inv, int load, const void *in, cd *out,
                          int64_t batch, const cd *tw, const cd *chirp, const cd *bhat,
                          double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  const int64_t nblk = (batch + j->tpw - 1) / j->tpw;
  if (batch < 1 || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipFunction_t f = inv ? j->inv : (load == LOAD_REAL ? j->real : j->fwd);
  void *args[] = {(void *)&in,    (void *)&out,  (void *)&batch, (void *)&tw,
                  (void *)&chirp, (void *)&bhat, (void *)&scale};
  return hipModuleLaunchKernel(f, (unsigned)nblk, 1, 1, (unsigned)j->wg, 1, 1, 0, s, args,
                               nullptr);
}

hipError_t jit_launch_rader(const JitRader *j, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, const cd *bhat, const int *gpow,
                            const int *ginv, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  const int64_t nblk = (batch + j->tpw - 1) / j->tpw;
  if (batch < 1 || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipFunction_t f = inv ? j->inv : (load == LOAD_REAL ? j->real : j->fwd);
  void *args[] = {(void *)&in,   (void *)&out,  (void *)&batch, (void *)&tw,
                  (void *)&bhat, (void *)&gpow, (void *)&ginv,  (void *)&scale};
  return hipModuleLaunchKernel(f, (unsigned)nblk, 1, 1, (unsigned)j->wg, 1, 1, 0, s, args,
                               nullptr);
}

hipError_t jit_launch_rowt(const JitRowT *j, bool conj_scale_out, const cd *in, cd *out,
                           int64_t rows, int64_t L, const cd *tw, double scale, hipStream_t s) {
  if (rows < 1 || L < 1 || rows % L) return hipErrorInvalidValue;
  const int64_t gx = (rows + j->w - 1) / j->w;
  if (gx > 0x7fffffff) return hipErrorInvalidValue;
  void *args[] = {(void *)&in, (void *)&out, (void *)&L, (void *)&rows, (void *)&tw,
                  (void *)&scale};
  return hipModuleLaunchKernel(conj_scale_out ? j->cso : j->fwd, (unsigned)gx, 1, 1,
                               (unsigned)j->wg, 1, 1, 0, s, args, nullptr);
}

hipError_t jit_launch_col(const JitCol *j, bool conj_in, const cd *in, cd *out, int64_t C,
                          int64_t n, int64_t batch, const cd *tw, const cd *twn, hipStream_t s) {
  if (batch < 1 || batch > 65535 || C < 1 || C * j->l != n) return hipErrorInvalidValue;
  const int64_t gx = (C + j->w - 1) / j->w;
  if (gx > 0x7fffffff) return hipErrorInvalidValue;
  void *args[] = {(void *)&in, (void *)&out, (void *)&C, (void *)&n, (void *)&tw, (void *)&twn};
  return hipModuleLaunchKernel(conj_in ? j->inv : j->fwd, (unsigned)gx, (unsigned)batch, 1,
                               (unsigned)j->wg, 1, 1, 0, s, args, nullptr);
}

hipError_t jit_launch_fft(const JitSpec *j, bool inv, int load, const void *in, cd *out,
                          int64_t batch, const cd *tw, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  const int64_t nblk = (batch + j->tpw - 1) / j->tpw;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipFunction_t f = inv ? j->inv : (load == LOAD_REAL ? j->real : j->fwd);
  void *args[] = {(void *)&in, (void *)&out, (void *)&batch, (void *)&tw, (void *)&scale};
  return hipModuleLaunchKernel(f, (unsigned)nblk, 1, 1, (unsigned)j->wg, 1, 1, 0, s, args,
                               nullptr);
}

int jit_pw_tpw(const JitSpec *j, int64_t span) {
  if (!j || (j->pw_stage && span > j->pw_stage)) return 0;
  return j->tpw;
}

hipError_t jit_launch_pwelch(const JitSpec *j, const double *x, int64_t nfft, int64_t stride,
                             int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                             const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (nworkers <= 0 || nworkers > 0x7fffffff || !jit_pw_tpw(j, stride + nfft))
    return hipErrorInvalidValue;
  const int64_t nblk = (nworkers + j->tpw - 1) / j->tpw;
  void *args[] = {(void *)&x,   (void *)&nfft,    (void *)&stride,
                  (void *)&seg_begin, (void *)&seg_end, (void *)&ppw,
                  (void *)&win, (void *)&tw,      (void *)&partial};
  return hipModuleLaunchKernel(j->pw, (unsigned)nblk, 1, 1, (unsigned)j->wg, 1, 1, 0, s, args,
                               nullptr);
}

}  // namespace gdsp

extern "C" int gdsp_jit_stats(int64_t *built, int64_t *cached, int64_t *failed, char *last_failure,
                              int64_t cap) {
  if (built) *built = gdsp::g_built.load();
  if (cached) *cached = gdsp::g_cached.load();
  if (failed) *failed = gdsp::g_failed.load();
  if (last_failure && cap > 0) {
    std::lock_guard<std::mutex> lk(gdsp::g_fail_mu);
    const size_t n = std::min<size_t>((size_t)cap - 1, gdsp::g_last_failure.size());
    memcpy(last_failure, gdsp::g_last_failure.data(), n);
    last_failure[n] = '\0';
  }
  return GDSP_OK;
}
