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
// fused Pwelch kernel, ~0.5-1 s once per length and process. Any failure
// (no hipRTC, no headers, a compile error) leaves the plan on the runtime-
// radix kernel or Bluestein, so this is a speed path only. GDSP_JIT=0
// disables it; GDSP_JIT_INCLUDE names the header directory (default: the
// csrc directory beside the library's lib/ directory).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "launch.hpp"

namespace gdsp {

struct JitSpec {
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr, real = nullptr, pw = nullptr;
  int n = 0, wg = 0, tpw = 0;
};

struct JitCol {  // colfixed_kernel for one column length
  hipModule_t mod = nullptr;
  hipFunction_t fwd = nullptr, inv = nullptr;
  int l = 0, w = 0, wg = 0;
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
};

bool better(const Choice &a, const Choice &b) {  // a before b?
  if (a.wide != b.wide) return !a.wide;
  if (a.np != b.np) return a.np < b.np;
  if (a.eff != b.eff) return a.eff > b.eff;
  if (a.pow2last != b.pow2last) return a.pow2last;
  return a.rad[0] > b.rad[0];
}

void search(int n, int depth, int maxdepth, Choice &cur, Choice &best) {
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
    if (best.np == 0 || better(c, best)) best = c;
    return;
  }
  for (int r : kRadices) {
    if (n % r) continue;
    cur.rad[depth] = r;
    search(n / r, depth + 1, maxdepth, cur, best);
  }
}

std::string include_dir() {
  if (const char *e = getenv("GDSP_JIT_INCLUDE")) return e;
  Dl_info info;
  if (dladdr((void *)&jit_radices, &info) && info.dli_fname) {
    std::string p = info.dli_fname;  // .../go-dsp_amd/lib/libgdspfft.so
    const size_t s = p.rfind('/');
    if (s != std::string::npos) return p.substr(0, s) + "/../csrc";
  }
  return "";
}

bool verbose() {
  static const bool v = getenv("GDSP_JIT_VERBOSE") != nullptr;
  return v;
}

}  // namespace

bool jit_enabled() {
  static const bool on = [] {
    const char *e = getenv("GDSP_JIT");
    // GDSP_MIXED_GENERIC=1 (tests of the runtime-radix kernel) turns it off too
    return !(e && e[0] == '0') && !getenv("GDSP_MIXED_GENERIC");
  }();
  return on;
}

bool jit_radices(int n, int *rad, int *npass) {
  if (n < 2 || n > kMixedSpecMax || (n & (n - 1)) == 0) return false;
  Choice cur, best;
  for (int k = 2; k <= 4; ++k) search(n, 0, k, cur, best);
  // five passes only where no shorter list exists (2 * 7^4 = 4802, 2 * 3^4
  // * 7^2 = 7938, ...: chirp-z otherwise)
  if (best.np == 0) search(n, 0, 5, cur, best);
  if (best.np == 0) return false;
  for (int q = 0; q < best.np; ++q) rad[q] = best.rad[q];
  *npass = best.np;
  return true;
}

namespace {

// Compile `names` (kernel template instances of mixed_fixed.hpp) for device
// dev into one module; fs[q] = the kernel of names[q]. false on any failure.
bool compile_module(int dev, const std::vector<std::string> &names, const std::string &what,
                    hipModule_t *mod, std::vector<hipFunction_t> &fs) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
  const char *src = "#include \"mixed_fixed.hpp\"\n";
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src, "gdsp_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return false;
  for (const auto &nm : names) hiprtcAddNameExpression(prog, nm.c_str());
  const std::string arch = std::string("--offload-arch=") + prop.gcnArchName;
  const std::string inc = "-I" + include_dir();
  const char *opts[] = {arch.c_str(), "-O3", "-std=c++17", inc.c_str()};
  bool ok = false;
  *mod = nullptr;
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc == HIPRTC_SUCCESS) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    fs.assign(names.size(), nullptr);
    ok = hipModuleLoadData(mod, code.data()) == hipSuccess;
    for (size_t q = 0; ok && q < names.size(); ++q) {
      const char *low = nullptr;
      ok = hiprtcGetLoweredName(prog, names[q].c_str(), &low) == HIPRTC_SUCCESS && low &&
           hipModuleGetFunction(&fs[q], *mod, low) == hipSuccess;
    }
    if (!ok && *mod) {
      (void)hipModuleUnload(*mod);
      *mod = nullptr;
    }
  } else if (verbose()) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    fprintf(stderr, "gdsp: hipRTC %s failed (%s; %s %s):\n%s\n", what.c_str(),
            hiprtcGetErrorString(rc), arch.c_str(), inc.c_str(), log.c_str());
  }
  hiprtcDestroyProgram(&prog);
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
  // both (GDSP_COL_LDS / GDSP_COL_SPLIT=0 to compare)
  const int sl = ((L + 7) & ~7) + 1;
  int lds_max = 81920;
  if (const char *e = getenv("GDSP_COL_LDS")) lds_max = atoi(e);
  const char *se = getenv("GDSP_COL_SPLIT");
  const bool split = !(se && se[0] == '0');
  const int bytes = split ? 8 : 16;
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

int jit_pw_tpw(const JitSpec *j) { return j ? j->tpw : 0; }

hipError_t jit_launch_pwelch(const JitSpec *j, const double *x, int64_t nfft, int64_t stride,
                             int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                             const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (nworkers <= 0 || nworkers > 0x7fffffff) return hipErrorInvalidValue;
  const int64_t nblk = (nworkers + j->tpw - 1) / j->tpw;
  void *args[] = {(void *)&x,   (void *)&nfft,    (void *)&stride,
                  (void *)&seg_begin, (void *)&seg_end, (void *)&ppw,
                  (void *)&win, (void *)&tw,      (void *)&partial};
  return hipModuleLaunchKernel(j->pw, (unsigned)nblk, 1, 1, (unsigned)j->wg, 1, 1, 0, s, args,
                               nullptr);
}

}  // namespace gdsp
