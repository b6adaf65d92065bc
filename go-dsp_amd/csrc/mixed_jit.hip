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

namespace {

// the radices dft_any has (mixed_core.hpp)
constexpr int kRadices[] = {25, 20, 16, 15, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2};

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
  int rad[4], np = 0;
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
  if (best.np == 0) return false;
  for (int q = 0; q < best.np; ++q) rad[q] = best.rad[q];
  *npass = best.np;
  return true;
}

JitSpec *jit_spec_build(int dev, const int *rad, int np, int n) {
  if (!jit_enabled()) return nullptr;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
  std::string list;
  for (int q = 0; q < np; ++q) list += ", " + std::to_string(rad[q]);
  const bool split = n > 4096, swz = rad[0] % 2 == 0;  // as spec_launch / launch_fixed
  const std::string sp = split ? "true" : "false", sw = swz ? "true" : "false";
  const std::string names[4] = {
      "&gdsp::fft_mixed_fixed_kernel<false, 0, " + sp + ", " + sw + list + ">",
      "&gdsp::fft_mixed_fixed_kernel<true, 0, " + sp + ", " + sw + list + ">",
      "&gdsp::fft_mixed_fixed_kernel<false, 1, " + sp + ", " + sw + list + ">",
      "&gdsp::pwelch_fixed_kernel<" + sw + list + ">"};
  const char *src = "#include \"mixed_fixed.hpp\"\n";
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src, "gdsp_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return nullptr;
  for (const auto &nm : names) hiprtcAddNameExpression(prog, nm.c_str());
  const std::string arch = std::string("--offload-arch=") + prop.gcnArchName;
  const std::string inc = "-I" + include_dir();
  const char *opts[] = {arch.c_str(), "-O3", "-std=c++17", inc.c_str()};
  JitSpec *j = nullptr;
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc == HIPRTC_SUCCESS) {
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    j = new JitSpec;
    j->n = n;
    int t1 = 0;
    fixed_geo(rad, np, &t1, &j->tpw);
    j->wg = t1 * j->tpw;
    hipFunction_t *fs[4] = {&j->fwd, &j->inv, &j->real, &j->pw};
    bool ok = hipModuleLoadData(&j->mod, code.data()) == hipSuccess;
    for (int q = 0; ok && q < 4; ++q) {
      const char *low = nullptr;
      ok = hiprtcGetLoweredName(prog, names[q].c_str(), &low) == HIPRTC_SUCCESS && low &&
           hipModuleGetFunction(fs[q], j->mod, low) == hipSuccess;
    }
    if (!ok) {
      if (j->mod) (void)hipModuleUnload(j->mod);
      delete j;
      j = nullptr;
    }
  } else if (verbose()) {
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    std::string log(ls, '\0');
    if (ls) hiprtcGetProgramLog(prog, &log[0]);
    fprintf(stderr, "gdsp: hipRTC specialisation for n = %d failed (%s; %s %s):\n%s\n", n,
            hiprtcGetErrorString(rc), arch.c_str(), inc.c_str(), log.c_str());
  }
  hiprtcDestroyProgram(&prog);
  if (verbose())
    fprintf(stderr, "gdsp: hipRTC specialisation for n = %d (%s): %s\n", n, list.c_str() + 2,
            j ? "built" : "not built");
  return j;
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
