// fft_mixed.hip — one-kernel mixed-radix Stockham FFT for non-power-of-2
// lengths whose prime factors are all in {2, 3, 5, 7, 11, 13}: the
// runtime-radix kernels (n <= 4096) and the dispatch to the compiled
// specialisations (fft_specs*.hip, n <= 8192).
//
// The reference computes every non-power-of-2 length with Bluestein's chirp-z
// (fft/fft.go:86 -> fft/bluestein.go:68-94): three radix-2 FFTs of
// M = NextPowerOf2(2n-1) per transform (M = 8192 for n = 3000). The DFT it
// approximates is the same one this kernel computes directly, with about a
// sixth of the arithmetic and one HBM read + one HBM write per element, so
// smooth lengths are HBM-bound here instead of FP64-bound. Lengths with a
// larger prime factor keep the fused chirp-z kernel (fft_kernels.hip), and
// gdsp_plan_create_chirpz forces it for any length.
//
// Pass p (radix R, Ns = product of the earlier radices) maps butterfly j to
// inputs j + r*n/R and outputs (j/Ns)*Ns*R + j%Ns + r*Ns with twiddle
// W_{Ns*R}^{(j%Ns)*r}: the same Stockham autosort as the power-of-2 kernels,
// with the radix chosen per pass. Pass 0 reads HBM, the last pass writes HBM,
// the passes between exchange through LDS (complex128, ds_*_b128). Per-pass
// twiddles come from a table laid out butterfly-major (long-double accurate,
// built with the plan), so a butterfly's R-1 factors are one contiguous run.
#include "gdsp_fft.h"
#include "mixed_core.hpp"
#include "mixed_specs.hpp"

#include <stdlib.h>

namespace gdsp {

// One Stockham pass of radix R over a transform of n points. MODE: 0 first
// (HBM -> LDS), 1 middle (LDS -> LDS), 2 last (LDS -> HBM), 3 single pass
// (HBM -> HBM). J = 16 / R butterflies per thread at most, so a pass never
// holds more than 16 complex128 per thread. Not inlined: each radix gets its
// own register allocation instead of the union over the kernel's switch.
enum { MP_FIRST = 0, MP_MID = 1, MP_LAST = 2, MP_SINGLE = 3 };

template <int R, bool INV, int LOAD, int MODE>
__device__ __attribute__((noinline)) void mixed_pass(int n, int ns, int t1, int tl, bool valid,
                                                     const void *__restrict__ gin,
                                                     cd *__restrict__ gout, cd *lds,
                                                     const cd *__restrict__ tw, double scale) {
  constexpr bool FROM_HBM = MODE == MP_FIRST || MODE == MP_SINGLE;
  constexpr bool TO_HBM = MODE == MP_LAST || MODE == MP_SINGLE;
  constexpr int J = R > 16 ? 1 : 16 / R;
  const int nb = n / R;
  cd v[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (valid && j < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        cd x;
        if constexpr (!FROM_HBM) {
          x = lds[lsw(j + r * nb)];
        } else if constexpr (LOAD == LOAD_REAL) {
          x = {reinterpret_cast<const double *>(gin)[j + r * nb], 0.0};
        } else {
          x = reinterpret_cast<const cd *>(gin)[j + r * nb];
          if constexpr (INV) x.y = -x.y;
        }
        v[jj][r] = x;
      }
    }
  }
  // a middle pass overwrites the buffer it read: every read lands first
  if constexpr (MODE == MP_MID) __syncthreads();
  // k = j % ns for j = tl + jj*t1, stepped instead of divided per butterfly
  // (one division per pass; dk is uniform)
  int k = FROM_HBM ? 0 : tl % ns;
  const int dk = FROM_HBM ? 0 : t1 % ns;
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (jj > 0 && !FROM_HBM) {
      k += dk;
      if (k >= ns) k -= ns;
    }
    if (valid && j < nb) {
      if constexpr (!FROM_HBM) twiddle_chain<R>(v[jj], tw[k]);
      dft_any<R>(v[jj]);
      const int o = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (TO_HBM) {
          cd y = v[jj][r];
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          gout[o + r * ns] = y;
        } else {
          lds[lsw(o + r * ns)] = v[jj][r];
        }
      }
    }
  }
}

// the radices of the generic lists (the runtime-radix kernels; compiled
// specialisations with composite radices have their own kernels)
#define GDSP_FOR_RADICES(X) X(2) X(3) X(4) X(5) X(7) X(8) X(11) X(13) X(16)

template <bool INV, int LOAD, int MODE>
__device__ __forceinline__ void mixed_dispatch(int R, int n, int ns, int t1, int tl, bool valid,
                                               const void *gin, cd *gout, cd *lds, const cd *tw,
                                               double scale) {
  switch (R) {
#define GDSP_MIXED_CASE(RR)                                                                 \
  case RR:                                                                                  \
    mixed_pass<RR, INV, LOAD, MODE>(n, ns, t1, tl, valid, gin, gout, lds, tw, scale);       \
    break;
    GDSP_FOR_RADICES(GDSP_MIXED_CASE)
#undef GDSP_MIXED_CASE
    default:
      break;
  }
}

// codes: radix of pass p in bits [5p, 5p+5). Workgroup = tpw transforms of
// t1 threads; LDS = tpw * n complex128 (dynamic).
template <bool INV, int LOAD>
__global__ __launch_bounds__(512) void fft_mixed_kernel(const void *__restrict__ in,
                                                        cd *__restrict__ out, int64_t batch,
                                                        MixedDesc d, const cd *__restrict__ tw,
                                                        double scale) {
  extern __shared__ cd lds_mixed[];
  const int sub = threadIdx.x / d.t1;
  const int tl = threadIdx.x - sub * d.t1;
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x) * d.tpw + sub;
  const bool valid = sub < d.tpw && row < batch;
  const int n = d.n;
  const void *gin = LOAD == LOAD_REAL
                        ? (const void *)(reinterpret_cast<const double *>(in) + row * n)
                        : (const void *)(reinterpret_cast<const cd *>(in) + row * n);
  cd *gout = out + row * n;
  cd *lds = lds_mixed + (sub < d.tpw ? sub : 0) * ((n + 7) & ~7);
  const int np = d.npass;
  int R = (int)(d.codes & 31);
  if (np == 1) {
    mixed_dispatch<INV, LOAD, MP_SINGLE>(R, n, 1, d.t1, tl, valid, gin, gout, lds, tw, scale);
    return;
  }
  mixed_dispatch<INV, LOAD, MP_FIRST>(R, n, 1, d.t1, tl, valid, gin, gout, lds, tw, scale);
  int ns = R, twoff = 0;
  for (int p = 1; p < np; ++p) {
    R = (int)((d.codes >> (5 * p)) & 31);
    __syncthreads();  // the previous pass's LDS writes are visible
    if (p < np - 1)
      mixed_dispatch<INV, LOAD, MP_MID>(R, n, ns, d.t1, tl, valid, gin, gout, lds, tw + twoff,
                                        scale);
    else
      mixed_dispatch<INV, LOAD, MP_LAST>(R, n, ns, d.t1, tl, valid, gin, gout, lds, tw + twoff,
                                         scale);
    twoff += ns;
    ns *= R;
  }
}

// ---------------------------------------------------------------------------
// Fused Pwelch over a mixed-radix segment length (spectral/pwelch.go:104-122
// for NFFT / Pad that are not powers of 2): the same packed segment pairs
// z = w*x_s + i*w*x_{s+1} and per-bin |Z_k|^2 sums as the power-of-2 kernels
// (finalize folds k and F-k), on the runtime-radix passes above. One
// transform per workgroup, persistent over a contiguous range of pairs; the
// per-bin sums live in LDS, each bin written by the one thread whose last
// pass produces it, so they need no synchronisation.
template <int R>
__device__ __attribute__((noinline)) void pw_first_pass(int flen, int nfft, int t1, int tl,
                                                        bool active, bool has1,
                                                        const double *__restrict__ x0,
                                                        const double *__restrict__ x1,
                                                        const double *__restrict__ win,
                                                        cd *lds) {
  constexpr int J = R > 16 ? 1 : 16 / R;
  const int nb = flen / R;
  cd v[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int i = j + r * nb;
        double a = 0.0, b = 0.0;
        if (active && i < nfft) {
          const double w = win[i];
          a = w * x0[i];
          if (has1) b = w * x1[i];
        }
        v[jj][r] = {a, b};
      }
      dft_any<R>(v[jj]);
#pragma unroll
      for (int r = 0; r < R; ++r) lds[lsw(j * R + r)] = v[jj][r];
    }
  }
}

template <int R>
__device__ __attribute__((noinline)) void pw_last_pass(int flen, int t1, int tl, bool active,
                                                       cd *lds, const cd *__restrict__ tw,
                                                       double *lacc) {
  constexpr int J = R > 16 ? 1 : 16 / R;
  const int nb = flen / R;  // = Ns of the last pass: butterfly j writes bins j + r*nb
  cd v[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (j < nb) {
#pragma unroll
      for (int r = 0; r < R; ++r) v[jj][r] = lds[lsw(j + r * nb)];
    }
  }
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (j < nb) {
      twiddle_chain<R>(v[jj], tw[j]);
      dft_any<R>(v[jj]);
      if (active) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          lacc[j + r * nb] += v[jj][r].x * v[jj][r].x + v[jj][r].y * v[jj][r].y;
      }
    }
  }
}

__global__ __launch_bounds__(512) void pwelch_mixed_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t pairs_per_worker, MixedDesc d, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  extern __shared__ double pw_lds[];
  const int flen = d.n, slots = (flen + 7) & ~7;
  cd *lds = reinterpret_cast<cd *>(pw_lds);
  double *lacc = pw_lds + 2 * slots;
  const int tl = threadIdx.x, t1 = d.t1;
  for (int i = tl; i < flen; i += t1) lacc[i] = 0.0;
  const int64_t worker = blockIdx.x;
  const int64_t p0 = worker * pairs_per_worker;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int np = d.npass;
  for (int64_t it = 0; it < pairs_per_worker; ++it) {
    const int64_t p = p0 + it;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * (active ? p : 0);
    const bool has1 = active && s0 + 1 < seg_end;
    const double *x0 = x + s0 * stride, *x1 = x0 + stride;
    __syncthreads();  // the previous pair's last-pass reads are done
    int R = (int)(d.codes & 31);
    switch (R) {
#define GDSP_PW_FIRST(RR)                                                                 \
  case RR:                                                                                \
    pw_first_pass<RR>(flen, (int)nfft, t1, tl, active, has1, x0, x1, win, lds);           \
    break;
      GDSP_FOR_RADICES(GDSP_PW_FIRST)
#undef GDSP_PW_FIRST
      default:
        break;
    }
    int ns = R, twoff = 0;
    for (int q = 1; q < np; ++q) {
      R = (int)((d.codes >> (5 * q)) & 31);
      __syncthreads();
      if (q < np - 1) {
        mixed_dispatch<false, LOAD_COMPLEX, MP_MID>(R, flen, ns, t1, tl, true, nullptr, nullptr,
                                                    lds, tw + twoff, 1.0);
      } else {
        switch (R) {
#define GDSP_PW_LAST(RR)                                                                   \
  case RR:                                                                                 \
    pw_last_pass<RR>(flen, t1, tl, active, lds, tw + twoff, lacc);                         \
    break;
          GDSP_FOR_RADICES(GDSP_PW_LAST)
#undef GDSP_PW_LAST
          default:
            break;
        }
      }
      twoff += ns;
      ns *= R;
    }
  }
  __syncthreads();
  if (p0 < npairs)
    for (int i = tl; i < flen; i += t1) partial[worker * flen + i] = lacc[i];
}

hipError_t launch_pwelch_mixed(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,
                               int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                               const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (d.npass < 2 || d.t1 <= 0 || d.t1 > 512 || nworkers > 0x7fffffff)
    return hipErrorInvalidValue;
  const size_t lds = (2 * (size_t)((d.n + 7) & ~7) + (size_t)d.n) * sizeof(double);
  static bool attr = false;
  if (!attr) {  // up to 4096 points: 96 KiB of dynamic LDS
    hipError_t e = hipFuncSetAttribute((const void *)pwelch_mixed_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(pwelch_mixed_kernel, dim3((unsigned)nworkers), dim3(d.t1), lds, s, x, nfft,
                     stride, seg_begin, seg_end, ppw, d, win, tw, partial);
  return hipGetLastError();
}

// Column pass of the mixed four-step for n = L * C with a single-radix L
// (every length dft_any has, <= 25): x as L rows x C columns, one thread per
// column holds the whole column in registers (no LDS), so each wave-
// instruction is a contiguous 1 KiB row segment. Column c: DFT_L over its L
// rows, times W_n^(c*k) (from W_n^c by recurrence), written in place of
// the rows. The rows DFT_C and the transpose follow (exec_mixed4).
template <int L, bool CONJ_IN>
__global__ __launch_bounds__(256) void colradix_kernel(const cd *__restrict__ in,
                                                       cd *__restrict__ out, int64_t C, int64_t n,
                                                       int64_t batch, const cd *__restrict__ tw) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = blockIdx.y;
  if (c >= C || b >= batch) return;
  const cd *src = in + b * n + c;
  cd v[L];
#pragma unroll
  for (int r = 0; r < L; ++r) {
    v[r] = ld_nt(src + r * C);
    if constexpr (CONJ_IN) v[r].y = -v[r].y;
  }
  dft_any<L>(v);
  cd *dst = out + b * n + c;
  st_nt(dst, v[0]);
  // W_n^(c*k) = (W_n^c)^k: one table read and a recurrence (L - 1 reads per
  // column would scatter over an n-entry table that misses L2 at large n)
  const cd w1 = tw[c];
  cd w = w1;
#pragma unroll
  for (int k = 1; k < L; ++k) {
    st_nt(dst + k * C, cmul(v[k], w));
    if (k + 1 < L) w = cmul(w, w1);
  }
}

bool colradix_supported(int L) {
  switch (L) {
    case 2: case 3: case 4: case 5: case 6: case 7: case 8: case 9: case 10: case 11: case 12:
    case 13: case 15: case 16: case 20: case 25:
      return true;
    default:
      return false;
  }
}

hipError_t launch_colradix(int L, bool conj_in, const cd *in, cd *out, int64_t C, int64_t n,
                           int64_t batch, const cd *tw, hipStream_t s) {
  if (batch < 1 || batch > 65535 || C < 1) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((C + 255) / 256), (unsigned)batch);
  switch (L) {
#define GDSP_CR(LL)                                                                          \
  case LL:                                                                                   \
    if (conj_in)                                                                             \
      hipLaunchKernelGGL((colradix_kernel<LL, true>), grid, dim3(256), 0, s, in, out, C, n,  \
                         batch, tw);                                                         \
    else                                                                                     \
      hipLaunchKernelGGL((colradix_kernel<LL, false>), grid, dim3(256), 0, s, in, out, C, n, \
                         batch, tw);                                                         \
    return hipGetLastError();
    GDSP_CR(2) GDSP_CR(3) GDSP_CR(4) GDSP_CR(5) GDSP_CR(6) GDSP_CR(7) GDSP_CR(8) GDSP_CR(9)
    GDSP_CR(10) GDSP_CR(11) GDSP_CR(12) GDSP_CR(13) GDSP_CR(15) GDSP_CR(16) GDSP_CR(20)
    GDSP_CR(25)
#undef GDSP_CR
    default: return hipErrorInvalidValue;
  }
}

// Radix list of the compiled specialisation for n, if there is one
// (launch_fft_mixed picks the kernel by n and list). GDSP_ALGO_GENERIC_MIXED
// disables them. n = 3000: 1.10 ms per 65536 transforms for 25*15*8 against
// 1.14-1.18 ms for the other orders of these radices and 1.82 ms for the
// generic 8*5*5*5*3 kernel; a split (re/im) exchange measured 3-4 % slower.
bool mixed_fixed_radices(int n, int *rad, int *npass) {
  if (algo_flags() & GDSP_ALGO_GENERIC_MIXED) return false;
  return specs0_find(n, rad, npass) || specs1_find(n, rad, npass) ||
         specs2_find(n, rad, npass) || specs3_find(n, rad, npass);
}

// A list for n's fused Pwelch other than its FFT list (the specspw group,
// fft_specs0.hip), if there is one.
bool pwelch_fixed_radices(int n, int *rad, int *npass) {
  if (algo_flags() & GDSP_ALGO_GENERIC_MIXED) return false;
  return specspw_find(n, rad, npass);
}

int pwelch_fixed_workers_per_block(const MixedDesc &d, int64_t span) {
  int t = specspw_pw_tpw(d, span);
  if (!t) t = specs0_pw_tpw(d, span);
  if (!t) t = specs1_pw_tpw(d, span);
  if (!t) t = specs2_pw_tpw(d, span);
  if (!t) t = specs3_pw_tpw(d, span);
  return t;
}

hipError_t launch_pwelch_fixed(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,
                               int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                               const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (nworkers <= 0 || nworkers > 0x7fffffff) return hipErrorInvalidValue;
#define GDSP_PWG(G) \
  G##_pw_launch(d, x, nfft, stride, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s)
  if (!(GDSP_PWG(specspw) || GDSP_PWG(specs0) || GDSP_PWG(specs1) || GDSP_PWG(specs2) ||
        GDSP_PWG(specs3)))
    return hipErrorInvalidValue;
#undef GDSP_PWG
  return hipGetLastError();
}

hipError_t launch_fft_mixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  if (d.t1 <= 0 || d.tpw <= 0 || d.t1 * d.tpw > 512) return hipErrorInvalidValue;
  const int64_t nblk = (batch + d.tpw - 1) / d.tpw;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  if (batch > (int64_t)0x7fffffff) return hipErrorInvalidValue;
#define GDSP_FXG(G) G##_launch(d, inv, load, in, out, batch, tw, scale, s)
  if (GDSP_FXG(specs0) || GDSP_FXG(specs1) || GDSP_FXG(specs2) || GDSP_FXG(specs3))
    return hipGetLastError();
#undef GDSP_FXG
  // the runtime-radix kernel keeps a transform's complex128 slots in dynamic
  // LDS (<= 64 KiB): lengths above kMixedMax exist only as specialisations
  if (d.n > kMixedMax) return hipErrorInvalidValue;
  const size_t lds = (size_t)d.tpw * (size_t)((d.n + 7) & ~7) * sizeof(cd);
  const dim3 grid((unsigned)nblk), block((unsigned)(d.t1 * d.tpw));
  if (inv) {
    hipLaunchKernelGGL((fft_mixed_kernel<true, LOAD_COMPLEX>), grid, block, lds, s, in, out,
                       batch, d, tw, scale);
  } else if (load == LOAD_REAL) {
    hipLaunchKernelGGL((fft_mixed_kernel<false, LOAD_REAL>), grid, block, lds, s, in, out, batch,
                       d, tw, scale);
  } else {
    hipLaunchKernelGGL((fft_mixed_kernel<false, LOAD_COMPLEX>), grid, block, lds, s, in, out,
                       batch, d, tw, scale);
  }
  return hipGetLastError();
}

}  // namespace gdsp
