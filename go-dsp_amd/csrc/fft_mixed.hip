// fft_mixed.hip — one-kernel mixed-radix Stockham FFT for non-power-of-2
// lengths whose prime factors are all in {2, 3, 5, 7, 11, 13} (n <= 4096).
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
#include "fft_device.hpp"
#include "launch.hpp"

#include <stdlib.h>

namespace gdsp {

template <int R>
struct OddTab;  // cos / sin(2 pi q / R), q < R
template <>
struct OddTab<3> {
  static constexpr double c[3] = {1, -0.5, -0.5};
  static constexpr double s[3] = {0, 0.8660254037844386, -0.8660254037844386};
};
template <>
struct OddTab<5> {
  static constexpr double c[5] = {1, 0.30901699437494745, -0.80901699437494745,
                                  -0.80901699437494745, 0.30901699437494745};
  static constexpr double s[5] = {0, 0.95105651629515353, 0.58778525229247314,
                                  -0.58778525229247314, -0.95105651629515353};
};
template <>
struct OddTab<7> {
  static constexpr double c[7] = {1,
                                  0.62348980185873348,
                                  -0.22252093395631439,
                                  -0.90096886790241915,
                                  -0.90096886790241915,
                                  -0.22252093395631439,
                                  0.62348980185873348};
  static constexpr double s[7] = {0,
                                  0.7818314824680298,
                                  0.97492791218182362,
                                  0.43388373911755812,
                                  -0.43388373911755812,
                                  -0.97492791218182362,
                                  -0.7818314824680298};
};
template <>
struct OddTab<11> {
  static constexpr double c[11] = {1,
                                   0.84125353283118121,
                                   0.41541501300188644,
                                   -0.14231483827328514,
                                   -0.6548607339452851,
                                   -0.95949297361449737,
                                   -0.95949297361449737,
                                   -0.6548607339452851,
                                   -0.14231483827328514,
                                   0.41541501300188644,
                                   0.84125353283118121};
  static constexpr double s[11] = {0,
                                   0.54064081745559756,
                                   0.90963199535451833,
                                   0.98982144188093268,
                                   0.75574957435425827,
                                   0.28173255684142967,
                                   -0.28173255684142967,
                                   -0.75574957435425827,
                                   -0.98982144188093268,
                                   -0.90963199535451833,
                                   -0.54064081745559756};
};
template <>
struct OddTab<13> {
  static constexpr double c[13] = {1,
                                   0.88545602565320991,
                                   0.56806474673115581,
                                   0.12053668025532305,
                                   -0.35460488704253562,
                                   -0.74851074817110108,
                                   -0.97094181742605201,
                                   -0.97094181742605201,
                                   -0.74851074817110108,
                                   -0.35460488704253562,
                                   0.12053668025532305,
                                   0.56806474673115581,
                                   0.88545602565320991};
  static constexpr double s[13] = {0,
                                   0.46472317204376856,
                                   0.82298386589365635,
                                   0.99270887409805397,
                                   0.93501624268541483,
                                   0.66312265824079519,
                                   0.23931566428755777,
                                   -0.23931566428755777,
                                   -0.66312265824079519,
                                   -0.93501624268541483,
                                   -0.99270887409805397,
                                   -0.82298386589365635,
                                   -0.46472317204376856};
};

// Forward DFT of odd prime size R: with a_m = v_m + v_{R-m}, b_m = v_m - v_{R-m},
// X_k = v_0 + sum_m cos(2 pi km/R) a_m - i sum_m sin(2 pi km/R) b_m and
// X_{R-k} the same with +i (k, m = 1 .. (R-1)/2).
template <int R>
__device__ __forceinline__ void dft_odd(cd (&v)[R]) {
  constexpr int H = (R - 1) / 2;
  cd a[H], b[H];
#pragma unroll
  for (int m = 1; m <= H; ++m) {
    a[m - 1] = v[m] + v[R - m];
    b[m - 1] = v[m] - v[R - m];
  }
  cd x0 = v[0];
#pragma unroll
  for (int m = 0; m < H; ++m) x0 = x0 + a[m];
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    cd A = v[0], B = {0.0, 0.0};
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      const double c = OddTab<R>::c[(k * m) % R], s = OddTab<R>::s[(k * m) % R];
      A.x += c * a[m - 1].x;
      A.y += c * a[m - 1].y;
      B.x += s * b[m - 1].x;
      B.y += s * b[m - 1].y;
    }
    v[k] = {A.x + B.y, A.y - B.x};      // A - i B
    v[R - k] = {A.x - B.y, A.y + B.x};  // A + i B
  }
  v[0] = x0;
}

template <int R>
__device__ __forceinline__ void dft_any(cd (&v)[R]) {
  if constexpr ((R & (R - 1)) == 0) {
    Dft<R>::run(v);
  } else {
    dft_odd<R>(v);
  }
}

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
  constexpr int J = 16 / R;
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
          x = lds[j + r * nb];
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
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * t1;
    if (valid && j < nb) {
      int k = 0;
      if constexpr (!FROM_HBM) {
        k = j % ns;
        const cd *w = tw + k * (R - 1);
#pragma unroll
        for (int r = 1; r < R; ++r) v[jj][r] = cmul(v[jj][r], w[r - 1]);
      }
      dft_any<R>(v[jj]);
      const int o = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (TO_HBM) {
          cd y = v[jj][r];
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          gout[o + r * ns] = y;
        } else {
          lds[o + r * ns] = v[jj][r];
        }
      }
    }
  }
}

template <bool INV, int LOAD, int MODE>
__device__ __forceinline__ void mixed_dispatch(int R, int n, int ns, int t1, int tl, bool valid,
                                               const void *gin, cd *gout, cd *lds, const cd *tw,
                                               double scale) {
  switch (R) {
#define GDSP_MIXED_CASE(RR)                                                                 \
  case RR:                                                                                  \
    mixed_pass<RR, INV, LOAD, MODE>(n, ns, t1, tl, valid, gin, gout, lds, tw, scale);       \
    break;
    GDSP_MIXED_CASE(2)
    GDSP_MIXED_CASE(3)
    GDSP_MIXED_CASE(4)
    GDSP_MIXED_CASE(5)
    GDSP_MIXED_CASE(7)
    GDSP_MIXED_CASE(8)
    GDSP_MIXED_CASE(11)
    GDSP_MIXED_CASE(13)
    GDSP_MIXED_CASE(16)
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
  cd *lds = lds_mixed + (sub < d.tpw ? sub : 0) * n;
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
    twoff += ns * (R - 1);
    ns *= R;
  }
}

// ---------------------------------------------------------------------------
// Compile-time specialisations for frequent lengths (BASELINE config 3 is
// n = 3000): the same passes with n, Ns, the thread count and the twiddle
// offsets known to the compiler, every pass inlined into one kernel.
template <int R, bool INV, int LOAD, int MODE, int N, int NS, int T1>
__device__ __forceinline__ void fixed_pass(int tl, bool valid, const void *__restrict__ gin,
                                           cd *__restrict__ gout, cd *lds,
                                           const cd *__restrict__ tw, double scale) {
  constexpr bool FROM_HBM = MODE == MP_FIRST || MODE == MP_SINGLE;
  constexpr bool TO_HBM = MODE == MP_LAST || MODE == MP_SINGLE;
  constexpr int NB = N / R;
  constexpr int J = (NB + T1 - 1) / T1;
  cd v[J][R];
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * T1;
    if (valid && (NB % T1 == 0 || j < NB)) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        cd x;
        if constexpr (!FROM_HBM) {
          x = lds[j + r * NB];
        } else if constexpr (LOAD == LOAD_REAL) {
          x = {reinterpret_cast<const double *>(gin)[j + r * NB], 0.0};
        } else {
          x = reinterpret_cast<const cd *>(gin)[j + r * NB];
          if constexpr (INV) x.y = -x.y;
        }
        v[jj][r] = x;
      }
    }
  }
  if constexpr (MODE == MP_MID) __syncthreads();
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = tl + jj * T1;
    if (valid && (NB % T1 == 0 || j < NB)) {
      const int k = j % NS;
      if constexpr (!FROM_HBM) {
        const cd *w = tw + k * (R - 1);
#pragma unroll
        for (int r = 1; r < R; ++r) v[jj][r] = cmul(v[jj][r], w[r - 1]);
      }
      dft_any<R>(v[jj]);
      const int o = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (TO_HBM) {
          cd y = v[jj][r];
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          gout[o + r * NS] = y;
        } else {
          lds[o + r * NS] = v[jj][r];
        }
      }
    }
  }
}

template <bool INV, int LOAD, int N, int T1, int NS, int TWOFF, int P, int NP, int R,
          int... REST>
__device__ __forceinline__ void fixed_passes(int tl, bool valid, const void *gin, cd *gout,
                                             cd *lds, const cd *tw, double scale) {
  constexpr int MODE = NP == 1 ? MP_SINGLE : P == 0 ? MP_FIRST : P == NP - 1 ? MP_LAST : MP_MID;
  if constexpr (P > 0) __syncthreads();
  fixed_pass<R, INV, LOAD, MODE, N, NS, T1>(tl, valid, gin, gout, lds, tw + TWOFF, scale);
  if constexpr (sizeof...(REST) > 0)
    fixed_passes<INV, LOAD, N, T1, NS * R, (P == 0 ? 0 : TWOFF + NS * (R - 1)), P + 1, NP,
                 REST...>(tl, valid, gin, gout, lds, tw, scale);
}

template <int... RS>
struct FixedGeo {
  static constexpr int N = (RS * ...);
  static constexpr int NP = sizeof...(RS);
  static constexpr int need() {
    int m = 1;
    for (int r : {RS...}) {
      const int nb = N / r, jm = 16 / r, q = (nb + jm - 1) / jm;
      m = q > m ? q : m;
    }
    return m;
  }
  static constexpr int T1 = (need() + 63) / 64 * 64;
};

template <bool INV, int LOAD, int... RS>
__global__ __launch_bounds__(FixedGeo<RS...>::T1) void fft_mixed_fixed_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t batch, const cd *__restrict__ tw,
    double scale) {
  using G = FixedGeo<RS...>;
  __shared__ cd lds[G::N];
  const int tl = threadIdx.x;
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x);
  const bool valid = row < batch;
  const void *gin = LOAD == LOAD_REAL
                        ? (const void *)(reinterpret_cast<const double *>(in) + row * G::N)
                        : (const void *)(reinterpret_cast<const cd *>(in) + row * G::N);
  fixed_passes<INV, LOAD, G::N, G::T1, 1, 0, 0, G::NP, RS...>(tl, valid, gin, out + row * G::N,
                                                              lds, tw, scale);
}

template <int... RS>
static bool launch_fixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                         int64_t batch, const cd *tw, double scale, hipStream_t s) {
  using G = FixedGeo<RS...>;
  uint64_t codes = 0;
  int q = 0;
  for (int r : {RS...}) codes |= (uint64_t)r << (5 * q++);
  if (d.n != G::N || d.codes != codes || G::N * sizeof(cd) > 65536) return false;
  const dim3 grid((unsigned)batch), block(G::T1);
  if (inv)
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<true, LOAD_COMPLEX, RS...>), grid, block, 0, s,
                       in, out, batch, tw, scale);
  else if (load == LOAD_REAL)
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<false, LOAD_REAL, RS...>), grid, block, 0, s, in,
                       out, batch, tw, scale);
  else
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<false, LOAD_COMPLEX, RS...>), grid, block, 0, s,
                       in, out, batch, tw, scale);
  return true;
}

hipError_t launch_fft_mixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  if (d.t1 <= 0 || d.tpw <= 0 || d.t1 * d.tpw > 512) return hipErrorInvalidValue;
  const int64_t nblk = (batch + d.tpw - 1) / d.tpw;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  if (batch <= 0x7fffffff && !getenv("GDSP_MIXED_GENERIC") &&
      launch_fixed<8, 5, 5, 5, 3>(d, inv, load, in, out, batch, tw, scale, s))
    return hipGetLastError();
  const size_t lds = (size_t)d.tpw * (size_t)d.n * sizeof(cd);
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
