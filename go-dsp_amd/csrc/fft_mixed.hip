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

#include <tuple>

namespace gdsp {

template <int R>
struct OddTab;  // cos / sin(2 pi q / R), q < R (primes and the composite radices)
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

template <>
struct OddTab<6> {
  static constexpr double c[6] = {1, 0.5, -0.5, -1, -0.5, 0.5};
  static constexpr double s[6] = {0, 0.8660254037844386, 0.8660254037844386, -3.8247850373932361e-40, -0.8660254037844386, -0.8660254037844386};
};
template <>
struct OddTab<9> {
  static constexpr double c[9] = {1, 0.76604444311897801, 0.17364817766693036, -0.5, -0.93969262078590843, -0.93969262078590843, -0.5, 0.17364817766693036, 0.76604444311897801};
  static constexpr double s[9] = {0, 0.64278760968653936, 0.98480775301220802, 0.8660254037844386, 0.34202014332566871, -0.34202014332566871, -0.8660254037844386, -0.98480775301220802, -0.64278760968653936};
};
template <>
struct OddTab<10> {
  static constexpr double c[10] = {1, 0.80901699437494745, 0.30901699437494745, -0.30901699437494745, -0.80901699437494745, -1, -0.80901699437494745, -0.30901699437494745, 0.30901699437494745, 0.80901699437494745};
  static constexpr double s[10] = {0, 0.58778525229247314, 0.95105651629515353, 0.95105651629515353, 0.58778525229247314, -3.8247850373932361e-40, -0.58778525229247314, -0.95105651629515353, -0.95105651629515353, -0.58778525229247314};
};
template <>
struct OddTab<12> {
  static constexpr double c[12] = {1, 0.8660254037844386, 0.5, -8.0778275495162712e-41, -0.5, -0.8660254037844386, -1, -0.8660254037844386, -0.5, -8.0778275495162712e-41, 0.5, 0.8660254037844386};
  static constexpr double s[12] = {0, 0.5, 0.8660254037844386, 1, 0.8660254037844386, 0.5, -3.8247850373932361e-40, -0.5, -0.8660254037844386, -1, -0.8660254037844386, -0.5};
};
template <>
struct OddTab<15> {
  static constexpr double c[15] = {1, 0.91354545764260087, 0.66913060635885824, 0.30901699437494745, -0.10452846326765347, -0.5, -0.80901699437494745, -0.97814760073380569, -0.97814760073380569, -0.80901699437494745, -0.5, -0.10452846326765347, 0.30901699437494745, 0.66913060635885824, 0.91354545764260087};
  static constexpr double s[15] = {0, 0.40673664307580021, 0.74314482547739424, 0.95105651629515353, 0.99452189536827329, 0.8660254037844386, 0.58778525229247314, 0.20791169081775934, -0.20791169081775934, -0.58778525229247314, -0.8660254037844386, -0.99452189536827329, -0.95105651629515353, -0.74314482547739424, -0.40673664307580021};
};
template <>
struct OddTab<20> {
  static constexpr double c[20] = {1, 0.95105651629515353, 0.80901699437494745, 0.58778525229247314, 0.30901699437494745, -8.0778275495162712e-41, -0.30901699437494745, -0.58778525229247314, -0.80901699437494745, -0.95105651629515353, -1, -0.95105651629515353, -0.80901699437494745, -0.58778525229247314, -0.30901699437494745, -8.0778275495162712e-41, 0.30901699437494745, 0.58778525229247314, 0.80901699437494745, 0.95105651629515353};
  static constexpr double s[20] = {0, 0.30901699437494745, 0.58778525229247314, 0.80901699437494745, 0.95105651629515353, 1, 0.95105651629515353, 0.80901699437494745, 0.58778525229247314, 0.30901699437494745, -3.8247850373932361e-40, -0.30901699437494745, -0.58778525229247314, -0.80901699437494745, -0.95105651629515353, -1, -0.95105651629515353, -0.80901699437494745, -0.58778525229247314, -0.30901699437494745};
};
template <>
struct OddTab<25> {
  static constexpr double c[25] = {1, 0.96858316112863108, 0.87630668004386358, 0.72896862742141155, 0.53582679497899666, 0.30901699437494745, 0.062790519529313374, -0.18738131458572463, -0.42577929156507266, -0.63742398974868975, -0.80901699437494745, -0.92977648588825146, -0.99211470131447788, -0.99211470131447788, -0.92977648588825146, -0.80901699437494745, -0.63742398974868975, -0.42577929156507266, -0.18738131458572463, 0.062790519529313374, 0.30901699437494745, 0.53582679497899666, 0.72896862742141155, 0.87630668004386358, 0.96858316112863108};
  static constexpr double s[25] = {0, 0.24868988716485479, 0.48175367410171527, 0.68454710592868873, 0.84432792550201508, 0.95105651629515353, 0.99802672842827156, 0.98228725072868872, 0.90482705246601958, 0.77051324277578925, 0.58778525229247314, 0.36812455268467797, 0.12533323356430426, -0.12533323356430426, -0.36812455268467797, -0.58778525229247314, -0.77051324277578925, -0.90482705246601958, -0.98228725072868872, -0.99802672842827156, -0.95105651629515353, -0.84432792550201508, -0.68454710592868873, -0.48175367410171527, -0.24868988716485479};
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
__device__ __forceinline__ void dft_any(cd (&v)[R]);

// Composite R = R1*R2 (n = R2*n1 + n2, k = k1 + R1*k2): R2 DFTs of size R1,
// twiddles W_R^(n2*k1) as constants, then R1 DFTs of size R2.
template <int R1, int R2>
__device__ __forceinline__ void dft_split_gen(cd (&a)[R1 * R2]) {
  constexpr int R = R1 * R2;
  cd y[R2][R1];
#pragma unroll
  for (int n2 = 0; n2 < R2; ++n2) {
    cd tmp[R1];
#pragma unroll
    for (int n1 = 0; n1 < R1; ++n1) tmp[n1] = a[R2 * n1 + n2];
    dft_any<R1>(tmp);
#pragma unroll
    for (int k1 = 0; k1 < R1; ++k1) {
      const int q = (n2 * k1) % R;
      if (q == 0) {
        y[n2][k1] = tmp[k1];
      } else {  // x * (c - i s)
        const double c = OddTab<R>::c[q], sn = OddTab<R>::s[q];
        y[n2][k1] = {tmp[k1].x * c + tmp[k1].y * sn, tmp[k1].y * c - tmp[k1].x * sn};
      }
    }
  }
#pragma unroll
  for (int k1 = 0; k1 < R1; ++k1) {
    cd tmp[R2];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) tmp[n2] = y[n2][k1];
    dft_any<R2>(tmp);
#pragma unroll
    for (int k2 = 0; k2 < R2; ++k2) a[k1 + R1 * k2] = tmp[k2];
  }
}

template <int R>
__device__ __forceinline__ void dft_any(cd (&v)[R]) {
  if constexpr ((R & (R - 1)) == 0) {
    Dft<R>::run(v);
  } else if constexpr (R == 3 || R == 5 || R == 7 || R == 11 || R == 13) {
    dft_odd<R>(v);
  } else if constexpr (R == 6 || R == 10) {
    dft_split_gen<2, R / 2>(v);
  } else if constexpr (R == 12 || R == 20) {
    dft_split_gen<4, R / 4>(v);
  } else if constexpr (R == 9 || R == 15) {
    dft_split_gen<3, R / 3>(v);
  } else {
    static_assert(R == 25, "radix without a DFT");
    dft_split_gen<5, 5>(v);
  }
}

// LDS slot of element i: XOR-swizzled inside aligned groups of 8 slots, so
// the stride-R ds_write_b128 of a first pass (8 lanes = 8 distinct bank
// quads) and the unit-stride reads are both conflict-free. Transforms are
// padded to a multiple of 8 slots.
__device__ __forceinline__ int lsw(int i) { return i ^ ((i >> 3) & 7); }

// v[r] *= W^r for r = 1..R-1 from the one table entry W (= W_{Ns*R}^k): two
// interleaved power chains (odd powers step by W^2 from W, even ones by W^2
// from W^2), depth about R/2.
template <int R>
__device__ __forceinline__ void twiddle_chain(cd (&v)[R], cd w) {
  if constexpr (R > 1) {
    const cd w2 = cmul(w, w);
    cd wo = w, we = w2;
    v[1] = cmul(v[1], wo);
#pragma unroll
    for (int r = 2; r < R; ++r) {
      if (r & 1) {
        wo = cmul(wo, w2);
        v[r] = cmul(v[r], wo);
      } else {
        if (r > 2) we = cmul(we, w2);
        v[r] = cmul(v[r], we);
      }
    }
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

// ---------------------------------------------------------------------------
// Compile-time specialisations for frequent lengths (BASELINE config 3 is
// n = 3000): n, Ns, the thread count and the twiddle offsets are known to the
// compiler and every pass is inlined. Each pass is load -> twiddle + DFT ->
// store; between passes the data crosses LDS either as complex128 (one
// exchange, two barriers) or, with SPLIT, as real then imaginary halves
// through an n-double buffer (half the LDS, so more workgroups per CU, for
// four barriers).
template <int R, int N, int NS, int T1>
struct FPass {
  static constexpr int NB = N / R;
  static constexpr int J = (NB + T1 - 1) / T1;
  static constexpr bool FULL = NB % T1 == 0;
  cd v[J][R];

  __device__ __forceinline__ static bool act(int j, bool valid) {
    return valid && (FULL || j < NB);
  }
  template <bool INV, int LOAD>
  __device__ __forceinline__ void load_hbm(int tl, bool valid, const void *__restrict__ gin) {
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = tl + jj * T1;
      if (act(j, valid)) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if constexpr (LOAD == LOAD_REAL) {
            v[jj][r] = {reinterpret_cast<const double *>(gin)[j + r * NB], 0.0};
          } else {
            v[jj][r] = reinterpret_cast<const cd *>(gin)[j + r * NB];
            if constexpr (INV) v[jj][r].y = -v[jj][r].y;
          }
        }
      }
    }
  }
  // PART 0: real halves, 1: imaginary halves (double buffer), 2: complex
  template <int PART, bool SWZ>
  __device__ __forceinline__ void load_lds(int tl, bool valid, void *lds) {
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = tl + jj * T1;
      if (act(j, valid)) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int i = SWZ ? lsw(j + r * NB) : j + r * NB;
          if constexpr (PART == 2) {
            v[jj][r] = reinterpret_cast<const cd *>(lds)[i];
          } else if constexpr (PART == 0) {
            v[jj][r].x = reinterpret_cast<const double *>(lds)[i];
          } else {
            v[jj][r].y = reinterpret_cast<const double *>(lds)[i];
          }
        }
      }
    }
  }
  __device__ __forceinline__ void compute(int tl, bool valid, const cd *__restrict__ tw) {
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = tl + jj * T1;
      if (act(j, valid)) {
        if constexpr (NS > 1) twiddle_chain<R>(v[jj], tw[j % NS]);
        dft_any<R>(v[jj]);
      }
    }
  }
  template <int PART, bool SWZ>
  __device__ __forceinline__ void store_lds(int tl, bool valid, void *lds) const {
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = tl + jj * T1;
      if (act(j, valid)) {
        const int k = j % NS, o = (j - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int i = SWZ ? lsw(o + r * NS) : o + r * NS;
          if constexpr (PART == 2) {
            reinterpret_cast<cd *>(lds)[i] = v[jj][r];
          } else if constexpr (PART == 0) {
            reinterpret_cast<double *>(lds)[i] = v[jj][r].x;
          } else {
            reinterpret_cast<double *>(lds)[i] = v[jj][r].y;
          }
        }
      }
    }
  }
  template <bool INV>
  __device__ __forceinline__ void store_hbm(int tl, bool valid, cd *__restrict__ gout,
                                            double scale) const {
#pragma unroll
    for (int jj = 0; jj < J; ++jj) {
      const int j = tl + jj * T1;
      if (act(j, valid)) {
        const int k = j % NS, o = (j - k) * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          cd y = v[jj][r];
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          gout[o + r * NS] = y;
        }
      }
    }
  }
};

// exchange prev -> pass (R, NS) through LDS, compute it, then continue
template <bool INV, bool SPLIT, bool SWZ, int N, int T1, int NS, int TWOFF, class Prev, int R,
          int... REST>
__device__ __forceinline__ void fixed_chain(const Prev &prev, int tl, bool valid, cd *gout,
                                            void *lds, const cd *tw, double scale) {
  FPass<R, N, NS, T1> cur;
  if constexpr (SPLIT) {
    prev.template store_lds<0, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<0, SWZ>(tl, valid, lds);
    __syncthreads();
    prev.template store_lds<1, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<1, SWZ>(tl, valid, lds);
  } else {
    prev.template store_lds<2, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<2, SWZ>(tl, valid, lds);
  }
  cur.compute(tl, valid, tw + TWOFF);
  if constexpr (sizeof...(REST) == 0) {
    cur.template store_hbm<INV>(tl, valid, gout, scale);
  } else {
    __syncthreads();  // every read of this exchange lands before the next one's writes
    fixed_chain<INV, SPLIT, SWZ, N, T1, NS * R, TWOFF + NS, FPass<R, N, NS, T1>, REST...>(
        cur, tl, valid, gout, lds, tw, scale);
  }
}

template <int R0, int... RS>
struct FixedGeo {
  static constexpr int N = R0 * (RS * ... * 1);
  static constexpr int need() {
    int m = 1;
    for (int r : {R0, RS...}) {
      const int nb = N / r, jm = r > 16 ? 1 : 16 / r, q = (nb + jm - 1) / jm;
      m = q > m ? q : m;
    }
    return m;
  }
  static constexpr int T1 = need();
  static constexpr int SLOTS = (N + 7) & ~7;
  // transforms per workgroup: about 256 threads, within 64 KiB of LDS
  static constexpr int tpw() {
    int t = 256 / T1 > 1 ? 256 / T1 : 1;
    while (t > 1 && t * SLOTS * 16 > 65536) --t;
    return t;
  }
  static constexpr int TPW = tpw();
  static constexpr int WG = TPW * T1;
};

template <bool INV, int LOAD, bool SPLIT, bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((FixedGeo<R0, RS...>::WG)) void fft_mixed_fixed_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t batch, const cd *__restrict__ tw,
    double scale) {
  using G = FixedGeo<R0, RS...>;
  __shared__ double lds[G::TPW * (SPLIT ? G::SLOTS : 2 * G::SLOTS)];
  const int sub = G::TPW == 1 ? 0 : (int)threadIdx.x / G::T1;
  const int tl = (int)threadIdx.x - sub * G::T1;
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x) * G::TPW + sub;
  const bool valid = row < batch;
  const void *gin = LOAD == LOAD_REAL
                        ? (const void *)(reinterpret_cast<const double *>(in) + row * G::N)
                        : (const void *)(reinterpret_cast<const cd *>(in) + row * G::N);
  double *ld = lds + sub * (SPLIT ? G::SLOTS : 2 * G::SLOTS);
  FPass<R0, G::N, 1, G::T1> p0;
  p0.template load_hbm<INV, LOAD>(tl, valid, gin);
  p0.compute(tl, valid, tw);
  if constexpr (sizeof...(RS) == 0)
    p0.template store_hbm<INV>(tl, valid, out + row * G::N, scale);
  else
    fixed_chain<INV, SPLIT, SWZ, G::N, G::T1, R0, 0, FPass<R0, G::N, 1, G::T1>, RS...>(
        p0, tl, valid, out + row * G::N, ld, tw, scale);
}

template <bool SPLIT, int... RS>
static bool launch_fixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                         int64_t batch, const cd *tw, double scale, hipStream_t s) {
  using G = FixedGeo<RS...>;
  // an odd first radix writes stride-R slots that are conflict-free as they
  // are; an even one goes through the swizzle
  constexpr int R0 = [] { constexpr int r[] = {RS...}; return r[0]; }();
  constexpr bool SWZ = R0 % 2 == 0;
  uint64_t codes = 0;
  int q = 0;
  for (int r : {RS...}) codes |= (uint64_t)r << (5 * q++);
  if (d.n != G::N || d.codes != codes) return false;
  const dim3 grid((unsigned)((batch + G::TPW - 1) / G::TPW)), block(G::WG);
  if (inv)
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<true, LOAD_COMPLEX, SPLIT, SWZ, RS...>), grid,
                       block, 0, s, in, out, batch, tw, scale);
  else if (load == LOAD_REAL)
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<false, LOAD_REAL, SPLIT, SWZ, RS...>), grid,
                       block, 0, s, in, out, batch, tw, scale);
  else
    hipLaunchKernelGGL((fft_mixed_fixed_kernel<false, LOAD_COMPLEX, SPLIT, SWZ, RS...>), grid,
                       block, 0, s, in, out, batch, tw, scale);
  return true;
}

// The compiled specialisations: radix lists of frequent lengths, each pass a
// radix <= 25 so a length takes 3 passes (2 LDS exchanges).
template <int... RS>
struct Spec {};
using Specs = std::tuple<Spec<25, 15, 8>,    // 3000 (BASELINE config 3)
                         Spec<10, 10, 10>,   // 1000
                         Spec<25, 5, 16>,    // 2000
                         Spec<15, 10, 10>,   // 1500
                         Spec<25, 6, 16>,    // 2400
                         Spec<25, 3, 16>,    // 1200
                         Spec<15, 8, 8>,     // 960
                         Spec<15, 16, 8>,    // 1920
                         Spec<15, 8, 4>,     // 480
                         Spec<12, 16, 8>,    // 1536
                         Spec<12, 16, 16>>;  // 3072

template <int... RS>
static bool spec_radices(Spec<RS...>, int n, int *rad, int *npass) {
  if (n != (RS * ...)) return false;
  int q = 0;
  for (int r : {RS...}) rad[q++] = r;
  *npass = q;
  return true;
}
template <class... S>
static bool find_spec(std::tuple<S...>, int n, int *rad, int *npass) {
  return (spec_radices(S{}, n, rad, npass) || ...);
}
template <int... RS>
static bool spec_launch(Spec<RS...>, const MixedDesc &d, bool inv, int load, const void *in,
                        cd *out, int64_t batch, const cd *tw, double scale, hipStream_t s) {
  return launch_fixed<false, RS...>(d, inv, load, in, out, batch, tw, scale, s);
}
template <class... S>
static bool launch_spec(std::tuple<S...>, const MixedDesc &d, bool inv, int load, const void *in,
                        cd *out, int64_t batch, const cd *tw, double scale, hipStream_t s) {
  return (spec_launch(S{}, d, inv, load, in, out, batch, tw, scale, s) || ...);
}

// ---------------------------------------------------------------------------
// Fused Welch accumulation on a compiled specialisation (spectral/pwelch.go:
// 104-122 for smooth NFFT / Pad = one of the Specs lengths): the same packed
// segment pairs as pwelch_kernel (z = w*x_s0 + i*w*x_s1, the k / F-k fold in
// finalise), but every pass inlined with compile-time radices instead of the
// runtime-radix pass functions of pwelch_mixed_kernel. Each workgroup slot is
// one persistent worker; the power sums of the bins a thread's last-pass
// butterflies produce stay in its registers across the worker's pairs.

// fixed_chain with the last pass handed to a sink instead of stored
template <bool SPLIT, bool SWZ, int N, int T1, int NS, int TWOFF, class Prev, class F, int R,
          int... REST>
__device__ __forceinline__ void fixed_chain_to(const Prev &prev, int tl, bool valid, void *lds,
                                               const cd *tw, F &sink) {
  FPass<R, N, NS, T1> cur;
  if constexpr (SPLIT) {
    prev.template store_lds<0, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<0, SWZ>(tl, valid, lds);
    __syncthreads();
    prev.template store_lds<1, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<1, SWZ>(tl, valid, lds);
  } else {
    prev.template store_lds<2, SWZ>(tl, valid, lds);
    __syncthreads();
    cur.template load_lds<2, SWZ>(tl, valid, lds);
  }
  cur.compute(tl, valid, tw + TWOFF);
  if constexpr (sizeof...(REST) == 0) {
    sink(cur);
  } else {
    __syncthreads();
    fixed_chain_to<SPLIT, SWZ, N, T1, NS * R, TWOFF + NS, FPass<R, N, NS, T1>, F, REST...>(
        cur, tl, valid, lds, tw, sink);
  }
}

template <int R0, int... RS>
struct FixedLast {
  static constexpr int rr[] = {R0, RS...};
  static constexpr int R = rr[sizeof...(RS)];
  static constexpr int N = FixedGeo<R0, RS...>::N;
  using Pass = FPass<R, N, N / R, FixedGeo<R0, RS...>::T1>;
};

template <bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((FixedGeo<R0, RS...>::WG)) void pwelch_fixed_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t pairs_per_worker, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  static_assert(sizeof...(RS) >= 1, "at least two passes");
  using G = FixedGeo<R0, RS...>;
  using L = FixedLast<R0, RS...>;
  using First = FPass<R0, G::N, 1, G::T1>;
  __shared__ double lds[G::TPW * 2 * G::SLOTS];
  const int sub = G::TPW == 1 ? 0 : (int)threadIdx.x / G::T1;
  const int tl = (int)threadIdx.x - sub * G::T1;
  const int64_t worker = (int64_t)blockIdx.x * G::TPW + sub;
  double *ld = lds + sub * 2 * G::SLOTS;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t p0 = worker * pairs_per_worker;
  double acc[L::Pass::J][L::R];
#pragma unroll
  for (int jj = 0; jj < L::Pass::J; ++jj)
#pragma unroll
    for (int r = 0; r < L::R; ++r) acc[jj][r] = 0.0;
  for (int64_t it = 0; it < pairs_per_worker; ++it) {
    const int64_t p = p0 + it;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * (active ? p : 0);
    const bool has1 = active && s0 + 1 < seg_end;
    const double *x0 = opaque_ptr(x) + s0 * stride, *x1 = x0 + stride;
    // laundered per pair: otherwise the compiler hoists the loop-invariant
    // window values and twiddle power chains out of the loop, and the
    // registers they pin halve the occupancy
    const double *w = opaque_ptr(win);
    const cd *twp = opaque_ptr(tw);
    const int tt = opaque_int(tl);
    First f0;
#pragma unroll
    for (int jj = 0; jj < First::J; ++jj) {
      const int j = tt + jj * G::T1;
      if (First::act(j, true)) {
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          const int i = j + r * First::NB;
          double a = 0.0, b = 0.0;
          if (active && i < nfft) {
            const double wi = w[i];
            a = wi * x0[i];
            if (has1) b = wi * x1[i];
          }
          f0.v[jj][r] = {a, b};
        }
      }
    }
    f0.compute(tt, true, twp);
    if (it > 0) __syncthreads();  // the previous pair's last exchange reads are done
    auto sink = [&](const typename L::Pass &c) {
      if (!active) return;
#pragma unroll
      for (int jj = 0; jj < L::Pass::J; ++jj) {
        const int j = tt + jj * G::T1;
        if (L::Pass::act(j, true)) {
#pragma unroll
          for (int r = 0; r < L::R; ++r)
            acc[jj][r] += c.v[jj][r].x * c.v[jj][r].x + c.v[jj][r].y * c.v[jj][r].y;
        }
      }
    };
    fixed_chain_to<false, SWZ, G::N, G::T1, R0, 0, First, decltype(sink), RS...>(f0, tt, true, ld,
                                                                                twp, sink);
  }
  if (p0 < npairs) {
    double *dst = partial + worker * G::N;
#pragma unroll
    for (int jj = 0; jj < L::Pass::J; ++jj) {
      const int j = tl + jj * G::T1;
      if (L::Pass::act(j, true)) {
        constexpr int NSL = G::N / L::R;
        const int k = j % NSL, o = (j - k) * L::R + k;
#pragma unroll
        for (int r = 0; r < L::R; ++r) dst[o + r * NSL] = acc[jj][r];
      }
    }
  }
}

template <int... RS>
static int spec_pw_tpw(Spec<RS...>, const MixedDesc &d) {
  uint64_t codes = 0;
  int q = 0;
  for (int r : {RS...}) codes |= (uint64_t)r << (5 * q++);
  return (d.n == FixedGeo<RS...>::N && d.codes == codes) ? FixedGeo<RS...>::TPW : 0;
}
template <class... S>
static int find_pw_tpw(std::tuple<S...>, const MixedDesc &d) {
  int t = 0;
  ((t = t ? t : spec_pw_tpw(S{}, d)), ...);
  return t;
}
int pwelch_fixed_workers_per_block(const MixedDesc &d) { return find_pw_tpw(Specs{}, d); }

template <int... RS>
static bool spec_pw_launch(Spec<RS...>, const MixedDesc &d, const double *x, int64_t nfft,
                           int64_t stride, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                           int64_t nworkers, const double *win, const cd *tw, double *partial,
                           hipStream_t s) {
  if (!spec_pw_tpw(Spec<RS...>{}, d)) return false;
  using G = FixedGeo<RS...>;
  constexpr int R0 = [] { constexpr int r[] = {RS...}; return r[0]; }();
  const dim3 grid((unsigned)((nworkers + G::TPW - 1) / G::TPW)), block(G::WG);
  hipLaunchKernelGGL((pwelch_fixed_kernel<R0 % 2 == 0, RS...>), grid, block, 0, s, x, nfft, stride,
                     seg_begin, seg_end, ppw, win, tw, partial);
  return true;
}
template <class... S>
static bool launch_pw_spec(std::tuple<S...>, const MixedDesc &d, const double *x, int64_t nfft,
                           int64_t stride, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                           int64_t nworkers, const double *win, const cd *tw, double *partial,
                           hipStream_t s) {
  return (spec_pw_launch(S{}, d, x, nfft, stride, seg_begin, seg_end, ppw, nworkers, win, tw,
                         partial, s) ||
          ...);
}

hipError_t launch_pwelch_fixed(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,
                               int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                               const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (nworkers <= 0 || nworkers > 0x7fffffff) return hipErrorInvalidValue;
  if (!launch_pw_spec(Specs{}, d, x, nfft, stride, seg_begin, seg_end, ppw, nworkers, win, tw,
                      partial, s))
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Radix list of the compiled specialisation for n, if there is one
// (launch_fft_mixed picks the kernel by n and list). GDSP_MIXED_GENERIC=1
// disables them. n = 3000: 1.10 ms per 65536 transforms for 25*15*8 against
// 1.14-1.18 ms for the other orders of these radices and 1.82 ms for the
// generic 8*5*5*5*3 kernel; a split (re/im) exchange measured 3-4 % slower.
bool mixed_fixed_radices(int n, int *rad, int *npass) {
  if (getenv("GDSP_MIXED_GENERIC")) return false;
  return find_spec(Specs{}, n, rad, npass);
}

hipError_t launch_fft_mixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  if (d.t1 <= 0 || d.tpw <= 0 || d.t1 * d.tpw > 512) return hipErrorInvalidValue;
  const int64_t nblk = (batch + d.tpw - 1) / d.tpw;
  if (nblk > 0x7fffffff) return hipErrorInvalidValue;
  if (batch > (int64_t)0x7fffffff) return hipErrorInvalidValue;
  if (launch_spec(Specs{}, d, inv, load, in, out, batch, tw, scale, s)) return hipGetLastError();
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
