// mixed_core.hpp — device building blocks of the mixed-radix kernels
// (fft_mixed.hip, fft_specs*.hip): constant tables and in-register DFTs for
// the odd primes and the composite radices, the XOR-swizzled LDS slot map and
// the per-butterfly twiddle power chain.
#pragma once
#include "fft_device.hpp"
#include "launch.hpp"

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

}  // namespace gdsp
