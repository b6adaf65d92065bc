// fft_device.hpp — gfx950 device building blocks for the go-dsp FFT engine:
// complex128 arithmetic, in-register radix-2/4/8/16 DFTs, the Stockham pass
// (register twiddle + DFT) and the LDS exchange between passes.
//
// Algorithm (replaces fft/radix2.go:80-154, the iterative radix-2 DIT with a
// bit-reversal copy): a Stockham autosort FFT, radix 16 per pass, so N = 4096
// needs 3 passes (vs 12 radix-2 stages) and no bit-reversal: pass p with
// radix R and Ns = product of earlier radices maps butterfly j to inputs
// j + r*N/R and outputs (j/Ns)*Ns*R + j%Ns + r*Ns, with twiddle
// W_{Ns*R}^{(j%Ns)*r}. Each thread owns E (<=16) elements at t + k*T, so the
// first load and the last store are fully coalesced 16-byte-per-lane streams.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#else  // hipRTC (mixed_jit.cpp): no system headers; its runtime header has the types
using __hip_internal::int16_t;
using __hip_internal::int64_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

namespace gdsp {

struct __attribute__((aligned(16))) cd {
  double x, y;
};

__device__ __forceinline__ cd operator+(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd operator-(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd cmul(cd a, cd b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ cd conjg(cd a) { return {a.x, -a.y}; }

// Streaming HBM access for data each launch touches exactly once (transform
// inputs and outputs, Pwelch samples): nontemporal (nt) global_load /
// global_store_dwordx4. Measured on the N = 4096 x 65536 batch: 1.437 ->
// 1.355 ms (5.98 -> 6.34 TB/s); loads alone gain nothing, stores alone half.
// Tables that every workgroup re-reads (twiddles, windows, chirps) keep the
// default policy.
__device__ __forceinline__ cd ld_nt(const cd *p) {
  return {__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y)};
}
__device__ __forceinline__ double ld_nt(const double *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(cd *p, cd v) {
  __builtin_nontemporal_store(v.x, &p->x);
  __builtin_nontemporal_store(v.y, &p->y);
}

// Bounds-checked buffer access to one wave-uniform region [base, base +
// bytes): loads past the end return 0 and stores past it are dropped by the
// hardware, so a row of n elements needs no per-element test or branch (and
// the address is a 32-bit lane offset, not 64-bit arithmetic per element).
// The descriptor must be built from wave-uniform values only.
using rsrc_t = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void *base, int64_t bytes) {
  const int nb = bytes <= 0 ? 0 : (bytes >= 0x7fffffff ? 0x7fffffff : (int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, nb, 0x00020000);
}
__device__ __forceinline__ cd buf_ld(rsrc_t r, uint32_t off) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  cd v;
  __builtin_memcpy(&v, &q, sizeof(cd));
  return v;
}
__device__ __forceinline__ double buf_ld1(rsrc_t r, uint32_t off) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  double v;
  __builtin_memcpy(&v, &q, sizeof(double));
  return v;
}
// soff: a wave-uniform byte offset (SGPR) added outside the range check
__device__ __forceinline__ double buf_ld1s(rsrc_t r, uint32_t off, int soff) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, off, soff, 0);
  double v;
  __builtin_memcpy(&v, &q, sizeof(double));
  return v;
}
// nontemporal store (aux bit 1: nt)
__device__ __forceinline__ void buf_st_nt(rsrc_t r, uint32_t off, cd v) {
  decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0)) q;
  __builtin_memcpy(&q, &v, sizeof(cd));
  __builtin_amdgcn_raw_buffer_store_b128(q, r, off, 0, 2);
}

// cos/sin(pi/8) and sqrt(2)/2 to double precision
#define GDSP_C8 0.92387953251128675613
#define GDSP_S8 0.38268343236508977173
#define GDSP_R2 0.70710678118654752440

// x * exp(-2*pi*i*m/16): forward-direction twiddle by a multiple of 2*pi/16.
// m is a compile-time constant once the callers' loops are unrolled, so the
// switch folds to the special case (free for multiples of 90 degrees, 2 mul
// for odd multiples of 45 degrees).
__device__ __forceinline__ cd rot16(cd x, int m) {
  switch (m & 15) {
    case 0: return x;
    case 4: return {x.y, -x.x};
    case 8: return {-x.x, -x.y};
    case 12: return {-x.y, x.x};
    case 2: return {GDSP_R2 * (x.x + x.y), GDSP_R2 * (x.y - x.x)};
    case 6: return {GDSP_R2 * (x.y - x.x), -GDSP_R2 * (x.x + x.y)};
    case 10: return {-GDSP_R2 * (x.x + x.y), GDSP_R2 * (x.x - x.y)};
    case 14: return {GDSP_R2 * (x.x - x.y), GDSP_R2 * (x.x + x.y)};
    default: break;
  }
  // odd m: w = c - i s with c = cos(2 pi m/16), s = sin(2 pi m/16)
  double c, s;
  switch (m & 15) {
    case 1: c = GDSP_C8; s = GDSP_S8; break;
    case 3: c = GDSP_S8; s = GDSP_C8; break;
    case 5: c = -GDSP_S8; s = GDSP_C8; break;
    case 7: c = -GDSP_C8; s = GDSP_S8; break;
    case 9: c = -GDSP_C8; s = -GDSP_S8; break;
    case 11: c = -GDSP_S8; s = -GDSP_C8; break;
    case 13: c = GDSP_S8; s = -GDSP_C8; break;
    default: c = GDSP_C8; s = -GDSP_S8; break;  // 15
  }
  return {x.x * c + x.y * s, x.y * c - x.x * s};
}

// cos/sin(pi/16) and cos/sin(3 pi/16)
#define GDSP_C16 0.98078528040323044913
#define GDSP_S16 0.19509032201612826785
#define GDSP_C316 0.83146961230254523708
#define GDSP_S316 0.55557023301960222474

// x * exp(-2*pi*i*m/32) (m compile-time after unrolling); even m -> rot16.
__device__ __forceinline__ cd rot32(cd x, int m) {
  m &= 31;
  if ((m & 1) == 0) return rot16(x, m >> 1);
  double c, s;  // w = c - i s, c = cos(pi m/16), s = sin(pi m/16)
  switch (m) {
    case 1: c = GDSP_C16; s = GDSP_S16; break;
    case 3: c = GDSP_C316; s = GDSP_S316; break;
    case 5: c = GDSP_S316; s = GDSP_C316; break;
    case 7: c = GDSP_S16; s = GDSP_C16; break;
    case 9: c = -GDSP_S16; s = GDSP_C16; break;
    case 11: c = -GDSP_S316; s = GDSP_C316; break;
    case 13: c = -GDSP_C316; s = GDSP_S316; break;
    case 15: c = -GDSP_C16; s = GDSP_S16; break;
    case 17: c = -GDSP_C16; s = -GDSP_S16; break;
    case 19: c = -GDSP_C316; s = -GDSP_S316; break;
    case 21: c = -GDSP_S316; s = -GDSP_C316; break;
    case 23: c = -GDSP_S16; s = -GDSP_C16; break;
    case 25: c = GDSP_S16; s = -GDSP_C16; break;
    case 27: c = GDSP_S316; s = -GDSP_C316; break;
    case 29: c = GDSP_C316; s = -GDSP_S316; break;
    default: c = GDSP_C16; s = -GDSP_S16; break;  // 31
  }
  return {x.x * c + x.y * s, x.y * c - x.x * s};
}

// x * W_32^m for a constant m as scale * u(x), with u(x) = (x.x + r x.y,
// x.y - r x.x) (form 1, |cos| >= |sin|: r = tan) or (r x.x + x.y,
// r x.y - x.x) (form 2: r = cot): two FMAs, and the scale folds into the
// add that follows (Linzer-Feig). Not for multiples of 8 (free rotations).
#define GDSP_T16 0.19891236737965800691
#define GDSP_T8 0.41421356237309504880
#define GDSP_T316 0.66817863791929891999
struct RotF {
  int form;
  double scale, r;
};
__device__ __forceinline__ constexpr RotF rotf(int m) {
  switch (m & 31) {
    case 1: return {1, GDSP_C16, GDSP_T16};
    case 2: return {1, GDSP_C8, GDSP_T8};
    case 3: return {1, GDSP_C316, GDSP_T316};
    case 4: return {2, GDSP_R2, 1.0};
    case 5: return {2, GDSP_C316, GDSP_T316};
    case 6: return {2, GDSP_C8, GDSP_T8};
    case 7: return {2, GDSP_C16, GDSP_T16};
    case 9: return {2, GDSP_C16, -GDSP_T16};
    case 10: return {2, GDSP_C8, -GDSP_T8};
    case 11: return {2, GDSP_C316, -GDSP_T316};
    case 12: return {1, -GDSP_R2, -1.0};
    case 13: return {1, -GDSP_C316, -GDSP_T316};
    case 14: return {1, -GDSP_C8, -GDSP_T8};
    case 15: return {1, -GDSP_C16, -GDSP_T16};
    case 17: return {1, -GDSP_C16, GDSP_T16};
    case 18: return {1, -GDSP_C8, GDSP_T8};
    case 19: return {1, -GDSP_C316, GDSP_T316};
    case 20: return {1, -GDSP_R2, 1.0};
    case 21: return {2, -GDSP_C316, GDSP_T316};
    case 22: return {2, -GDSP_C8, GDSP_T8};
    case 23: return {2, -GDSP_C16, GDSP_T16};
    case 25: return {2, -GDSP_C16, -GDSP_T16};
    case 26: return {2, -GDSP_C8, -GDSP_T8};
    case 27: return {2, -GDSP_C316, -GDSP_T316};
    case 28: return {2, -GDSP_R2, -1.0};
    case 29: return {1, GDSP_C316, -GDSP_T316};
    case 30: return {1, GDSP_C8, -GDSP_T8};
    case 31: return {1, GDSP_C16, -GDSP_T16};
    default: return {0, 0.0, 0.0};
  }
}

// p = a + W_32^m b, q = a - W_32^m b (m a compile-time constant after
// unrolling): six FMAs for a nontrivial rotation instead of a complex
// multiply and four adds (eight instructions)
__device__ __forceinline__ void fused_pm(cd a, cd b, int m, cd &p, cd &q) {
  m &= 31;
  if ((m & 7) == 0) {
    const cd wb = rot16(b, m >> 1);
    p = a + wb;
    q = a - wb;
    return;
  }
  const RotF f = rotf(m);
  const cd u = f.form == 1 ? cd{fma(f.r, b.y, b.x), fma(-f.r, b.x, b.y)}
                           : cd{fma(f.r, b.x, b.y), fma(f.r, b.y, -b.x)};
  p = {fma(f.scale, u.x, a.x), fma(f.scale, u.y, a.y)};
  q = {fma(-f.scale, u.x, a.x), fma(-f.scale, u.y, a.y)};
}

// The second stage of an R1 x R2 split (R2 = 2 or 4) with its twiddles
// W_R^(n2 k1) folded into the butterflies (fused_pm): y[n2] are the first
// stage's outputs k1 before rotation, s = 32 / R; out[k2] = sum_n2
// W_R^(n2 k1) y[n2] W_R2^(n2 k2).
template <int R2>
__device__ __forceinline__ void dft_rot_stage(const cd (&y)[R2], int k1, int s, cd (&out)[R2]) {
  if constexpr (R2 == 2) {
    fused_pm(y[0], y[1], k1 * s, out[0], out[1]);
  } else {
    static_assert(R2 == 4, "fused second stage for R2 = 2 or 4");
    cd t0, t1, t2, d;
    fused_pm(y[0], y[2], 2 * k1 * s, t0, t1);
    const cd y1 = rot32(y[1], k1 * s);
    fused_pm(y1, y[3], 3 * k1 * s, t2, d);
    const cd t3 = {d.y, -d.x};  // (a1 - a3) * (-i)
    out[0] = t0 + t2;
    out[1] = t1 + t3;
    out[2] = t0 - t2;
    out[3] = t1 - t3;
  }
}

// In-register forward DFT of size R (natural order in, natural order out).
template <int R>
struct Dft;

template <>
struct Dft<1> {
  __device__ __forceinline__ static void run(cd (&)[1]) {}
};

template <>
struct Dft<2> {
  __device__ __forceinline__ static void run(cd (&a)[2]) {
    cd t = a[0];
    a[0] = t + a[1];
    a[1] = t - a[1];
  }
};

template <>
struct Dft<4> {
  __device__ __forceinline__ static void run(cd (&a)[4]) {
    cd t0 = a[0] + a[2], t1 = a[0] - a[2];
    cd t2 = a[1] + a[3], d = a[1] - a[3];
    cd t3 = {d.y, -d.x};  // (a1 - a3) * (-i)
    a[0] = t0 + t2;
    a[1] = t1 + t3;
    a[2] = t0 - t2;
    a[3] = t1 - t3;
  }
};

// R = R1*R2 split: n = R2*n1 + n2, k = k1 + R1*k2; the twiddles between the
// stages fold into the second stage's butterflies (dft_rot_stage).
template <int R1, int R2>
__device__ __forceinline__ void dft_split(cd (&a)[R1 * R2]) {
  constexpr int R = R1 * R2;
  cd y[R2][R1];
#pragma unroll
  for (int n2 = 0; n2 < R2; ++n2) {
    cd tmp[R1];
#pragma unroll
    for (int n1 = 0; n1 < R1; ++n1) tmp[n1] = a[R2 * n1 + n2];
    Dft<R1>::run(tmp);
#pragma unroll
    for (int k1 = 0; k1 < R1; ++k1) y[n2][k1] = tmp[k1];
  }
#pragma unroll
  for (int k1 = 0; k1 < R1; ++k1) {
    cd col[R2], out[R2];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) col[n2] = y[n2][k1];
    dft_rot_stage<R2>(col, k1, 32 / R, out);
#pragma unroll
    for (int k2 = 0; k2 < R2; ++k2) a[k1 + R1 * k2] = out[k2];
  }
}

template <>
struct Dft<8> {
  __device__ __forceinline__ static void run(cd (&a)[8]) { dft_split<4, 2>(a); }
};
template <>
struct Dft<16> {
  __device__ __forceinline__ static void run(cd (&a)[16]) { dft_split<4, 4>(a); }
};
template <>
struct Dft<32> {
  __device__ __forceinline__ static void run(cd (&a)[32]) { dft_split<8, 4>(a); }
};

// DFTs of inputs known to be zero past a point (a[j] = 0 for j >= NZ, a
// compile-time count), as in the first pass of a chirp-z FFT where the input
// fills at most n of M points: the radix-2 stages that would add a zero are
// left out (compile-time zeros do not fold away by themselves: x + 0.0 is
// not x for x = -0.0).
template <int R, int NZ>
struct DftZ;

// split R1*R2 as dft_split, column n2 of the first stage holding
// ceil((NZ - n2) / R2) nonzero inputs
template <int R1, int R2, int NZ, int N2 = 0>
struct SplitZCol {
  __device__ __forceinline__ static void run(const cd (&a)[R1 * R2], cd (&y)[R2][R1]) {
    if constexpr (N2 < R2) {
      constexpr int C0 = (NZ - N2 + R2 - 1) / R2;
      constexpr int C = C0 < 0 ? 0 : (C0 > R1 ? R1 : C0);
      cd tmp[R1];
#pragma unroll
      for (int n1 = 0; n1 < R1; ++n1) tmp[n1] = a[R2 * n1 + N2];
      if constexpr (C == 0) {
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) y[N2][k1] = {0.0, 0.0};
      } else {
        DftZ<R1, C>::run(tmp);
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) y[N2][k1] = tmp[k1];
      }
      SplitZCol<R1, R2, NZ, N2 + 1>::run(a, y);
    }
  }
};

template <int R1, int R2, int NZ>
__device__ __forceinline__ void dft_split_z(cd (&a)[R1 * R2]) {
  static_assert(NZ >= R2, "every first-stage column holds an input");
  cd y[R2][R1];
  SplitZCol<R1, R2, NZ>::run(a, y);
#pragma unroll
  for (int k1 = 0; k1 < R1; ++k1) {
    cd col[R2], out[R2];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) col[n2] = y[n2][k1];
    dft_rot_stage<R2>(col, k1, 32 / (R1 * R2), out);
#pragma unroll
    for (int k2 = 0; k2 < R2; ++k2) a[k1 + R1 * k2] = out[k2];
  }
}

template <int R, int NZ>
struct DftZ {
  __device__ __forceinline__ static void run(cd (&a)[R]) {
    static_assert(NZ >= 1, "at least one nonzero input");
    if constexpr (NZ >= R) {
      Dft<R>::run(a);
    } else if constexpr (R == 2) {
      a[1] = a[0];
    } else if constexpr (R == 4) {
      // t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3 with zeros left out
      const cd t0 = NZ >= 3 ? a[0] + a[2] : a[0];
      const cd t1 = NZ >= 3 ? a[0] - a[2] : a[0];
      const cd t2 = NZ >= 2 ? a[1] : cd{0.0, 0.0};
      const cd t3 = {t2.y, -t2.x};  // d * (-i), d = a1
      if constexpr (NZ == 1) {
        a[1] = a[0];
        a[2] = a[0];
        a[3] = a[0];
      } else {
        a[0] = t0 + t2;
        a[1] = t1 + t3;
        a[2] = t0 - t2;
        a[3] = t1 - t3;
      }
    } else if constexpr (R == 8) {
      dft_split_z<4, 2, NZ>(a);
    } else if constexpr (R == 16) {
      dft_split_z<4, 4, NZ>(a);
    } else {
      static_assert(R == 32, "pruned DFTs up to 32");
      dft_split_z<8, 4, NZ>(a);
    }
  }
};

// DFT_R of an input that fills at most half of it (a[j] = 0 for j >= NZ,
// NZ <= R/2): X[2m] = DFT_{R/2}(a)[m] and X[2m+1] = DFT_{R/2}(a_j W_R^j)[m],
// one radix-2 stage fewer than Dft<R>, each half pruned to its NZ inputs.
template <int R, int NZ = R / 2>
__device__ __forceinline__ void dft_half_in(cd (&a)[R]) {
  static_assert(R >= 4 && R <= 32, "rot32 covers W_R for R <= 32");
  static_assert(NZ >= 1 && NZ <= R / 2, "input within the first half");
  constexpr int H = R / 2;
  cd e[H], o[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    e[j] = a[j];
    o[j] = j < NZ ? rot32(a[j], j * (32 / R)) : cd{0.0, 0.0};
  }
  DftZ<H, NZ>::run(e);
  DftZ<H, NZ>::run(o);
#pragma unroll
  for (int m = 0; m < H; ++m) {
    a[2 * m] = e[m];
    a[2 * m + 1] = o[m];
  }
}

// XOR-swizzled exchange slots (lds_off; the padded layout i + i/16 it
// replaced left 33 % of the chirp-z kernel's LDS cycles bank-conflicted)
constexpr bool kLdsXor = true;
__host__ __device__ constexpr int clog2(int v) { return v <= 1 ? 0 : 1 + clog2(v / 2); }

// ---------------------------------------------------------------------------
// Geometry of the one-kernel (LDS-resident) transform of N = 2^LOG2N points
// with E = 2^LOG2E elements per thread (16 by default; 8 trades one more
// radix-8 pass for half the data registers).
template <int LOG2N, int LOG2E = 4>
struct Geo {
  static constexpr int N = 1 << LOG2N;
  static constexpr int EMAX = 1 << LOG2E;
  static constexpr int E = N < EMAX ? N : EMAX;    // elements per thread
  static constexpr int T = N / E;                  // threads per transform
  static constexpr int WG = T >= 256 ? T : 256;    // threads per workgroup
  static constexpr int TPW = WG / T;               // transforms per workgroup
  static constexpr int NPE = LOG2N >= LOG2E ? LOG2N / LOG2E : 0;  // radix-E passes
  static constexpr int REM = LOG2N >= LOG2E ? LOG2N % LOG2E : LOG2N;
  static constexpr int NPASS = NPE + (REM ? 1 : 0);
  // exchange slot layout: XOR-swizzled (lds_off) when a transform spans at
  // least 32 threads, padded (one slot per 16 doubles) below
  static constexpr bool XOR = T >= 32 && kLdsXor;
  // doubles per transform: room for every layout lds_off may use
  static constexpr int STRIDE = T >= 32 ? N + N / E : N + N / 16;
  static constexpr int LDS_DOUBLES = NPASS > 1 ? TPW * STRIDE : 1;
  __host__ __device__ static constexpr int radix(int p) { return p < NPE ? EMAX : (1 << REM); }
  __host__ __device__ static constexpr int ns(int p) { return p == 0 ? 1 : ns(p - 1) * radix(p - 1); }
};

// XCD-aware workgroup -> row-group map. Workgroups are dealt round-robin
// over the 8 XCDs (b and b+8 share one), so this gives each XCD a contiguous
// run of rows: the rows an XCD streams at any moment are neighbours in HBM.
// Speed only (MI355X_MICROARCH.md: placement is never a correctness
// property); measured +8.5 % on a 64 KiB-per-workgroup copy and +3 % on the
// N = 4096 batch. Bijective: the tail past a multiple of 8 maps to itself.
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
  const int64_t full = nb & ~(int64_t)7;
  return b < full ? (b & 7) * (full >> 3) + (b >> 3) : b;
}

// one padding slot every 16 doubles keeps the stride-16 writes of pass 0
// conflict-free for ds_write_b64 (bank = (addr/4) mod 32 per 16-lane group)
__device__ __forceinline__ int padi(int i) { return i + (i >> 4); }

// Twiddle + DFT of one Stockham pass on the thread's registers. v[b + r*B]
// holds input r of butterfly j = t + b*T. tw: forward table T_N[k] =
// exp(-2 pi i k/N).
// ZIN: only the first ZIN inputs of every butterfly are nonzero (first pass,
// NS = 1, of a transform whose input fills at most half the points)
// Epilogue of a transform's last pass (EPI::on): butterfly b's outputs k =
// b + r B go through epi.apply(v, k, u, f) with f = epi.load(k) loaded before
// the butterfly's twiddles and DFT, so the load's L2 latency hides behind that
// arithmetic instead of stalling after the pass (outputs with !epi.want(k)
// are neither loaded nor applied). The chirp-z kernel fuses its bhat step and
// its output postmultiply this way.
struct NoEpi {
  static constexpr bool on = false;
  __device__ static constexpr bool want(int) { return false; }
  __device__ cd load(int) const { return {0.0, 0.0}; }
  template <int E>
  __device__ void apply(cd (&)[E], int, cd, cd) const {}
};

// Twiddle base of butterfly j in pass (R, NS): W_{NS R}^(j % NS)
template <int N, int R, int NS>
__device__ __forceinline__ cd pass_base(const cd *__restrict__ tw, int j) {
  return tw[(j & (NS - 1)) * (N / (NS * R))];
}

// Twiddles held in registers (a persistent kernel's loop over many
// transforms of one geometry, every pass of radix R with one butterfly per
// thread, j = t): pass p's base W_{NS R}^(t % NS) is the same for every
// transform, so it is read once per kernel instead of from a table per
// transform. Passed as fft_regs' TWP.
template <int NP>
struct RegTw {
  cd base[NP];  // base[p], p >= 1
};
template <class T>
struct is_regtw {
  static constexpr bool v = false;
};
template <int NP>
struct is_regtw<RegTw<NP>> {
  static constexpr bool v = true;
};

__device__ __forceinline__ cd opaque_cd(cd w) {
  asm volatile("" : "+v"(w.x), "+v"(w.y));
  return w;
}

// WPRE: the butterflies' twiddle bases come in wpre[b] (loaded by the caller
// a pass ahead: fft_regs PREW) instead of being read here
// PASS: this pass's index (selects a RegTw's base)
// CHEB: the powers w^3 .. w^(R-1) by the three-term recurrence
// w^(r+2) = 2 cos(2 theta) w^r - w^(r-2) (two FMAs each) instead of complex
// products (four instructions each); its error grows with the chain length
// (numpy model, largest over the bases: 2.3e-15 at R = 8, 4-10e-15 at
// R = 16, 2e-14 at R = 32 against 1-3e-15 for the products), so callers ask
// for it up to radix 16
template <int N, int E, int T, int R, int NS, int ZIN = 0, class EPI = NoEpi,
          bool WPRE = false, int PASS = 0, class TWP = const cd *, bool CHEB = false>
__device__ __forceinline__ void pass_compute(cd (&v)[E], int t, TWP tw,
                                             const EPI &epi = EPI(), const cd *wpre = nullptr) {
  constexpr int B = E / R;
#pragma unroll
  for (int b = 0; b < B; ++b) {
    const int j = t + b * T;
    cd mf[EPI::on ? R : 1];
    if constexpr (EPI::on) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (EPI::want(b + r * B)) mf[r] = epi.load(b + r * B);
    }
    cd u[R];
#pragma unroll
    for (int r = 0; r < R; ++r) u[r] = v[b + r * B];
    if constexpr (NS > 1) {
      // W_{NS*R}^{(j%NS)*r}: one table read, powers by two interleaved
      // recurrences (odd and even exponents) to keep the product depth ~R/2
      cd w;
      if constexpr (WPRE) w = wpre[b];
      else if constexpr (is_regtw<TWP>::v) {
        static_assert(B == 1, "register twiddles need one butterfly per thread");
        w = tw.base[PASS];
      } else w = pass_base<N, R, NS>(tw, j);
      u[1] = cmul(u[1], w);
      if constexpr (R > 2 && CHEB) {
        const cd w2 = cmul(w, w);
        u[2] = cmul(u[2], w2);
        const double c2 = w2.x + w2.x;
        cd om = conjg(w), o = w;      // odd powers: w^(r-2), w^r
        cd em = {1.0, 0.0}, e = w2;   // even powers
#pragma unroll
        for (int r = 3; r < R; ++r) {
          if (r & 1) {
            const cd n = {fma(c2, o.x, -om.x), fma(c2, o.y, -om.y)};
            om = o;
            o = n;
            u[r] = cmul(u[r], o);
          } else {
            const cd n = {fma(c2, e.x, -em.x), fma(c2, e.y, -em.y)};
            em = e;
            e = n;
            u[r] = cmul(u[r], e);
          }
        }
      } else if constexpr (R > 2) {
        const cd w2 = cmul(w, w);
        cd wo = w, we = w2;
        u[2] = cmul(u[2], w2);
#pragma unroll
        for (int r = 3; r < R; ++r) {
          if (r & 1) {
            wo = cmul(wo, w2);
            u[r] = cmul(u[r], wo);
          } else {
            we = cmul(we, w2);
            u[r] = cmul(u[r], we);
          }
        }
      }
    }
    if constexpr (ZIN > 0 && NS == 1 && R >= 4) {
      static_assert(B == 1, "input pruning of a pass with one butterfly per thread");
      dft_half_in<R, ZIN>(u);
    }
    else Dft<R>::run(u);
    if constexpr (EPI::on) {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (EPI::want(b + r * B)) epi.apply(v, b + r * B, u[r], mf[r]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) v[b + r * B] = u[r];
    }
  }
}

// Stockham exchange through LDS after pass (R, NS): output r of butterfly j
// goes to (j/NS)*NS*R + j%NS + r*NS, then every thread reads back t + k*T.
// SPLIT: real and imaginary halves go through one N-double buffer in turn
// (half the LDS, two more barriers); otherwise two buffers.
// LDS offset of element i of a transform: padded contiguous (ILV = 0), or
// interleaved with ILV transforms (element-major, transform-minor: the
// column tiles of FFT2, where neighbouring lanes are neighbouring columns).
//
// Conflict-free exchange layout (ILV = 0, XOR): slot i ^ ((i >> log2 E) & 15).
// Pass 0 writes i = E*j + r for 16 consecutive j (one ds_write_b64 lane group,
// bank (a/4) mod 32): the XOR spreads them over 16 distinct slot residues
// mod 16; later passes write 16 contiguous slots, and every read is 32
// contiguous slots (one ds_read_b64 group, bank (a/4) mod 64), both permuted
// within an aligned 32-slot block. The earlier padding (i + i/16) left the
// reads 2-way conflicted (slot 32 lands on slot 0's banks) and, at E = 32,
// the pass-0 writes too (stride 34 = 2 mod 16): 33 % of the chirp-z kernel's
// LDS-array cycles were bank conflicts. It needs no pad slots either.

//
// LINEAR (padE): slot i + i / E. Pass 0's stride-E writes become stride E+1,
// every other write and every read a contiguous run, and each address is a
// per-thread base plus a compile-time offset (no VALU per element). At E = 32
// it is conflict-free too; at E = 16 the 32-lane reads stay 2-way conflicted.
// The VALU-bound kernels (fused chirp-z, Pwelch) take it: there an address
// instruction costs what an FP64 one does, while the LDS has slack.
template <int ILV, int E = 16, bool XOR = false, bool LINEAR = false>
__device__ __forceinline__ int lds_off(int i) {
  if constexpr (ILV != 0) return i * ILV;
  else if constexpr (LINEAR && E >= 16) return i + (i >> clog2(E));
  else if constexpr (XOR && kLdsXor) return i ^ ((i >> clog2(E)) & 15);
  else return padi(i);
}

// LAYOUT 2 (E = 16, T >= 32): the first exchange (after a pass with NS = 1,
// whose stride-E writes need the XOR swizzle) as XOR; every later one as
// i + 16 * (i / 256): its writes are runs of >= 16 contiguous slots and its
// reads runs of 32, so a 16-slot shift per 256-block keeps both
// conflict-free, and every address is a per-thread base plus a compile-time
// offset (no vector instruction per element).
template <int ILV, int E, bool XOR, int LAYOUT, int NS_PREV>
__device__ __forceinline__ int xoff(int i) {
  if constexpr (LAYOUT == 2 && ILV == 0 && XOR && E == 16 && NS_PREV > 1)
    return i + ((i >> 8) << 4);
  else
    return lds_off<ILV, E, XOR, LAYOUT == 1>(i);
}

// Exchange synchronisation: the workgroup barrier, or (WS: every transform of
// the workgroup lies inside one wave, in an LDS region of its own) only an
// ordering fence for the compiler — a wave's LDS instructions execute in
// order, so its reads see its own writes without a barrier.
template <bool WS>
__device__ __forceinline__ void xsync() {
  if constexpr (WS) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

template <int N, int E, int T, int R, int NS, bool SPLIT, int ILV = 0, int LAYOUT = 0,
          bool WS = false>
__device__ __forceinline__ void pass_exchange(cd (&v)[E], int t, double *lre, double *lim,
                                              bool first) {
  static_assert(!WS || T <= 64, "wave-synchronised exchanges need a transform inside one wave");
  constexpr int B = E / R;
  // LAYOUT 2 with one butterfly per thread and T = 256 (N = 4096, E = 16),
  // written out so the compiler sees the per-thread base: the first exchange
  // writes 16 t + (r ^ (t & 15)) and reads (t ^ ((t >> 4) & 15)) + 256 k; the
  // second (NS R = 256) writes (t / NS) 272 + t % NS + r NS and reads
  // t + 272 k
  constexpr bool L2 = LAYOUT == 2 && ILV == 0 && E == 16 && T == 256 && B == 1 &&
                      (NS == 1 || NS * R == 256);
  constexpr int BLK = 272;
  // LAYOUT 1 (LINEAR, slot i + i / E) where it is a per-thread base plus a
  // compile-time offset: a first exchange of one butterfly per thread
  // (i = E t + r), or NS a multiple of E (i / E splits exactly)
  constexpr bool LIN = LAYOUT == 1 && ILV == 0 && T >= 32 && E >= 16 && T % E == 0 &&
                       ((NS == 1 && B == 1) || NS % E == 0);
  int dst[E];
  if constexpr (LIN && NS == 1) {
#pragma unroll
    for (int r = 0; r < R; ++r) dst[r] = t * (E + 1) + r;
  } else if constexpr (LIN) {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int j = t + b * T;
      const int a = (j / NS) * (NS * R) + (j & (NS - 1));
      const int base = a + (j / NS) * (NS * R / E) + (j & (NS - 1)) / E;
#pragma unroll
      for (int r = 0; r < R; ++r) dst[b + r * B] = base + r * (NS + NS / E);
    }
  } else if constexpr (L2 && NS == 1) {
    const int m = t & 15;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[r] = 16 * t + (r ^ m);
  } else if constexpr (L2) {
    const int base = (t / NS) * BLK + (t & (NS - 1));
#pragma unroll
    for (int r = 0; r < R; ++r) dst[r] = base + r * NS;
  } else {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int j = t + b * T;
      const int base = (j / NS) * (NS * R) + (j & (NS - 1));
#pragma unroll
      for (int r = 0; r < R; ++r)
        dst[b + r * B] = xoff<ILV, E, (T >= 32), (T >= 32 ? LAYOUT : 0), NS>(base + r * NS);
    }
  }
  // reads of element t + k T: rbase + k rstep
  int rbase = 0, rstep = 0;
  if constexpr (LIN) {
    rbase = t + t / E;
    rstep = T + T / E;
  } else if constexpr (L2 && NS == 1) {
    rbase = t ^ ((t >> 4) & 15);
    rstep = 256;
  } else if constexpr (L2) {
    rbase = t;
    rstep = BLK;
  }
  auto src = [&](int k) -> int {
    if constexpr (L2 || LIN) return rbase + k * rstep;
    else return xoff<ILV, E, (T >= 32), (T >= 32 ? LAYOUT : 0), NS>(t + k * T);
  };
  if (!first) xsync<WS>();
  if constexpr (SPLIT) {
#pragma unroll
    for (int k = 0; k < E; ++k) lre[dst[k]] = v[k].x;
    xsync<WS>();
#pragma unroll
    for (int k = 0; k < E; ++k) v[k].x = lre[src(k)];
    xsync<WS>();
#pragma unroll
    for (int k = 0; k < E; ++k) lre[dst[k]] = v[k].y;
    xsync<WS>();
#pragma unroll
    for (int k = 0; k < E; ++k) v[k].y = lre[src(k)];
  } else {
#pragma unroll
    for (int k = 0; k < E; ++k) {
      lre[dst[k]] = v[k].x;
      lim[dst[k]] = v[k].y;
    }
    xsync<WS>();
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int o = src(k);
      v[k] = {lre[o], lim[o]};
    }
  }
}

// Full forward FFT of the thread's registers (natural order t + k*T in and
// out). The final pass needs no exchange: its outputs already sit at t + k*T.
// Opaque copies of values the compiler would otherwise treat as identical
// across two transforms in one kernel (Bluestein's FFT and inverse FFT, the
// Pwelch loop): without them it keeps every twiddle power and LDS address of
// the first transform live for the second (GVN / LICM), which doubles the
// register footprint (226 -> 128 VGPRs for M = 8192) and halves occupancy.
template <class T>
__device__ __forceinline__ T *opaque_ptr(T *p) {
  // global-memory pointers only: laundered as an address_space(1) pointer,
  // so the loads through it stay global_load (a laundered generic pointer
  // becomes flat_load, which also counts in lgkmcnt and makes every LDS wait
  // wait for the HBM loads in flight)
  __attribute__((address_space(1))) T *q = (__attribute__((address_space(1))) T *)p;
  asm volatile("" : "+s"(q));
  return (T *)q;
}
__device__ __forceinline__ int opaque_int(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// the thread's register array for a transform of geometry Geo<LOG2N, LOG2E>
template <int LOG2N, int LOG2E = 4>
using RegArr = cd[Geo<LOG2N, LOG2E>::E];

// OPAQUE: 0 none; 1 launder the thread index and the twiddle pointer (no
// address or twiddle value survives from one call to the next); 2 launder
// only the thread index — enough to keep twiddle loads inside a loop, and it
// leaves an LDS twiddle pointer's address space visible (ds_read, not flat).
// HALF_IN: elements t + k T with k >= HALF_IN (<= E/2; 0: none) are zero on
// entry (pass 0 prunes one radix-2 stage and the additions of zeros;
// pass_compute)
// EPI: the last pass's epilogue (pass_compute)
// CHEBR: passes of radix <= CHEBR take their twiddle powers by the
// three-term recurrence (pass_compute CHEB; 0: none)
// PREW: each pass's twiddle bases are read before the previous pass's
// arithmetic and exchange (wpre carries them down), so their L1/L2 or LDS
// latency hides behind that work instead of opening the pass; only for
// passes with at most PREW bases per thread (0: off)
// WS: wave-synchronised exchanges (xsync), for transforms inside one wave
template <int LOG2N, bool SPLIT, int OPAQUE = 0, int LOG2E = 4, int ILV = 0, int P = 0,
          class TWP = const cd *, int LINEAR = 0, int HALF_IN = 0, class EPI = NoEpi,
          int PREW = 0, int CHEBR = 0, bool WS = false>
__device__ __forceinline__ void fft_regs(RegArr<LOG2N, LOG2E> &v, int t, TWP tw, double *lre,
                                         double *lim, bool first_exchange = true,
                                         const EPI &epi = EPI(), const cd *wpre = nullptr) {
  using G = Geo<LOG2N, LOG2E>;
  if constexpr (OPAQUE && P == 0 && G::NPASS > 1) {
    t = opaque_int(t);
    if constexpr (OPAQUE == 1 && !is_regtw<TWP>::v) tw = opaque_ptr(tw);
  }
  if constexpr (P < G::NPASS) {
    constexpr int R = G::radix(P);
    constexpr int NS = G::ns(P);
    if constexpr (P > 0) {
      // exchange after the previous pass
      constexpr int RP = G::radix(P - 1);
      constexpr int NSP = G::ns(P - 1);
      pass_exchange<G::N, G::E, G::T, RP, NSP, SPLIT, ILV, LINEAR, WS>(v, t, lre, lim,
                                                                        first_exchange && P == 1);
    }
    // PREW: the next pass's bases, read now
    constexpr int PN = P + 1 < G::NPASS ? P + 1 : P;
    constexpr int RN = G::radix(PN), NSN = G::ns(PN), BN = G::E / RN;
    constexpr bool PRE_NEXT = PREW >= BN && P + 1 < G::NPASS && NSN > 1;
    cd wn[PRE_NEXT ? BN : 1];
    if constexpr (PRE_NEXT) {
#pragma unroll
      for (int b = 0; b < BN; ++b) wn[b] = pass_base<G::N, RN, NSN>(tw, t + b * G::T);
    }
    constexpr bool USE_PRE = PREW >= G::E / R && P > 0 && NS > 1;
    constexpr bool CH = R <= CHEBR;
    if constexpr (P == G::NPASS - 1)
      pass_compute<G::N, G::E, G::T, R, NS, P == 0 ? HALF_IN : 0, EPI, USE_PRE, P, TWP, CH>(
          v, t, tw, epi, wpre);
    else
      pass_compute<G::N, G::E, G::T, R, NS, P == 0 ? HALF_IN : 0, NoEpi, USE_PRE, P, TWP, CH>(
          v, t, tw, NoEpi(), wpre);
    fft_regs<LOG2N, SPLIT, 0, LOG2E, ILV, P + 1, TWP, LINEAR, false, EPI, PREW, CHEBR, WS>(
        v, t, tw, lre, lim, first_exchange, epi, PRE_NEXT ? wn : nullptr);
  }
}

}  // namespace gdsp
