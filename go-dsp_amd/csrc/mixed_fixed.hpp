// mixed_fixed.hpp — compile-time mixed-radix specialisations: the inlined
// pass chain (FPass / fixed_chain), the batched transform kernel and the
// fused Pwelch kernel on it, and GDSP_SPEC_GROUP, which instantiates a list
// of radix lists in one translation unit (fft_specs*.hip).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdlib.h>

#include <tuple>
#endif

#include "mixed_core.hpp"

namespace gdsp {

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
  static constexpr int RV = R, NSV = NS;  // (the pass's radix and stride, for sinks)
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
    constexpr int rl[] = {R0, RS...};  // (no std::initializer_list under hipRTC)
    for (int r : rl) {
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

#ifndef __HIPCC_RTC__  // host-side launch helpers
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

template <int... RS>
struct Spec {};

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
  // above 4096 points the complex exchange would exceed 64 KiB: re/im halves
  return launch_fixed<(FixedGeo<RS...>::N > 4096), RS...>(d, inv, load, in, out, batch, tw, scale,
                                                          s);
}
template <class... S>
static bool launch_spec(std::tuple<S...>, const MixedDesc &d, bool inv, int load, const void *in,
                        cd *out, int64_t batch, const cd *tw, double scale, hipStream_t s) {
  return (spec_launch(S{}, d, inv, load, in, out, batch, tw, scale, s) || ...);
}

#endif  // __HIPCC_RTC__

// ---------------------------------------------------------------------------
// Fused Welch accumulation on a compiled specialisation (spectral/pwelch.go:
// 104-122 for smooth NFFT / Pad = a specialised length): the same packed
// segment pairs as pwelch_kernel (z = w*x_s0 + i*w*x_s1, the k / F-k fold in
// finalise), but every pass inlined with compile-time radices instead of the
// runtime-radix pass functions of pwelch_mixed_kernel. Each workgroup slot is
// one persistent worker; the power sums of the bins a thread's last-pass
// butterflies produce stay in its registers across the worker's pairs.

// Workgroup barrier of the fixed chains: __syncthreads, or (BARE) only
// s_waitcnt lgkmcnt(0) + s_barrier — what an LDS exchange needs, without the
// workgroup fence, which would also wait for an LDS-DMA still in flight (a
// pending LDS write, counted in vmcnt).
template <bool BARE>
__device__ __forceinline__ void chain_sync() {
  if constexpr (BARE)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else
    __syncthreads();
}

// fixed_chain with the last pass handed to a sink instead of stored
template <bool BARE, bool SPLIT, bool SWZ, int N, int T1, int NS, int TWOFF, class Prev, class F,
          int R, int... REST>
__device__ __forceinline__ void fixed_chain_sink(const Prev &prev, int tl, bool valid, void *lds,
                                                 const cd *tw, F &sink) {
  FPass<R, N, NS, T1> cur;
  if constexpr (SPLIT) {
    prev.template store_lds<0, SWZ>(tl, valid, lds);
    chain_sync<BARE>();
    cur.template load_lds<0, SWZ>(tl, valid, lds);
    chain_sync<BARE>();
    prev.template store_lds<1, SWZ>(tl, valid, lds);
    chain_sync<BARE>();
    cur.template load_lds<1, SWZ>(tl, valid, lds);
  } else {
    prev.template store_lds<2, SWZ>(tl, valid, lds);
    chain_sync<BARE>();
    cur.template load_lds<2, SWZ>(tl, valid, lds);
  }
  cur.compute(tl, valid, tw + TWOFF);
  if constexpr (sizeof...(REST) == 0) {
    sink(cur);
  } else {
    chain_sync<BARE>();
    fixed_chain_sink<BARE, SPLIT, SWZ, N, T1, NS * R, TWOFF + NS, FPass<R, N, NS, T1>, F, REST...>(
        cur, tl, valid, lds, tw, sink);
  }
}
template <bool SPLIT, bool SWZ, int N, int T1, int NS, int TWOFF, class Prev, class F, int R,
          int... REST>
__device__ __forceinline__ void fixed_chain_to(const Prev &prev, int tl, bool valid, void *lds,
                                               const cd *tw, F &sink) {
  fixed_chain_sink<false, SPLIT, SWZ, N, T1, NS, TWOFF, Prev, F, R, REST...>(prev, tl, valid, lds,
                                                                             tw, sink);
}

// Rows of a two-pass mixed four-step (n = L * N, N = prod RS a smooth
// non-power-of-2 length <= 1024; gdsp_api.hip exec_mixed4): W consecutive
// rows k1 of the L x N matrix per workgroup, DFT_N along each (the inlined
// chain, exchanges as real / imaginary halves), then the transpose
// X[k1 + L k2] = Y[k1][k2] through LDS into the store, so each store
// wave-instruction writes W consecutive k1 (W * 16-B segments; the power-of-2
// rows' rowfft_t_kernel does the same). CSO: conj and scale on the way out
// (an inverse). `rows` = batch * L; rows past it load a valid row and store
// nothing.
template <int W, bool CSO, int N, int T1>
struct RowtSink {  // the last pass's outputs, staged transposed and stored
  double *lds;
  cd *out;
  int64_t L, rows, g0;
  int sub, tl;
  double scale;
  template <class P>
  __device__ __forceinline__ void operator()(const P &cur) const {
    constexpr int NQ = (N + T1 - 1) / T1;
    const int lt = (int)threadIdx.x, s = lt % W, a0 = lt / W;
    const int64_t g = g0 + s, b = g / L, k1 = g - b * L;
    cd *dst = out + b * L * N + k1;
    double re[NQ];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // every read of the last exchange (or the real parts) is done
#pragma unroll
      for (int jj = 0; jj < P::J; ++jj) {
        const int j = tl + jj * T1;
        if (P::act(j, true)) {
          const int k = j % P::NSV, o = (j - k) * P::RV + k;
#pragma unroll
          for (int r = 0; r < P::RV; ++r)
            lds[(o + r * P::NSV) * (W + 1) + sub] = h ? cur.v[jj][r].y : cur.v[jj][r].x;
        }
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int a = a0 + q * T1;
        if (a < N) {
          const double d = lds[a * (W + 1) + s];
          if (h == 0) {
            re[q] = d;
          } else if (g < rows) {
            cd o = {re[q], d};
            if constexpr (CSO) o = {o.x * scale, -o.y * scale};
            st_nt(&dst[(int64_t)a * L], o);
          }
        }
      }
    }
  }
};

template <int W, bool CSO, bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((W * FixedGeo<R0, RS...>::T1)) void rowt_fixed_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t L, int64_t rows,
    const cd *__restrict__ tw, double scale) {
  using G = FixedGeo<R0, RS...>;
  constexpr int N = G::N, T1 = G::T1, SL = G::SLOTS;
  constexpr int XD = W * SL, SD = N * (W + 1);
  __shared__ double lds[XD > SD ? XD : SD];
  const int sub = (int)threadIdx.x / T1;
  const int tl = (int)threadIdx.x - sub * T1;
  const int64_t g0 = (int64_t)blockIdx.x * W;
  const int64_t gl = g0 + sub < rows ? g0 + sub : rows - 1;
  RowtSink<W, CSO, N, T1> sink{lds, out, L, rows, g0, sub, tl, scale};
  FPass<R0, N, 1, T1> p0;
  p0.template load_hbm<false, LOAD_COMPLEX>(tl, true, in + gl * N);
  p0.compute(tl, true, tw);
  if constexpr (sizeof...(RS) == 0)
    sink(p0);
  else
    fixed_chain_to<true, SWZ, N, T1, R0, 0, FPass<R0, N, 1, T1>, RowtSink<W, CSO, N, T1>, RS...>(
        p0, tl, true, lds + sub * SL, tw, sink);
}

template <int R0, int... RS>
struct FixedLast {
  static constexpr int rr[sizeof...(RS) + 1] = {R0, RS...};
  static constexpr int R = rr[sizeof...(RS)];
  static constexpr int N = FixedGeo<R0, RS...>::N;
  using Pass = FPass<R, N, N / R, FixedGeo<R0, RS...>::T1>;
};

// twiddle bases the chained passes of a fixed chain read (tw + TWOFF, TWOFF
// = the sum of the earlier passes' NS): R0 + R0 R1 + ... + N / R_last
template <int R0, int... RS>
struct FixedTwN {
  static constexpr int n() {
    constexpr int rl[] = {R0, RS...};
    int ns = 1, t = 0;
    for (int i = 0; i + 1 < (int)(sizeof...(RS) + 1); ++i) {
      ns *= rl[i];
      t += ns;
    }
    return t;
  }
  static constexpr int N = n();
};

// The fused Pwelch's LDS-DMA form: one transform per workgroup, the next
// pair's samples landing in an LDS stage by LDS-DMA while this pair's FFT
// runs (the exchange as re/im halves, the chained passes' twiddle bases in
// LDS so that no global load's wait drains the DMA: vmcnt is in order), where
// the three fit 80 KiB (two workgroups per CU) — taken for a radix-25 first
// pass, whose 25 points per thread of both segments and the window, loaded by
// the pass itself, hold the registers to two waves per SIMD with the loads
// exposed at every pair. Per 2^28 samples (profiles/r05/pwelch_fixed_dma_ab.txt):
// 3000 / 1500 (25 15 8) 1.90 -> 1.69 ms, 2000 / 1000 (25 5 16) 2.83 -> 2.34.
// The other lists measured slower this way (1500 / 700, 15 10 10: 1.21 ->
// 1.33; 2205 / 1102: 1.24 -> 1.55), as did staging each pair through the
// exchange buffer without the DMA (10 10 10, 12 16 8, 15 8 4: 7-20 %).
// Lists whose fused Pwelch is faster held to more waves per SIMD than the
// compiler's natural count, measured per list (scripts/archive/gpu_r05_w4.sh, w5.sh,
// profiles/r05/pwelch_wpe_ab.txt); it pays where it adds a resident workgroup
// per CU for few spills:
//  - 6000 15 5 5 16 (the fused Pwelch's own list; seven-wave workgroups) at
//    four waves per SIMD — 128 VGPRs, 32 spilled, two workgroups per CU
//    instead of one — 2.16-2.17 against 2.45-2.46 ms per 2^28 samples;
//  - 4500 15 20 15 (five-wave workgroups) at four — 128 VGPRs, 30 spilled,
//    three workgroups per CU instead of two — 2.36-2.38 against 2.77 ms.
// Not kept: 2000 10 10 20 at four (45 spilled) 1.49-1.50 against 1.30 ms,
// 2400 15 16 10 at three (30 spilled) 1.57 against 1.26-1.28 ms (they had
// two or more workgroups per CU already); the other lists above 4096 spill
// 140-510 VGPRs held to two workgroups per CU; and of seven more lists with
// 4-42 spills at the cap that adds a workgroup per CU (160, 150, 1000, 882,
// 4410, 2880, 2560; scripts/archive/gpu_r05_w6.sh) six lost 2-58 % and 150 gained
// 2 %. 0: no override.
template <int... RS>
struct PwWpe {
  static constexpr int v = 0;
};
template <>
struct PwWpe<15, 5, 5, 16> {
  static constexpr int v = 4;
};
template <>
struct PwWpe<15, 20, 15> {
  static constexpr int v = 4;
};

template <int R0, int... RS>
struct PwfDma {
  using G = FixedGeo<R0, RS...>;
  static constexpr int STG = (2 * G::SLOTS + 127) / 128 * 128;  // whole 1 KiB DMA pieces
  static constexpr bool on = R0 == 25 && G::TPW == 1 && G::N <= 4096 &&
                             8 * (G::SLOTS + STG) + 16 * FixedTwN<R0, RS...>::N <= 81920;
  // registers held to two waves per SIMD (amdgpu_waves_per_eu), except for a
  // radix-25 first pass loading its own elements: there the cap serialises
  // its 75 loads (25 15 8 direct: 3.25 ms per 2^28 samples held to two waves
  // against 1.90 at the compiler's choice, one wave with AGPRs); elsewhere it
  // helps or is neutral (1500 / 700, 15 10 10: 1.18 against 1.47 ms;
  // profiles/r05/pwelch_fixed_dma_ab.txt)
  static constexpr int wpe() {
    return PwWpe<R0, RS...>::v ? PwWpe<R0, RS...>::v : on || R0 != 25 ? 2 : 1;
  }
};

template <bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((FixedGeo<R0, RS...>::WG))
__attribute__((amdgpu_waves_per_eu(PwfDma<R0, RS...>::wpe()))) void pwelch_fixed_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t pairs_per_worker, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  static_assert(sizeof...(RS) >= 1, "at least two passes");
  using G = FixedGeo<R0, RS...>;
  using L = FixedLast<R0, RS...>;
  using First = FPass<R0, G::N, 1, G::T1>;
  constexpr bool SPL = G::N > 4096;  // re/im halves: the complex exchange would exceed 64 KiB
  constexpr int TWN = FixedTwN<R0, RS...>::N;
  constexpr int STG = PwfDma<R0, RS...>::STG;
  constexpr bool DMA = PwfDma<R0, RS...>::on;
  constexpr int LDSD = DMA ? G::SLOTS + STG + 2 * TWN : G::TPW * (SPL ? 1 : 2) * G::SLOTS;
  __shared__ double lds[LDSD];
  const int sub = G::TPW == 1 ? 0 : (int)threadIdx.x / G::T1;
  const int tl = (int)threadIdx.x - sub * G::T1;
  const int64_t worker = (int64_t)blockIdx.x * G::TPW + sub;
  double *ld = lds + sub * (SPL ? 1 : 2) * G::SLOTS;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t nfull = (seg_end - seg_begin) / 2;  // pairs with both segments
  const bool nopad = nfft == G::N;
  const int64_t p0 = worker * pairs_per_worker;
  double acc[L::Pass::J][L::R];
#pragma unroll
  for (int jj = 0; jj < L::Pass::J; ++jj)
#pragma unroll
    for (int r = 0; r < L::R; ++r) acc[jj][r] = 0.0;
  // |Z_k|^2 of the last pass's outputs into the thread's sums
  auto accumulate = [&](const typename L::Pass &c, int tt) {
#pragma unroll
    for (int jj = 0; jj < L::Pass::J; ++jj) {
      const int j = tt + jj * G::T1;
      if (L::Pass::act(j, true)) {
#pragma unroll
        for (int r = 0; r < L::R; ++r)
          acc[jj][r] = fma(c.v[jj][r].y, c.v[jj][r].y, fma(c.v[jj][r].x, c.v[jj][r].x, acc[jj][r]));
      }
    }
  };
  // first-pass inputs of the pair whose samples sit at src (segment s0 at
  // src[0 ..), s0 + 1 at src[stride ..)): windowed, masked unless the pair is
  // full and unpadded
  auto first_from = [&](First &f0, const double *src, const double *w, int tt, bool full,
                        bool active, bool has1) {
    const int so = (int)stride;
#pragma unroll
    for (int jj = 0; jj < First::J; ++jj) {
      const int j = tt + jj * G::T1;
      if (First::act(j, true)) {
#pragma unroll
        for (int r = 0; r < R0; ++r) {
          const int i = j + r * First::NB;
          const bool in = i < nfft;
          const double wi = w[in ? i : (int)nfft - 1];
          const double a = src[i], b = src[so + i];
          if (full)
            f0.v[jj][r] = {wi * a, wi * b};
          else
            f0.v[jj][r] = {active && in ? wi * a : 0.0, has1 && in ? wi * b : 0.0};
        }
      }
    }
  };
  if constexpr (DMA) {
    double *const xs = lds;            // exchange (re / im halves)
    double *const stg = lds + G::SLOTS;  // the pair's samples, by LDS-DMA
    cd *const twl = reinterpret_cast<cd *>(lds + G::SLOTS + STG);
    for (int i = tl; i < TWN; i += G::T1) twl[i] = tw[i];
    const int64_t pend = p0 + pairs_per_worker < npairs ? p0 + pairs_per_worker : npairs;
    // pair pp's samples [s stride, s stride + U) into stg: 1 KiB per wave-
    // instruction (16 B per lane) from the full waves; the descriptor ends at
    // U, so the last piece's tail reads zeros (the offset is in the
    // range-checked voffset; soffset is not range-checked)
    auto dma = [&](int64_t pp) {
      const int64_t s = seg_begin + 2 * pp;
      const int U = (int)(s + 1 < seg_end ? stride + nfft : nfft);
      const rsrc_t r = make_rsrc(x + s * stride, (int64_t)U * 8);
      constexpr int FW = G::T1 / 64;
      const int wv = __builtin_amdgcn_readfirstlane(tl >> 6);
      const uint32_t lane16 = (uint32_t)(tl & 63) * 16u;
      const int pieces = (U * 8 + 1023) / 1024;
      if (wv < FW) {
        for (int piece = wv; piece < pieces; piece += FW)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              r, (__attribute__((address_space(3))) void *)(stg + piece * 128), 16,
              (uint32_t)piece * 1024u + lane16, 0, 0, 0);
      }
    };
    if (p0 < pend) dma(p0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int64_t p = p0; p < pend; ++p) {
      const int64_t s0 = seg_begin + 2 * p;
      const bool has1 = s0 + 1 < seg_end;
      const double *w = opaque_ptr(win);
      const int tt = opaque_int(tl);
      First f0;
      first_from(f0, stg, w, tt, p < nfull && nopad, true, has1);
      f0.compute(tt, true, twl);
      // pinned before the DMA is issued: a first-pass value computed after it
      // would make its window load's wait (vmcnt is in order) wait for the DMA
#pragma unroll
      for (int jj = 0; jj < First::J; ++jj)
#pragma unroll
        for (int r = 0; r < R0; ++r) asm volatile("" : "+v"(f0.v[jj][r].x), "+v"(f0.v[jj][r].y));
      chain_sync<true>();  // every thread has read the stage
      if (p + 1 < pend) dma(p + 1);
      auto sink = [&](const typename L::Pass &c) { accumulate(c, tt); };
      fixed_chain_sink<true, true, SWZ, G::N, G::T1, R0, 0, First, decltype(sink), RS...>(
          f0, tt, true, xs, twl, sink);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces landed
      chain_sync<true>();  // every wave's, and the last exchange's reads are done
    }
  } else {
    for (int64_t it = 0; it < pairs_per_worker; ++it) {
      const int64_t p = p0 + it;
      const bool active = p < npairs;
      const int64_t s0 = seg_begin + 2 * (active ? p : 0);
      const bool has1 = active && s0 + 1 < seg_end;
      const double *x0 = opaque_ptr(x) + s0 * stride;
      // laundered per pair: otherwise the compiler hoists the loop-invariant
      // window values and twiddle power chains out of the loop, and the
      // registers they pin halve the occupancy
      const double *w = opaque_ptr(win);
      const cd *twp = opaque_ptr(tw);
      const int tt = opaque_int(tl);
      First f0;
      if constexpr (!SPL) {
        // Loads are unconditional: a full pair without padding (every pair
        // but the signal's last, whenever Pad = NFFT; wave-uniform with one
        // worker per workgroup) takes its samples as they are; otherwise the
        // index is clamped and the mask applied where the samples are used. A
        // load inside a per-lane branch is waited for inside it, one
        // s_waitcnt per element: per 2^28 samples 480 / 240 1.82 -> 1.11 ms,
        // 1000 / 500 1.37 -> 1.10, 1536 / 768 1.40 -> 0.99.
        const double *x1 = has1 ? x0 + stride : x0;  // (a missing partner: loaded, not used)
        if (p < nfull && nopad) {
#pragma unroll
          for (int jj = 0; jj < First::J; ++jj) {
            const int j = tt + jj * G::T1;
            if (First::act(j, true)) {
#pragma unroll
              for (int r = 0; r < R0; ++r) {
                const int i = j + r * First::NB;
                const double wi = w[i];
                f0.v[jj][r] = {wi * x0[i], wi * x1[i]};
              }
            }
          }
        } else {
#pragma unroll
          for (int jj = 0; jj < First::J; ++jj) {
            const int j = tt + jj * G::T1;
            if (First::act(j, true)) {
#pragma unroll
              for (int r = 0; r < R0; ++r) {
                const int i = j + r * First::NB;
                const bool in = i < nfft;
                const int ic = in ? i : (int)nfft - 1;
                const double wi = w[ic], a = x0[ic], b = x1[ic];
                f0.v[jj][r] = {active && in ? wi * a : 0.0, has1 && in ? wi * b : 0.0};
              }
            }
          }
        }
      } else {
        // re/im exchange halves (N > 4096): the buffer holds only N doubles, so
        // the first pass loads its own elements (in a per-lane branch: 6000 /
        // 3000 measured 2.80 ms per 2^28 samples that way against 3.10 with
        // unconditional clamped loads)
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
                if (has1) b = wi * x0[stride + i];
              }
              f0.v[jj][r] = {a, b};
            }
          }
        }
      }
      f0.compute(tt, true, twp);
      if (it > 0) __syncthreads();  // the previous pair's last exchange reads are done
      auto sink = [&](const typename L::Pass &c) {
        if (active) accumulate(c, tt);
      };
      fixed_chain_to<SPL, SWZ, G::N, G::T1, R0, 0, First, decltype(sink), RS...>(f0, tt, true, ld,
                                                                                twp, sink);
    }
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

// ---------------------------------------------------------------------------
// Column pass of the mixed four-step for n = L * C (x as L rows x C columns)
// with a smooth L that has a radix list (26 <= L <= 1016; L <= 25 is
// colradix_kernel, a power of 2 colfft_tile_kernel). A workgroup takes W
// adjacent columns; thread (t, c) = threadIdx.x / W, % W works on column c,
// so every wave-instruction of the first pass's loads and the last pass's
// stores covers 64 / W row segments of W * 16 B, all of a thread's loads in
// flight at once. The exchanges between passes go through LDS per column
// (column stride SL odd, so the 16-B lanes of a row land on distinct banks).
// Column c's DFT_L[k] is written times W_n^(c*k) (two table reads and a
// recurrence per butterfly) in place of the rows; the rows DFT_C and the transpose follow
// (exec_mixed4). Compiled at plan creation with hipRTC (mixed_jit.hip).
template <int W, bool SPLIT, bool CONJ_IN, bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((W * FixedGeo<R0, RS...>::T1)) void colfixed_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t C, int64_t n,
    const cd *__restrict__ tw, const cd *__restrict__ twn) {
  using G = FixedGeo<R0, RS...>;
  using First = FPass<R0, G::N, 1, G::T1>;
  using Last = typename FixedLast<R0, RS...>::Pass;
  constexpr int SL = G::SLOTS + 1;  // per column, in complex (or, with SPLIT, double) slots
  __shared__ double lds[W * SL * (SPLIT ? 1 : 2)];
  const int tid = (int)threadIdx.x, c = tid % W, tl = tid / W;
  const int64_t col = (int64_t)blockIdx.x * W + c;
  const bool valid = col < C;
  const cd *src = in + (int64_t)blockIdx.y * n + col;
  cd *dst = out + (int64_t)blockIdx.y * n + col;
  double *ld = lds + c * SL * (SPLIT ? 1 : 2);
  First p0;
#pragma unroll
  for (int jj = 0; jj < First::J; ++jj) {
    const int j = tl + jj * G::T1;
    if (First::act(j, valid)) {
#pragma unroll
      for (int r = 0; r < R0; ++r) {
        cd v = ld_nt(src + (int64_t)(j + r * First::NB) * C);
        if constexpr (CONJ_IN) v.y = -v.y;
        p0.v[jj][r] = v;
      }
    }
  }
  p0.compute(tl, valid, tw);
  auto sink = [&](const Last &q) {
#pragma unroll
    for (int jj = 0; jj < Last::J; ++jj) {
      const int j = tl + jj * G::T1;
      if (Last::act(j, valid)) {
        constexpr int RL = FixedLast<R0, RS...>::R, NSL = G::N / RL;  // as FPass::store_hbm
        const int k0 = j % NSL, o = (j - k0) * RL + k0;
        // W_n^(col*k) for k = o + r*NSL: two table reads and a recurrence
        // (one read per element would scatter over an n-entry table that
        // does not stay in L2 at n ~ 10^6)
        cd w = twn[col * o];
        const cd ws = twn[col * NSL];
#pragma unroll
        for (int r = 0; r < RL; ++r) {
          const int64_t k = o + r * NSL;
          st_nt(dst + k * C, cmul(q.v[jj][r], w));
          if (r + 1 < RL) w = cmul(w, ws);
        }
      }
    }
  };
  fixed_chain_to<SPLIT, SWZ, G::N, G::T1, R0, 0, First, decltype(sink), RS...>(p0, tl, valid, ld,
                                                                               tw, sink);
}

// ---------------------------------------------------------------------------
// Rader's algorithm for a prime length P = N + 1 whose N = prod(R0, RS...) is
// smooth (the reference sends every non-power-of-2 length to Bluestein,
// fft/bluestein.go:68-94: three FFTs of NextPowerOf2(2P - 1), ~4 P points
// each). With g a primitive root mod P, gpow[q] = g^q and ginv[r] = g^-r:
//   X[0]       = y[0] + sum_q a[q],            a[q] = y[gpow[q]],
//   X[ginv[r]] = y[0] + (a (*) b)[r],          b[q] = W_P^ginv[q],
// a cyclic convolution of length N, done as FFT_N(a) * bhat (bhat = FFT_N(b)
// / N, built on the device at plan creation) and an inverse FFT_N by the
// conjugation identity. The same DFT with two N-point FFTs instead of three
// 2^ceil(log2(2P - 1))-point ones. One workgroup slot per row:
//  1. the row's P samples (coalesced, nontemporal) into LDS in natural order;
//  2. the first pass gathers a[q] = LDS[gpow[q]] and FFT_N runs as the
//     mixed-radix chain (fixed_chain_to);
//  3. A[k] * bhat[k] in the last pass's registers; the thread holding k = 0
//     keeps A[0] (X[0] = y[0] + A[0]) and adds y[0] to C[0], which adds y[0]
//     to every output of the inverse transform; conjugated for it;
//  4. LDS exchange into natural order, FFT_N again, conjugated back;
//  5. c[r] scattered to LDS slot ginv[r] (X[0] from the k = 0 thread), then a
//     coalesced nontemporal store of the row.
// The row never leaves the chip between its load and its store: 16 B read +
// 16 B written per sample, as any one-kernel transform. SPLIT (N > 4096):
// every LDS round trip goes as real then imaginary halves. In place is safe:
// a slot reads its whole row before the first barrier and stores it after
// the last. INV: IDFT = conj(DFT(conj(x))) * scale; LOAD_REAL: float64 rows.
template <int R0, int... RS>
struct RaderGeo {
  using G = FixedGeo<R0, RS...>;
  static constexpr int N = G::N, P = N + 1, T1 = G::T1;
  static constexpr bool SPLIT = N > 4096;
  static constexpr int SLOTS = (P + 7) & ~7;  // staging slots (>= the FFT exchange's)
  static constexpr int DPT = SPLIT ? SLOTS : 2 * SLOTS;  // doubles of LDS per transform
  static constexpr int NQ = (P + T1 - 1) / T1;           // row elements per thread
  static constexpr int tpw() {
    int t = 256 / T1 > 1 ? 256 / T1 : 1;
    while (t > 1 && t * DPT * 8 > 65536) --t;
    return t;
  }
  static constexpr int TPW = tpw();
  static constexpr int WG = TPW * T1;
};

template <bool INV, int LOAD, bool SWZ, int R0, int... RS>
__global__ __launch_bounds__((RaderGeo<R0, RS...>::WG)) void rader_fixed_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t batch, const cd *__restrict__ tw,
    const cd *__restrict__ bhat, const int *__restrict__ gpow, const int *__restrict__ ginv,
    double scale) {
  using RG = RaderGeo<R0, RS...>;
  constexpr int N = RG::N, P = RG::P, T1 = RG::T1, NQ = RG::NQ;
  constexpr bool SPLIT = RG::SPLIT;
  using First = FPass<R0, N, 1, T1>;
  using FL = FixedLast<R0, RS...>;
  using Last = typename FL::Pass;
  constexpr int RL = FL::R, NSL = N / RL;
  __shared__ double lds[RG::TPW * RG::DPT];
  const int sub = RG::TPW == 1 ? 0 : (int)threadIdx.x / T1;
  const int tl = (int)threadIdx.x - sub * T1;
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x) * RG::TPW + sub;
  const bool valid = row < batch;
  const int64_t lrow = valid ? row : batch - 1;  // a slot past the batch reads a valid row
  double *ld = lds + sub * RG::DPT;
  cd *lc = reinterpret_cast<cd *>(ld);
  // 1. the row, natural order. TPW > 1 (short rows: few threads per
  // transform) loads the workgroup's TPW contiguous rows as one chunk, every
  // thread a lane of one coalesced stream (threads-per-row loads would touch
  // 64 / T1 rows per wave-instruction; at P = 17, T1 = 1, a lane per row).
  constexpr int CH = RG::TPW * P, NC = (CH + RG::WG - 1) / RG::WG;
  const int64_t c0 = xcd_remap(blockIdx.x, gridDim.x) * (int64_t)CH, cend = batch * P;
  auto chunk_slot = [&](int e) -> cd * {  // chunk element e -> its row's staging slot
    const int s2 = e / P;
    return reinterpret_cast<cd *>(lds + s2 * RG::DPT) + (e - s2 * P);
  };
  cd xr[RG::TPW > 1 ? 1 : NQ];
  if constexpr (RG::TPW > 1) {
    static_assert(!SPLIT, "several rows per workgroup only with complex staging");
    cd xc[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int e = (int)threadIdx.x + q * RG::WG;
      xc[q] = {0.0, 0.0};
      if ((q + 1) * RG::WG <= CH || e < CH) {
        if (c0 + e < cend) {
          if constexpr (LOAD == LOAD_REAL) {
            xc[q] = {ld_nt(reinterpret_cast<const double *>(in) + c0 + e), 0.0};
          } else {
            xc[q] = ld_nt(reinterpret_cast<const cd *>(in) + c0 + e);
            if constexpr (INV) xc[q].y = -xc[q].y;
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int e = (int)threadIdx.x + q * RG::WG;
      if ((q + 1) * RG::WG <= CH || e < CH) *chunk_slot(e) = xc[q];
    }
  } else {
    // (An L2 touch-ahead of the row the block 16 places later on this XCD
    // will load, as the chirp-z kernel does, made 65 536 x 3001 slower: 1.74-
    // 1.76 against 1.68-1.69 ms, profiles/r05/rader_pf_ab.txt.)
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = tl + q * T1;
      if (q * T1 + T1 <= P || i < P) {
        if constexpr (LOAD == LOAD_REAL) {
          xr[q] = {ld_nt(reinterpret_cast<const double *>(in) + lrow * P + i), 0.0};
        } else {
          xr[q] = ld_nt(reinterpret_cast<const cd *>(in) + lrow * P + i);
          if constexpr (INV) xr[q].y = -xr[q].y;
        }
      }
    }
  }
  // 2. gather a[q] = y[gpow[q]] into the first pass's registers
  First p0;
  int gi[First::J][R0];
#pragma unroll
  for (int jj = 0; jj < First::J; ++jj) {
    const int j = tl + jj * T1;
#pragma unroll
    for (int r = 0; r < R0; ++r) gi[jj][r] = First::act(j, true) ? gpow[j + r * First::NB] : 0;
  }
  cd y0;  // element 0 of the row (X[0] = y0 + A[0]; y0 is added to every other output)
  if constexpr (SPLIT) {
    y0 = xr[0];  // (meaningful in the thread with tl = 0)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h) __syncthreads();  // the real parts' gathers are done
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int i = tl + q * T1;
        if (q * T1 + T1 <= P || i < P) ld[i] = h ? xr[q].y : xr[q].x;
      }
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < First::J; ++jj) {
        const int j = tl + jj * T1;
        if (First::act(j, true)) {
#pragma unroll
          for (int r = 0; r < R0; ++r) {
            if (h) p0.v[jj][r].y = ld[gi[jj][r]];
            else p0.v[jj][r].x = ld[gi[jj][r]];
          }
        }
      }
    }
  } else {
    if constexpr (RG::TPW == 1) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int i = tl + q * T1;
        if (q * T1 + T1 <= P || i < P) lc[i] = xr[q];
      }
    }
    __syncthreads();
    y0 = lc[0];
#pragma unroll
    for (int jj = 0; jj < First::J; ++jj) {
      const int j = tl + jj * T1;
      if (First::act(j, true)) {
#pragma unroll
        for (int r = 0; r < R0; ++r) p0.v[jj][r] = lc[gi[jj][r]];
      }
    }
  }
  // FFT_N(a)
  p0.compute(tl, true, tw);
  Last keep;
  if constexpr (sizeof...(RS) == 0) {
    keep = p0;
  } else {
    __syncthreads();  // every gather is done before the first exchange writes
    auto sink = [&](const Last &c) { keep = c; };
    fixed_chain_to<SPLIT, SWZ, N, T1, R0, 0, First, decltype(sink), RS...>(p0, tl, true, ld, tw,
                                                                          sink);
  }
  // 3. C = A * bhat (+ y0 at k = 0), conjugated for the inverse transform
  cd a0 = {0.0, 0.0};
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = tl + jj * T1;
    if (Last::act(j, true)) {
      const int k0 = j % NSL, o = (j - k0) * RL + k0;
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        const int k = o + r * NSL;
        const cd A = keep.v[jj][r];
        cd c = cmul(A, bhat[k]);
        if (k == 0) {
          a0 = A;
          c = c + y0;
        }
        keep.v[jj][r] = conjg(c);
      }
    }
  }
  // 4. natural order for the second FFT's first pass, FFT_N, conjugated back
  const int t2 = opaque_int(tl);
  const cd *tw2 = opaque_ptr(tw);
  First p1;
  __syncthreads();  // the last exchange's reads (or the gathers) are done
  if constexpr (SPLIT) {
    keep.template store_lds<0, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<0, SWZ>(t2, true, ld);
    __syncthreads();
    keep.template store_lds<1, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<1, SWZ>(t2, true, ld);
  } else {
    keep.template store_lds<2, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<2, SWZ>(t2, true, ld);
  }
  p1.compute(t2, true, tw2);
  Last fin;
  if constexpr (sizeof...(RS) == 0) {
    fin = p1;
  } else {
    __syncthreads();
    auto sink = [&](const Last &c) { fin = c; };
    fixed_chain_to<SPLIT, SWZ, N, T1, R0, 0, First, decltype(sink), RS...>(p1, t2, true, ld, tw2,
                                                                          sink);
  }
  // 5. X[ginv[r]] = conj(fin[r]); X[0] = y0 + A[0]; then the row's store
  int oi[Last::J][RL];
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = t2 + jj * T1;
    const int k0 = j % NSL, o = (j - k0) * RL + k0;
#pragma unroll
    for (int r = 0; r < RL; ++r) oi[jj][r] = Last::act(j, true) ? ginv[o + r * NSL] : 0;
  }
  const cd x0 = y0 + a0;
  cd *dst = out + lrow * P;
  cd res[RG::TPW > 1 ? NC : NQ];
#pragma unroll
  for (int h = 0; h < (SPLIT ? 2 : 1); ++h) {
    __syncthreads();  // the previous LDS reads are done
#pragma unroll
    for (int jj = 0; jj < Last::J; ++jj) {
      const int j = t2 + jj * T1;
      if (Last::act(j, true)) {
#pragma unroll
        for (int r = 0; r < RL; ++r) {
          const cd c = conjg(fin.v[jj][r]);
          if constexpr (SPLIT) ld[oi[jj][r]] = h ? c.y : c.x;
          else lc[oi[jj][r]] = c;
        }
      }
    }
    if (t2 == 0) {
      if constexpr (SPLIT) ld[0] = h ? x0.y : x0.x;
      else lc[0] = x0;
    }
    __syncthreads();
    if constexpr (RG::TPW > 1) {
#pragma unroll
      for (int q = 0; q < NC; ++q) {
        const int e = (int)threadIdx.x + q * RG::WG;
        if ((q + 1) * RG::WG <= CH || e < CH) res[q] = *chunk_slot(e);
      }
    } else {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int i = t2 + q * T1;
        if (q * T1 + T1 <= P || i < P) {
          if constexpr (SPLIT) {
            if (h) res[q].y = ld[i];
            else res[q].x = ld[i];
          } else {
            res[q] = lc[i];
          }
        }
      }
    }
  }
  if constexpr (RG::TPW > 1) {
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int e = (int)threadIdx.x + q * RG::WG;
      if (((q + 1) * RG::WG <= CH || e < CH) && c0 + e < cend) {
        cd y = res[q];
        if constexpr (INV) y = {y.x * scale, -y.y * scale};
        st_nt(out + c0 + e, y);
      }
    }
  } else if (valid) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = t2 + q * T1;
      if (q * T1 + T1 <= P || i < P) {
        cd y = res[q];
        if constexpr (INV) y = {y.x * scale, -y.y * scale};
        st_nt(dst + i, y);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// A composite n = M * P with a prime factor P > 31 whose P - 1 has a radix
// list, and gcd(M, P) = 1 (the reference sends it to Bluestein like every
// non-power-of-2 length, fft/fft.go:82-86 -> fft/bluestein.go:68-94: three
// FFTs of NextPowerOf2(2n - 1) points). Good-Thomas (prime-factor) index maps
// make the DFT an M x P two-dimensional one without twiddles:
//   X[(k1 E1 + k2 E2) mod n] = sum_i2 W_P^(i2 k2) sum_i1 W_M^(i1 k1)
//                              x[(i1 P + i2 M) mod n],
// E1 = P (P^-1 mod M) (= 1 mod M, 0 mod P), E2 = M (M^-1 mod P). The DFT_M
// along i1 runs in registers (one column per thread); the M DFT_P along i2
// run as Rader's cyclic convolutions of length N = P - 1 on the inlined
// mixed-radix chain, side by side in one workgroup (rader_fixed_kernel for M
// sub-transforms). One HBM read and one write per sample, as any one-kernel
// transform:
//  1. the workgroup's TPW rows (contiguous) into LDS, coalesced, natural order;
//  2. column q of row s (q < N: i2 = gpow[q]; q = N: i2 = 0) gathers its M
//     samples x[(i1 P + i2 M) mod n], DFT_M; output k1 goes to slot q of
//     sub-transform k1 — Rader's a[q] = y[gpow[q]] in natural order — or, for
//     q = N, to the sub-transform's y0;
//  3. each sub-transform: FFT_N, x bhat (+ y0 at k = 0), conj, FFT_N, conj
//     (rader_fixed_kernel steps 2-4, the same tables as the prime P's plan);
//  4. output r of sub-transform k1 is X_P[k2 = ginv[r]]: scattered to LDS slot
//     (k1 E1 + k2 E2) mod n (k2 = 0: y0 + A[0]), then a coalesced store.
// The LDS a row uses for its samples, its M sub-transforms' exchanges and
// its output staging is one region, separated by barriers.
// (pfa_gcd, pfa_inv, dft_m: mixed_core.hpp)
template <int M, int R0, int... RS>
struct PfaGeo {
  using G = FixedGeo<R0, RS...>;
  static constexpr int N = G::N, P = N + 1, T1 = G::T1, NN = M * P;
  static constexpr int SUBS = G::SLOTS;                      // a sub-transform's slots
  static constexpr int RSL = M * SUBS > NN ? M * SUBS : NN;  // complex slots per row
  static constexpr int RT = M * T1;                          // threads per row
  // rows per workgroup: about 256 threads within 40 KiB of row slots, so
  // that four workgroups share a CU's LDS where the registers allow it (at
  // 64 KiB, rows of 74 = 2 x 37 ran two 252-thread workgroups per CU)
  static constexpr int tpw() {
    int t = 256 / RT > 1 ? 256 / RT : 1;
    while (t > 1 && t * (RSL + M) * 16 > 40960) --t;
    return t;
  }
  static constexpr int TPW = tpw();
  static constexpr int WG = TPW * RT;
  static constexpr int NCOL = TPW * P, CA = (NCOL + WG - 1) / WG;  // stage-A columns
  static constexpr int CH = TPW * NN, NC = (CH + WG - 1) / WG;     // row elements per thread
  static constexpr int E1 = P * pfa_inv(P % M, M) % NN, E2 = M * pfa_inv(M % P, P) % NN;
};

template <bool INV, int LOAD, bool SWZ, int M, int R0, int... RS>
__global__ __launch_bounds__((PfaGeo<M, R0, RS...>::WG)) void rader_pfa_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t batch, const cd *__restrict__ tw,
    const cd *__restrict__ bhat, const int *__restrict__ gpow, const int *__restrict__ ginv,
    double scale) {
  using PG = PfaGeo<M, R0, RS...>;
  constexpr int N = PG::N, P = PG::P, T1 = PG::T1, NN = PG::NN, WG = PG::WG;
  constexpr int RSL = PG::RSL, SUBS = PG::SUBS, CH = PG::CH, NC = PG::NC;
  static_assert(N <= 4096, "the sub-transforms exchange as complex128 (N <= 4096)");
  using First = FPass<R0, N, 1, T1>;
  using FL = FixedLast<R0, RS...>;
  using Last = typename FL::Pass;
  constexpr int RL = FL::R, NSL = N / RL;
  __shared__ double lds[2 * PG::TPW * RSL + 2 * PG::TPW * M];
  cd *const xs = reinterpret_cast<cd *>(lds);                       // rows (RSL slots each)
  cd *const dcs = reinterpret_cast<cd *>(lds + 2 * PG::TPW * RSL);  // y0 of each sub-transform
  const int tid = (int)threadIdx.x;
  const int rs = PG::TPW == 1 ? 0 : tid / PG::RT;  // row slot of this thread's sub-transform
  const int tr = tid - rs * PG::RT;
  const int k1 = tr / T1, tl = tr - k1 * T1;
  const int64_t c0 = xcd_remap(blockIdx.x, gridDim.x) * (int64_t)CH, cend = batch * NN;
  auto slot = [&](int e) -> cd * {  // workgroup chunk element e -> its row's LDS slot
    const int s = e / NN;
    return xs + s * RSL + (e - s * NN);
  };
  // the stage-A columns' i2 = gpow[q] (q = P - 1: 0), read before the rows
  // so that the table's latency hides behind the row loads
  int i2a[PG::CA];
#pragma unroll
  for (int a = 0; a < PG::CA; ++a) {
    const int c = tid + a * WG;
    i2a[a] = 0;
    if ((a + 1) * WG <= PG::NCOL || c < PG::NCOL) {
      const int q = c - (c / P) * P;
      if (q < N) i2a[a] = gpow[q];
    }
  }
  // 1. the rows, natural order
  {
    cd xc[NC];
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int e = tid + q * WG;
      xc[q] = {0.0, 0.0};
      if (((q + 1) * WG <= CH || e < CH) && c0 + e < cend) {
        if constexpr (LOAD == LOAD_REAL) {
          xc[q] = {ld_nt(reinterpret_cast<const double *>(in) + c0 + e), 0.0};
        } else {
          xc[q] = ld_nt(reinterpret_cast<const cd *>(in) + c0 + e);
          if constexpr (INV) xc[q].y = -xc[q].y;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int e = tid + q * WG;
      if ((q + 1) * WG <= CH || e < CH) *slot(e) = xc[q];
    }
  }
  __syncthreads();
  // 2. DFT_M down each column, into the sub-transforms' Rader order
  {
    cd ya[PG::CA][M];
    int qa[PG::CA];
#pragma unroll
    for (int a = 0; a < PG::CA; ++a) {
      const int c = tid + a * WG;
      qa[a] = -1;
      if ((a + 1) * WG <= PG::NCOL || c < PG::NCOL) {
        const int s = c / P;
        const cd *row = xs + s * RSL;
        int idx = M * i2a[a];  // (i1 P + i2 M) mod n for i1 = 0, 1, ...
#pragma unroll
        for (int i1 = 0; i1 < M; ++i1) {
          ya[a][i1] = row[idx];
          idx += P;
          if (idx >= NN) idx -= NN;
        }
        dft_m<M>(ya[a]);
        qa[a] = c;
      }
    }
    __syncthreads();  // every gather of the rows is done
#pragma unroll
    for (int a = 0; a < PG::CA; ++a) {
      if (qa[a] >= 0) {
        const int s = qa[a] / P, q = qa[a] - s * P;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          if (q < N) xs[s * RSL + k * SUBS + q] = ya[a][k];
          else dcs[s * M + k] = ya[a][k];
        }
      }
    }
  }
  __syncthreads();
  // 3. sub-transform k1 of row rs: Rader's convolution (rader_fixed_kernel)
  cd *const lc = xs + rs * RSL + k1 * SUBS;
  const cd y0 = dcs[rs * M + k1];
  First p0;
#pragma unroll
  for (int jj = 0; jj < First::J; ++jj) {
    const int j = tl + jj * T1;
    if (First::act(j, true)) {
#pragma unroll
      for (int r = 0; r < R0; ++r) p0.v[jj][r] = lc[j + r * First::NB];
    }
  }
  p0.compute(tl, true, tw);
  Last keep;
  if constexpr (sizeof...(RS) == 0) {
    keep = p0;
  } else {
    __syncthreads();  // every first-pass load is done before the first exchange writes
    auto sink = [&](const Last &c) { keep = c; };
    fixed_chain_to<false, SWZ, N, T1, R0, 0, First, decltype(sink), RS...>(p0, tl, true, lc, tw,
                                                                           sink);
  }
  cd a0 = {0.0, 0.0};
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = tl + jj * T1;
    if (Last::act(j, true)) {
      const int kb = j % NSL, o = (j - kb) * RL + kb;
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        const int k = o + r * NSL;
        const cd A = keep.v[jj][r];
        cd c = cmul(A, bhat[k]);
        if (k == 0) {
          a0 = A;
          c = c + y0;
        }
        keep.v[jj][r] = conjg(c);
      }
    }
  }
  const int t2 = opaque_int(tl);
  const cd *tw2 = opaque_ptr(tw);
  First p1;
  __syncthreads();  // the last exchange's reads (or the first-pass loads) are done
  keep.template store_lds<2, SWZ>(t2, true, lc);
  __syncthreads();
  p1.template load_lds<2, SWZ>(t2, true, lc);
  p1.compute(t2, true, tw2);
  Last fin;
  if constexpr (sizeof...(RS) == 0) {
    fin = p1;
  } else {
    __syncthreads();
    auto sink = [&](const Last &c) { fin = c; };
    fixed_chain_to<false, SWZ, N, T1, R0, 0, First, decltype(sink), RS...>(p1, t2, true, lc, tw2,
                                                                           sink);
  }
  // 4. X[(k1 E1 + k2 E2) mod n], k2 = ginv[r]; k2 = 0: y0 + A[0]
  int oi[Last::J][RL];
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = t2 + jj * T1;
    const int kb = j % NSL, o = (j - kb) * RL + kb;
#pragma unroll
    for (int r = 0; r < RL; ++r) oi[jj][r] = Last::act(j, true) ? ginv[o + r * NSL] : 0;
  }
  cd *const ro = xs + rs * RSL;
  const int kb1 = k1 * PG::E1 % NN;
  __syncthreads();  // every sub-transform's LDS reads are done (the regions overlap)
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = t2 + jj * T1;
    if (Last::act(j, true)) {
#pragma unroll
      for (int r = 0; r < RL; ++r) {
        int idx = kb1 + oi[jj][r] * PG::E2 % NN;
        if (idx >= NN) idx -= NN;
        ro[idx] = conjg(fin.v[jj][r]);
      }
    }
  }
  if (t2 == 0) ro[kb1] = y0 + a0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NC; ++q) {
    const int e = tid + q * WG;
    if (((q + 1) * WG <= CH || e < CH) && c0 + e < cend) {
      cd y = *slot(e);
      if constexpr (INV) y = {y.x * scale, -y.y * scale};
      st_nt(out + c0 + e, y);
    }
  }
}

// ---------------------------------------------------------------------------
// Chirp-z (Bluestein, fft/bluestein.go:68-94) with the convolution on a
// smooth length L = prod(R0, RS...) >= 2n - 1 instead of NextPowerOf2(2n - 1)
// (bluestein.go:70): the same linear convolution, hence the same DFT, on up
// to half the points where n sits just above a power of 2 (n = 4099: L =
// 8232 against 16384). The inlined mixed-radix chain (fixed_chain_to) twice,
// one transform per workgroup slot:
//  1. the first pass loads a[i] = x[i] conj(w_i) (i < n; zero for n <= i < L)
//     straight from HBM (element j + r L / R0 of the slot's row: each wave-
//     instruction a contiguous run) — chirp = conj(w), a table every slot
//     re-reads from L2;
//  2. FFT_L, then C = conj(A bhat) in the last pass's registers (bhat =
//     FFT_L(b) / L, built at plan creation with the engine itself);
//  3. an LDS exchange into natural order, FFT_L again;
//  4. X[k] = conj(C'[k]) chirp[k] for k < n from the last pass's registers
//     (the outputs k >= n are not stored). INV: conj in, conj and 1/n out.
// SPLIT (L > 4096): the exchanges as real then imaginary halves.
template <bool INV, int LOAD, bool SPLIT, bool SWZ, int NLEN, int R0, int... RS>
__global__ __launch_bounds__((FixedGeo<R0, RS...>::WG)) void bluestein_fixed_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t batch, const cd *__restrict__ tw,
    const cd *__restrict__ chirp, const cd *__restrict__ bhat, double scale) {
  using G = FixedGeo<R0, RS...>;
  constexpr int L = G::N, T1 = G::T1;
  static_assert(2 * NLEN - 1 <= L, "the convolution must hold 2n - 1 points");
  using First = FPass<R0, L, 1, T1>;
  using FL = FixedLast<R0, RS...>;
  using Last = typename FL::Pass;
  constexpr int RL = FL::R, NSL = L / RL;
  __shared__ double lds[G::TPW * (SPLIT ? G::SLOTS : 2 * G::SLOTS)];
  const int sub = G::TPW == 1 ? 0 : (int)threadIdx.x / T1;
  const int tl = (int)threadIdx.x - sub * T1;
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x) * G::TPW + sub;
  const bool valid = row < batch;
  const int64_t lrow = valid ? row : batch - 1;  // a slot past the batch reads a valid row
  double *ld = lds + sub * (SPLIT ? G::SLOTS : 2 * G::SLOTS);
  // 1. a = x conj(w), zero-padded to L, into the first pass
  First p0;
#pragma unroll
  for (int jj = 0; jj < First::J; ++jj) {
    const int j = tl + jj * T1;
    if (First::act(j, true)) {
#pragma unroll
      for (int r = 0; r < R0; ++r) {
        const int i = j + r * First::NB;
        cd a = {0.0, 0.0};
        if (r * First::NB < NLEN && i < NLEN) {
          cd x;
          if constexpr (LOAD == LOAD_REAL) {
            x = {ld_nt(reinterpret_cast<const double *>(in) + lrow * NLEN + i), 0.0};
          } else {
            x = ld_nt(reinterpret_cast<const cd *>(in) + lrow * NLEN + i);
            if constexpr (INV) x.y = -x.y;
          }
          a = cmul(x, chirp[i]);
        }
        p0.v[jj][r] = a;
      }
    }
  }
  p0.compute(tl, true, tw);
  Last keep;
  if constexpr (sizeof...(RS) == 0) {
    keep = p0;
  } else {
    auto sink = [&](const Last &c) { keep = c; };
    fixed_chain_to<SPLIT, SWZ, L, T1, R0, 0, First, decltype(sink), RS...>(p0, tl, true, ld, tw,
                                                                          sink);
  }
  // 2. C = conj(A bhat)
#pragma unroll
  for (int jj = 0; jj < Last::J; ++jj) {
    const int j = tl + jj * T1;
    if (Last::act(j, true)) {
      const int kb = j % NSL, o = (j - kb) * RL + kb;
#pragma unroll
      for (int r = 0; r < RL; ++r) keep.v[jj][r] = conjg(cmul(keep.v[jj][r], bhat[o + r * NSL]));
    }
  }
  // 3. natural order, FFT_L
  const int t2 = opaque_int(tl);
  const cd *tw2 = opaque_ptr(tw);
  First p1;
  __syncthreads();  // the last exchange's reads are done
  if constexpr (SPLIT) {
    keep.template store_lds<0, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<0, SWZ>(t2, true, ld);
    __syncthreads();
    keep.template store_lds<1, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<1, SWZ>(t2, true, ld);
  } else {
    keep.template store_lds<2, SWZ>(t2, true, ld);
    __syncthreads();
    p1.template load_lds<2, SWZ>(t2, true, ld);
  }
  p1.compute(t2, true, tw2);
  Last fin;
  if constexpr (sizeof...(RS) == 0) {
    fin = p1;
  } else {
    __syncthreads();
    auto sink = [&](const Last &c) { fin = c; };
    fixed_chain_to<SPLIT, SWZ, L, T1, R0, 0, First, decltype(sink), RS...>(p1, t2, true, ld, tw2,
                                                                          sink);
  }
  // 4. X[k] = conj(fin[k]) chirp[k], k < n
  if (valid) {
    const cd *ch = opaque_ptr(chirp);
    cd *dst = out + row * NLEN;
#pragma unroll
    for (int jj = 0; jj < Last::J; ++jj) {
      const int j = t2 + jj * T1;
      if (Last::act(j, true)) {
        const int kb = j % NSL, o = (j - kb) * RL + kb;
#pragma unroll
        for (int r = 0; r < RL; ++r) {
          const int k = o + r * NSL;
          if (r * NSL < NLEN && k < NLEN) {
            cd y = cmul(conjg(fin.v[jj][r]), ch[k]);
            if constexpr (INV) y = {y.x * scale, -y.y * scale};
            st_nt(dst + k, y);
          }
        }
      }
    }
  }
}

#ifndef __HIPCC_RTC__
// Workers per workgroup of the fused Pwelch on d's list, 0 where d is not
// this list or where a pair's samples (span = stride + nfft doubles) exceed
// the LDS-DMA stage of a PwfDma list (a negative Noverlap makes stride >
// nfft; spectral/spectral.go:22-43 allows it): the caller then takes another
// path instead of a DMA that would overrun the stage into the twiddle table.
template <int... RS>
static int spec_pw_tpw(Spec<RS...>, const MixedDesc &d, int64_t span) {
  uint64_t codes = 0;
  int q = 0;
  for (int r : {RS...}) codes |= (uint64_t)r << (5 * q++);
  if (d.n != FixedGeo<RS...>::N || d.codes != codes) return 0;
  if (PwfDma<RS...>::on && span > PwfDma<RS...>::STG) return 0;
  return FixedGeo<RS...>::TPW;
}
template <class... S>
static int find_pw_tpw(std::tuple<S...>, const MixedDesc &d, int64_t span) {
  int t = 0;
  ((t = t ? t : spec_pw_tpw(S{}, d, span)), ...);
  return t;
}

template <int... RS>
static bool spec_pw_launch(Spec<RS...>, const MixedDesc &d, const double *x, int64_t nfft,
                           int64_t stride, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                           int64_t nworkers, const double *win, const cd *tw, double *partial,
                           hipStream_t s) {
  if (!spec_pw_tpw(Spec<RS...>{}, d, stride + nfft)) return false;
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
#endif  // __HIPCC_RTC__

}  // namespace gdsp

#ifndef __HIPCC_RTC__
// One translation unit per group of specialisations (fft_specs*.hip), so the
// groups compile in parallel; fft_mixed.hip asks each group in turn.
#define GDSP_SPEC_GROUP(NAME, ...)                                                            \
  namespace gdsp {                                                                            \
  using NAME##_list = std::tuple<__VA_ARGS__>;                                                \
  bool NAME##_find(int n, int *rad, int *npass) {                                             \
    return find_spec(NAME##_list{}, n, rad, npass);                                           \
  }                                                                                           \
  bool NAME##_launch(const MixedDesc &d, bool inv, int load, const void *in, cd *out,         \
                     int64_t batch, const cd *tw, double scale, hipStream_t s) {             \
    return launch_spec(NAME##_list{}, d, inv, load, in, out, batch, tw, scale, s);            \
  }                                                                                           \
  int NAME##_pw_tpw(const MixedDesc &d, int64_t span) {                                     \
    return find_pw_tpw(NAME##_list{}, d, span);                                               \
  }                                                                                           \
  bool NAME##_pw_launch(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,    \
                        int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,   \
                        const double *win, const cd *tw, double *partial, hipStream_t s) {   \
    return launch_pw_spec(NAME##_list{}, d, x, nfft, stride, seg_begin, seg_end, ppw,         \
                          nworkers, win, tw, partial, s);                                     \
  }                                                                                           \
  }
#endif  // __HIPCC_RTC__
