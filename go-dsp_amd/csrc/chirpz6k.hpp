// chirpz6k.hpp — the fused chirp-z kernel on M = 16 * RB * 16 (chirpz6k.hip
// has the design notes and the length table; chirpz6k*.hip instantiate it).
#pragma once
#include "fft_device.hpp"
#include "launch.hpp"
#include "mixed_core.hpp"

namespace gdsp {

// (kernel and helpers outside an anonymous namespace, so profiler kernel
// names read gdsp::chirpz6k_kernel<...>)
constexpr int kC6B = 256;  // pass-B butterflies (every RB)
// Waves per SIMD the registers are held to (tools/resusage.py, round 6): 4
// (128 VGPRs) where that spills at most 8 VGPRs and lets more workgroups
// share a CU — RB = 18, 20, 21 (no spills), 24 (round 3: 2.37 against 3.13 ms
// at 144), 25 (8 spills, two 7-wave workgroups instead of one); elsewhere the
// natural count at 3 per SIMD: RB < 18 (140-168 VGPRs; at 128 they spill
// 4-172).
constexpr int c6_wpe(int rb) { return (rb >= 18 && rb <= 21) || rb == 24 || rb == 25 ? 4 : 3; }
template <int RB>
struct C6Geo {
  static constexpr int M = 256 * RB;  // points
  static constexpr int NA = M / 16;   // pass A / C butterflies of one transform
  // transforms per workgroup: one, or for RB <= 8 (NA <= 128) as many as keep
  // the 256 threads busy in passes A and C (pass B: 256 butterflies each)
  static constexpr int TPW = NA >= kC6B ? 1 : kC6B / NA;
  static constexpr int T = TPW * NA > kC6B ? TPW * NA : kC6B;  // threads
  static constexpr int WPE = c6_wpe(RB);
};

// x * W_24^q (q a compile-time constant after unrolling)
#define GDSP_C24 0.96592582628906828675  // cos(pi/12)
#define GDSP_S24 0.25881904510252076235  // sin(pi/12)
#define GDSP_C12 0.86602540378443864676  // cos(pi/6)
__device__ __forceinline__ cd rot24(cd x, int q) {
  q %= 24;
  if (q % 3 == 0) return rot16(x, 2 * (q / 3));  // W_24^(3k) = W_16^(2k)
  double c, s;                                   // W_24^q = c - i s
  switch (q) {
    case 1: c = GDSP_C24; s = GDSP_S24; break;
    case 2: c = GDSP_C12; s = 0.5; break;
    case 4: c = 0.5; s = GDSP_C12; break;
    case 5: c = GDSP_S24; s = GDSP_C24; break;
    case 7: c = -GDSP_S24; s = GDSP_C24; break;
    case 8: c = -0.5; s = GDSP_C12; break;
    case 10: c = -GDSP_C12; s = 0.5; break;
    case 11: c = -GDSP_C24; s = GDSP_S24; break;
    case 13: c = -GDSP_C24; s = -GDSP_S24; break;
    case 14: c = -GDSP_C12; s = -0.5; break;
    case 16: c = -0.5; s = -GDSP_C12; break;
    case 17: c = -GDSP_S24; s = -GDSP_C24; break;
    case 19: c = GDSP_S24; s = -GDSP_C24; break;
    case 20: c = 0.5; s = -GDSP_C12; break;
    case 22: c = GDSP_C12; s = -0.5; break;
    default: c = GDSP_C24; s = -GDSP_S24; break;  // 23
  }
  return {fma(x.x, c, x.y * s), fma(x.y, c, -(x.x * s))};
}

// DFT_R, R = 3 Q (Q = 8: 24, Q = 4: 12): DFT_Q over n1 (n = 3 n1 + n2),
// twiddles W_R^(n2 k1) (= W_24^((24 / R) n2 k1)), DFT_3 over n2 (k = k1 + Q k2)
template <int R>
__device__ __forceinline__ void dft3x(cd (&a)[R]) {
  constexpr int Q = R / 3, S = 24 / R;
  cd y[3][Q];
#pragma unroll
  for (int n2 = 0; n2 < 3; ++n2) {
    cd tmp[Q];
#pragma unroll
    for (int n1 = 0; n1 < Q; ++n1) tmp[n1] = a[3 * n1 + n2];
    Dft<Q>::run(tmp);
#pragma unroll
    for (int k1 = 0; k1 < Q; ++k1) y[n2][k1] = tmp[k1];
  }
#pragma unroll
  for (int k1 = 0; k1 < Q; ++k1) {
    const cd a0 = y[0][k1], a1 = rot24(y[1][k1], S * k1), a2 = rot24(y[2][k1], 2 * S * k1);
    // DFT_3: X1 = a0 - (a1 + a2)/2 - i sin(2 pi/3) (a1 - a2), X2 its mirror
    const cd s = a1 + a2, d = a1 - a2;
    const cd m = {fma(-0.5, s.x, a0.x), fma(-0.5, s.y, a0.y)};
    a[k1] = a0 + s;
    a[k1 + Q] = {fma(GDSP_C12, d.y, m.x), fma(-GDSP_C12, d.x, m.y)};
    a[k1 + 2 * Q] = {fma(-GDSP_C12, d.y, m.x), fma(GDSP_C12, d.x, m.y)};
  }
}

// v[r] *= w^r, r = 1..R-1, the powers by the three-term recurrence
// w^(r+2) = 2 cos(2 theta) w^r - w^(r-2) (two FMAs each, as pass_compute's
// CHEB) instead of twiddle_chain's products: 1.5 % faster, parity 3.7e-15
// against 1.6e-15 vs the oracle (profiles/r03/chirpz6k_ab.txt)
template <int R>
__device__ __forceinline__ void c6_twiddle(cd (&v)[R], cd w) {
  if constexpr (R == 2) {
    v[1] = cmul(v[1], w);
  } else {
    const cd w2 = cmul(w, w);
    v[1] = cmul(v[1], w);
    v[2] = cmul(v[2], w2);
    const double c2 = w2.x + w2.x;
    cd om = conjg(w), o = w;     // odd powers w^(r-2), w^r
    cd em = {1.0, 0.0}, e = w2;  // even powers
#pragma unroll
    for (int r = 3; r < R; ++r) {
      if (r & 1) {
        const cd q = {fma(c2, o.x, -om.x), fma(c2, o.y, -om.y)};
        om = o;
        o = q;
        v[r] = cmul(v[r], o);
      } else {
        const cd q = {fma(c2, e.x, -em.x), fma(c2, e.y, -em.y)};
        em = e;
        e = q;
        v[r] = cmul(v[r], e);
      }
    }
  }
}

// The steps after each FFT's last DFT: FFT 1's bhat step, FFT 2's
// postmultiply and store (issue: the loads, apply: the arithmetic). Issued
// before the pass-C twiddles or the last exchange's reads instead, the loads
// push the kernel past 128 VGPRs into spills: 2.43 against 2.37 ms.
template <class G>
struct C6BhatG {
  rsrc_t rb;
  uint32_t off;
  cd f[16];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      f[r] = buf_ld(rb, off + (uint32_t)(r * G::NA * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = conjg(cmul(v[r], f[r]));
  }
};
template <class G, int KN, bool INV>
struct C6OutG {
  rsrc_t rch, rout;
  uint32_t off;
  double scale;
  bool ok;  // the row exists (TPW > 1: the last workgroup's extra slots)
  cd f[KN];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < KN; ++r)
      f[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      cd y = cmul(conjg(v[r]), f[r]);
      if constexpr (INV) y = {y.x * scale, -y.y * scale};
      if (G::TPW == 1 || ok) buf_st_nt(rout, off + (uint32_t)(r * G::NA * 16), y);
    }
  }
};
template <int RB>
using C6Bhat = C6BhatG<C6Geo<RB>>;
template <int RB, int KN, bool INV>
using C6Out = C6OutG<C6Geo<RB>, KN, INV>;

// One FFT_M of the thread's registers v[r] = element t + NA r, in place
// (natural order in and out), then epi. ZIN: inputs r >= ZIN are zero (pass
// A pruned); first: no exchange precedes this one in the kernel. tw: the pass
// twiddle bases, W_{16 RB}^k (k < 16, pass B) then W_M^k (k < NA, pass C).
// Threads t >= NA (M = 6144: none) sit out passes A and C, threads t >= 256
// (M = 3072: none) pass B; all take part in the barriers.
template <int RB, int ZIN, class EPI>
__device__ __forceinline__ void c6_fft(cd (&v)[16], int t, const cd *__restrict__ tw, double *lds,
                                       bool first, EPI &epi) {
  using G = C6Geo<RB>;
  const bool pa = G::NA == G::T || t < G::NA;
  const bool pb = kC6B == G::T || t < kC6B;
  // pass A
  if (pa) {
    if constexpr (ZIN > 0 && ZIN <= 8) dft_half_in<16, ZIN>(v);
    else Dft<16>::run(v);
  }
  // exchange 1: write 16 t + r, read t + 256 r (t < 256)
  // (the twiddle bases are read where they are used: read a pass ahead,
  // 3.2-3.3 against 2.37 ms)
  const int wa = 16 * t, ma = t & 15;
  const int ra = t ^ ((t >> 4) & 15);
  cd u[RB];
  if (!first) __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].x;
  }
  __syncthreads();
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) u[r].x = lds[ra + kC6B * r];
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].y;
  }
  __syncthreads();
  // pass B
  const int wbo = (t >> 4) * (16 * RB) + (t & 15);
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) u[r].y = lds[ra + kC6B * r];
    c6_twiddle<RB>(u, tw[t & 15]);
    if constexpr (RB == 24 || RB == 12) dft3x<RB>(u);  // (measured, round 3)
    else dft_m<RB>(u);
  }
  __syncthreads();
  // exchange 2: write (t / 16) 16 RB + t % 16 + 16 r, read t + NA r
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) lds[wbo + 16 * r] = u[r].x;
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].x = lds[t + G::NA * r];
  }
  __syncthreads();
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) lds[wbo + 16 * r] = u[r].y;
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].y = lds[t + G::NA * r];
  }
  if (pa) {
    // pass C: twiddle W_M^(t r), DFT_16, the epilogue
    c6_twiddle<16>(v, tw[16 + t]);
    Dft<16>::run(v);
    epi.issue();
    epi.apply(v);
  }
}

// c6_fft for TPW > 1 transforms per workgroup (RB <= 8): thread t holds
// element tt + NA r of transform s (t = s NA + tt) in passes A and C, and
// takes pass-B butterfly t of every transform; transform s exchanges through
// lds + s M. (A separate function: folding TPW = 1 into it, the same
// arithmetic, cost the RB = 24 / 25 kernels 14-36 spilled VGPRs.)
template <int RB, int ZIN, class EPI>
__device__ __forceinline__ void c6_fft_multi(cd (&v)[16], int t, int s, int tt,
                                       const cd *__restrict__ tw, double *lds, bool first,
                                       EPI &epi) {
  using G = C6Geo<RB>;
  constexpr int TPW = G::TPW, M = G::M;
  static_assert(TPW > 1 && G::T == kC6B, "several transforms per 256-thread workgroup");
  const bool pa = t < TPW * G::NA;
  double *const la = lds + s * M;
  // pass A
  if (pa) {
    if constexpr (ZIN > 0 && ZIN <= 8) dft_half_in<16, ZIN>(v);
    else Dft<16>::run(v);
  }
  // exchange 1: write 16 tt + r, read t + 256 r (t < 256)
  // (the twiddle bases are read where they are used: read a pass ahead,
  // 3.2-3.3 against 2.37 ms)
  const int wa = 16 * tt, ma = tt & 15;
  const int ra = t ^ ((t >> 4) & 15);
  cd u[TPW][RB];
  if (!first) __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) la[wa + (r ^ ma)] = v[r].x;
  }
  __syncthreads();
  {
#pragma unroll
    for (int q = 0; q < TPW; ++q)
#pragma unroll
      for (int r = 0; r < RB; ++r) u[q][r].x = lds[q * M + ra + kC6B * r];
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) la[wa + (r ^ ma)] = v[r].y;
  }
  __syncthreads();
  // pass B
  const int wbo = (t >> 4) * (16 * RB) + (t & 15);
  {
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
#pragma unroll
      for (int r = 0; r < RB; ++r) u[q][r].y = lds[q * M + ra + kC6B * r];
      c6_twiddle<RB>(u[q], tw[t & 15]);
      if constexpr (RB == 24 || RB == 12) dft3x<RB>(u[q]);  // (measured, round 3)
      else dft_m<RB>(u[q]);
    }
  }
  __syncthreads();
  // exchange 2: write (t / 16) 16 RB + t % 16 + 16 r, read tt + NA r
  {
#pragma unroll
    for (int q = 0; q < TPW; ++q)
#pragma unroll
      for (int r = 0; r < RB; ++r) lds[q * M + wbo + 16 * r] = u[q][r].x;
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].x = la[tt + G::NA * r];
  }
  __syncthreads();
  {
#pragma unroll
    for (int q = 0; q < TPW; ++q)
#pragma unroll
      for (int r = 0; r < RB; ++r) lds[q * M + wbo + 16 * r] = u[q][r].y;
  }
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].y = la[tt + G::NA * r];
  }
  if (pa) {
    // pass C: twiddle W_M^(tt r), DFT_16, the epilogue
    c6_twiddle<16>(v, tw[16 + tt]);
    Dft<16>::run(v);
    epi.issue();
    epi.apply(v);
  }
}

// M = 6144: two workgroups of 6 waves share a CU. Held to 128 VGPRs (4 waves
// per SIMD of room): at 144 (3 per SIMD) the second workgroup's waves did not
// fit beside the first's 2-2-1-1 placement and the kernel ran 3.13 against
// 2.43 ms (profiles/r03/chirpz6k_ab.txt). M = 3072 (4-wave workgroups, one
// wave per SIMD each) takes its natural 144-146 VGPRs, three per SIMD: at 128
// it spills 54-78.
// KN: n <= NA KN (inputs and wanted outputs at r < KN)
// REAL: float64 input rows (fft.FFTReal, fft/fft.go:25-27), read directly
// (no complex copy of the input first)
//
// One transform (row g) of the workgroup: premultiply, FFT 1, bhat, FFT 2,
// postmultiply and store.
// Measured and not kept (round 4, profiles/r04/chirpz6k_ablation.txt): with the
// row's loads replaced by constants the launch takes 16 % less, but hiding
// them did not pay at the 128 VGPRs two workgroups per CU allow — an L2
// touch-ahead of a later block's row (1-6 % slower at every distance), a
// persistent form touching its next row (29 spilled VGPRs, 2.97 ms), the row
// by LDS-DMA into the idle exchange buffer (equal), two rows per workgroup
// with the second one's DMA in flight (26 spilled VGPRs, 5 % slower).
template <int RB, bool INV, int KN, bool REAL>
__device__ __forceinline__ void c6_transform(const void *__restrict__ in, cd *__restrict__ out,
                                             int64_t n, int64_t g, bool ok, int t, int s, int tt,
                                             const cd *tw, const cd *chirp, const cd *bhat,
                                             double scale, double *lds) {
  using G = C6Geo<RB>;
  const uint32_t off = (uint32_t)tt * 16u;
  const int64_t rowb = n * 16;
  const int64_t inb = REAL ? n * 8 : rowb;
  cd v[16];
  if (G::TPW * G::NA == G::T || t < G::TPW * G::NA) {
    cd xv[KN], cv[KN];
    if (G::TPW == 1 || ok) {
      const rsrc_t rin = make_rsrc(static_cast<const char *>(in) + g * inb, inb);
      const rsrc_t rch = make_rsrc(chirp, rowb);
#pragma unroll
      for (int r = 0; r < KN; ++r) {
        if constexpr (REAL)
          xv[r] = {buf_ld1(rin, (uint32_t)tt * 8u + (uint32_t)(r * G::NA * 8)), 0.0};
        else
          xv[r] = buf_ld(rin, off + (uint32_t)(r * G::NA * 16));
        cv[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
      }
    } else {
#pragma unroll
      for (int r = 0; r < KN; ++r) xv[r] = cv[r] = {0.0, 0.0};
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r < KN) {
        cd x = xv[r];
        if constexpr (INV) x.y = -x.y;
        v[r] = cmul(x, cv[r]);
      } else {
        v[r] = {0.0, 0.0};
      }
    }
  }
  C6Bhat<RB> be{make_rsrc(bhat, (int64_t)G::M * 16), off, {}};
  if constexpr (G::TPW == 1) c6_fft<RB, KN, C6Bhat<RB>>(v, t, tw, lds, true, be);
  else c6_fft_multi<RB, KN, C6Bhat<RB>>(v, t, s, tt, tw, lds, true, be);
  // the second FFT must not share the first one's addresses (opaque copies:
  // otherwise the compiler keeps them live across both)
  const int t2 = opaque_int(t), tt2 = G::TPW == 1 ? t2 : opaque_int(tt);
  C6Out<RB, KN, INV> oe{make_rsrc(opaque_ptr(chirp), rowb), make_rsrc(out + g * n, rowb),
                        (uint32_t)tt2 * 16u, scale, G::TPW == 1 || ok, {}};
  if constexpr (G::TPW == 1)
    c6_fft<RB, 0, C6Out<RB, KN, INV>>(v, t2, opaque_ptr(tw), lds, false, oe);
  else
    c6_fft_multi<RB, 0, C6Out<RB, KN, INV>>(v, t2, s, tt2, opaque_ptr(tw), lds, false, oe);
}

template <int RB, bool INV, int KN, bool REAL = false>
__global__ __launch_bounds__(C6Geo<RB>::T) __attribute__((amdgpu_waves_per_eu(C6Geo<RB>::WPE))) void chirpz6k_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ tw, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale) {
  using G = C6Geo<RB>;
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  __shared__ double lds[G::TPW * G::M];
  const int t = (int)threadIdx.x;
  const int s = G::TPW == 1 ? 0 : t / G::NA, tt = t - s * G::NA;
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x) * G::TPW + s;
  if constexpr (G::TPW == 1) {
    if (g >= batch) return;  // (grid = batch: never taken)
  }
  const bool ok = s < G::TPW && g < batch;  // (TPW > 1: every thread reaches the barriers)
  c6_transform<RB, INV, KN, REAL>(in, out, n, g, ok, t, s, tt, tw, chirp, bhat, scale, lds);
}

template <int RB>
hipError_t launch_c6(bool inv, int load, const void *in, cd *out, int64_t n, int64_t batch,
                     const cd *tw, const cd *chirp, const cd *bhat, double scale, hipStream_t s) {
  const dim3 grid((unsigned)((batch + C6Geo<RB>::TPW - 1) / C6Geo<RB>::TPW)), block(C6Geo<RB>::T);
  if (load == LOAD_REAL)
    hipLaunchKernelGGL((chirpz6k_kernel<RB, false, 8, true>), grid, block, 0, s, in, out, n, batch,
                       tw, chirp, bhat, scale);
  else if (inv)
    hipLaunchKernelGGL((chirpz6k_kernel<RB, true, 8>), grid, block, 0, s, in, out, n, batch, tw,
                       chirp, bhat, scale);
  else
    hipLaunchKernelGGL((chirpz6k_kernel<RB, false, 8>), grid, block, 0, s, in, out, n, batch, tw,
                       chirp, bhat, scale);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The same fused chirp-z with pass B split in two: M = 16 * R1 * R2 * 16
// (chirpz4_kernel, round 6), for the convolution lengths pass B cannot hold in
// registers (R1 R2 = 36, 40, 48 as kept, chirpz6k.hip kC4: M = 9216 ...
// 12288, 4097 <= n <= 6144, where the reference pads to 16384). One workgroup
// per transform of T = M / 16 threads:
//   pass A   R = 16, NS = 1:          DFT_16 of t + NA r (pruned input), as c6
//   pass B1  R = R1, NS = 16:         butterflies j = t + T q (q < J1)
//   pass B2  R = R2, NS = 16 R1:      butterflies j = t + T q (q < J2)
//   pass C   R = 16, NS = 16 R1 R2:   outputs t + NA r (natural order)
// then, as c6, v = conj(A * bhat) in registers, FFT 2 on the same passes, X =
// conj(v) * conj(w) for r < KN. Exchanges as real then imaginary halves
// through one M-double buffer: A -> B1 through c6's swizzle (slot e ^ ((e >>
// 4) & 15)), B1 -> B2 and B2 -> C plain. Twiddle bases (make_mixed_desc of
// {16, R1, R2, 16}): W_{16 R1}^k (16), W_{16 R1 R2}^k (16 R1), W_M^k (NA);
// powers by c6_twiddle's recurrence.
template <int R1_, int R2_>
struct C4Geo {
  static constexpr int R1 = R1_, R2 = R2_;
  static constexpr int M = 256 * R1 * R2;
  static constexpr int NA = M / 16;  // pass A / C butterflies = threads
  static constexpr int T = NA;
  static constexpr int TPW = 1;
  static constexpr int NB1 = M / R1, NB2 = M / R2;  // pass B1 / B2 butterflies
  static constexpr int J1 = (NB1 + T - 1) / T, J2 = (NB2 + T - 1) / T;
  static_assert(T <= 1024, "one workgroup per transform");
};

__device__ __forceinline__ int c6_swz(int e) { return e ^ ((e >> 4) & 15); }

// one middle pass (radix R, stride NS, twiddle bases twb) between two
// exchanges: read its J butterflies' inputs from the buffer (SWZ: written by
// pass A), compute into u
template <int M, int T, int R, int NS, int J, bool SWZ>
__device__ __forceinline__ void c4_read(cd (&u)[J][R], int t, const double *lds, int part) {
  constexpr int NB = M / R;
#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = t + T * q;
    if (NB % T == 0 || j < NB) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int e = j + NB * r;
        const double x = lds[SWZ ? c6_swz(e) : e];
        if (part) u[q][r].y = x;
        else u[q][r].x = x;
      }
    }
  }
}
template <int M, int T, int R, int NS, int J>
__device__ __forceinline__ void c4_compute(cd (&u)[J][R], int t, const cd *__restrict__ twb) {
  constexpr int NB = M / R;
#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = t + T * q;
    if (NB % T == 0 || j < NB) {
      c6_twiddle<R>(u[q], twb[j % NS]);
      dft_m<R>(u[q]);
    }
  }
}
template <int M, int T, int R, int NS, int J>
__device__ __forceinline__ void c4_write(const cd (&u)[J][R], int t, double *lds, int part) {
  constexpr int NB = M / R;
#pragma unroll
  for (int q = 0; q < J; ++q) {
    const int j = t + T * q;
    if (NB % T == 0 || j < NB) {
      const int k = j % NS, o = (j - k) * R + k;
#pragma unroll
      for (int r = 0; r < R; ++r) lds[o + NS * r] = part ? u[q][r].y : u[q][r].x;
    }
  }
}

template <class G, int ZIN, class EPI>
__device__ __forceinline__ void c4_fft(cd (&v)[16], int t, const cd *__restrict__ tw, double *lds,
                                       bool first, EPI &epi) {
  constexpr int M = G::M, T = G::T, NA = G::NA, R1 = G::R1, R2 = G::R2;
  // pass A
  if constexpr (ZIN > 0 && ZIN <= 8) dft_half_in<16, ZIN>(v);
  else Dft<16>::run(v);
  // exchange A -> B1 (write 16 t + r, swizzled)
  const int wa = 16 * t, ma = t & 15;
  cd u1[G::J1][R1];
  if (!first) __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].x;
  __syncthreads();
  c4_read<M, T, R1, 16, G::J1, true>(u1, t, lds, 0);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].y;
  __syncthreads();
  c4_read<M, T, R1, 16, G::J1, true>(u1, t, lds, 1);
  // pass B1
  c4_compute<M, T, R1, 16, G::J1>(u1, t, tw);
  // exchange B1 -> B2
  cd u2[G::J2][R2];
  __syncthreads();
  c4_write<M, T, R1, 16, G::J1>(u1, t, lds, 0);
  __syncthreads();
  c4_read<M, T, R2, 16 * R1, G::J2, false>(u2, t, lds, 0);
  __syncthreads();
  c4_write<M, T, R1, 16, G::J1>(u1, t, lds, 1);
  __syncthreads();
  c4_read<M, T, R2, 16 * R1, G::J2, false>(u2, t, lds, 1);
  // pass B2
  c4_compute<M, T, R2, 16 * R1, G::J2>(u2, t, tw + 16);
  // exchange B2 -> C (read t + NA r)
  __syncthreads();
  c4_write<M, T, R2, 16 * R1, G::J2>(u2, t, lds, 0);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r].x = lds[t + NA * r];
  __syncthreads();
  c4_write<M, T, R2, 16 * R1, G::J2>(u2, t, lds, 1);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r].y = lds[t + NA * r];
  // pass C: twiddle W_M^(t r), DFT_16, the epilogue
  c6_twiddle<16>(v, tw[16 + 16 * R1 + t]);
  Dft<16>::run(v);
  epi.issue();
  epi.apply(v);
}

template <int R1, int R2, bool INV, int KN, bool REAL = false>
__global__ __launch_bounds__((C4Geo<R1, R2>::T)) void chirpz4_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ tw, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale) {
  using G = C4Geo<R1, R2>;
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  __shared__ double lds[G::M];
  const int t = (int)threadIdx.x;
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  if (g >= batch) return;  // (grid = batch: never taken)
  const uint32_t off = (uint32_t)t * 16u;
  const int64_t rowb = n * 16;
  const int64_t inb = REAL ? n * 8 : rowb;
  cd v[16];
  {
    const rsrc_t rin = make_rsrc(static_cast<const char *>(in) + g * inb, inb);
    const rsrc_t rch = make_rsrc(chirp, rowb);
    cd xv[KN], cv[KN];
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      if constexpr (REAL)
        xv[r] = {buf_ld1(rin, (uint32_t)t * 8u + (uint32_t)(r * G::NA * 8)), 0.0};
      else
        xv[r] = buf_ld(rin, off + (uint32_t)(r * G::NA * 16));
      cv[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r < KN) {
        cd x = xv[r];
        if constexpr (INV) x.y = -x.y;
        v[r] = cmul(x, cv[r]);
      } else {
        v[r] = {0.0, 0.0};
      }
    }
  }
  C6BhatG<G> be{make_rsrc(bhat, (int64_t)G::M * 16), off, {}};
  c4_fft<G, KN, C6BhatG<G>>(v, t, tw, lds, true, be);
  const int t2 = opaque_int(t);
  C6OutG<G, KN, INV> oe{make_rsrc(opaque_ptr(chirp), rowb), make_rsrc(out + g * n, rowb),
                        (uint32_t)t2 * 16u, scale, true, {}};
  c4_fft<G, 0, C6OutG<G, KN, INV>>(v, t2, opaque_ptr(tw), lds, false, oe);
}

template <int R1, int R2>
hipError_t launch_c4(bool inv, int load, const void *in, cd *out, int64_t n, int64_t batch,
                     const cd *tw, const cd *chirp, const cd *bhat, double scale, hipStream_t s) {
  const dim3 grid((unsigned)batch), block(C4Geo<R1, R2>::T);
  if (load == LOAD_REAL)
    hipLaunchKernelGGL((chirpz4_kernel<R1, R2, false, 8, true>), grid, block, 0, s, in, out, n,
                       batch, tw, chirp, bhat, scale);
  else if (inv)
    hipLaunchKernelGGL((chirpz4_kernel<R1, R2, true, 8>), grid, block, 0, s, in, out, n, batch,
                       tw, chirp, bhat, scale);
  else
    hipLaunchKernelGGL((chirpz4_kernel<R1, R2, false, 8>), grid, block, 0, s, in, out, n, batch,
                       tw, chirp, bhat, scale);
  return hipGetLastError();
}
#define GDSP_C4_LAUNCH(PRE, R1, R2)                                                             \
  PRE template hipError_t launch_c4<R1, R2>(bool, int, const void *, cd *, int64_t, int64_t,    \
                                            const cd *, const cd *, const cd *, double,         \
                                            hipStream_t);

// explicit instantiations (chirpz6k*.hip) and their declarations
#define GDSP_C6_LAUNCH(PRE, RB)                                                                 \
  PRE template hipError_t launch_c6<RB>(bool, int, const void *, cd *, int64_t, int64_t,        \
                                        const cd *, const cd *, const cd *, double, hipStream_t);
}  // namespace gdsp
