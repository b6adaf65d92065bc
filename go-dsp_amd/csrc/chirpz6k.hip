// chirpz6k.hip — fused chirp-z (Bluestein, fft/bluestein.go:68-94) on the
// convolution length M = 16 * RB * 16 = 3 * 2^k: M = 6144 (RB = 24) for
// 2049 <= n <= 3072 and M = 3072 (RB = 12) for 1025 <= n <= 1536.
//
// bluestein.go:70 pads the circular convolution to NextPowerOf2(2n - 1)
// (8192, 4096) for these n because its FFT is radix 2. Any M >= 2n - 1 gives
// the same linear convolution, hence the same DFT; 3 * 2^k is a quarter fewer
// points. At M = 6144 the exchange buffer (48 KiB) and a 16-point-per-thread
// register set let two 384-thread workgroups share a CU at 128 VGPRs, where
// the M = 8192 kernel (bluestein_kernel<13>, 32 points per thread, 256 VGPRs)
// runs two 256-thread ones.
//
// One workgroup per transform, T = max(M / 16, 256) threads (thread t):
//   premultiply  a[t + NA r] = x * conj(w), r < KN (n <= NA KN; rest zero),
//                NA = M / 16 (pass A and C butterflies)
//   FFT 1        pass A  R = 16, NS = 1:      DFT_16 of t + NA r (pruned input)
//                pass B  R = RB, NS = 16:     t < 256, inputs t + 256 r
//                pass C  R = 16, NS = 16 RB:  outputs t + NA r (natural order)
//   middle       v = conj(A * bhat) in registers: pass C's outputs are pass
//                A's inputs of FFT 2, so no exchange between the two FFTs
//   FFT 2        pass A, B, C again; the outputs r < KN are the wanted ones:
//                X = conj(v) * conj(w) (the rest of the last DFT is dead code)
// Stockham passes (fft_device.hpp): butterfly j of pass (R, NS) reads
// j + r M/R and writes (j / NS) NS R + j % NS + r NS, twiddle W_{NS R}^{(j %
// NS) r}. Exchanges go through one M-double LDS buffer, real then imaginary
// parts. Slots: after pass A (stride-16 writes) XOR-swizzled, i ^ ((i >> 4)
// & 15) — every 16-lane write group and 32-lane read group hits distinct
// banks; after pass B plain (16 contiguous writes, 32 contiguous reads).
#include "fft_device.hpp"
#include "launch.hpp"
#include "mixed_core.hpp"

#ifndef GDSP_C6_TOUCH
#define GDSP_C6_TOUCH 1
#endif
namespace gdsp {

// (kernel and helpers outside an anonymous namespace, so profiler kernel
// names read gdsp::chirpz6k_kernel<...>)
constexpr int kC6B = 256;  // pass-B butterflies (both sizes)
template <int RB>
struct C6Geo {
  static constexpr int M = 256 * RB;               // points
  static constexpr int NA = M / 16;                // pass A / C butterflies
  static constexpr int T = NA > kC6B ? NA : kC6B;  // threads
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
  {
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
template <int RB, int ABL = 0>
struct C6Bhat {
  using G = C6Geo<RB>;
  rsrc_t rb;
  uint32_t off;
  cd f[16];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      f[r] = (ABL & 2) ? cd{1.0 + 1e-3 * r, (double)off * 1e-9} : buf_ld(rb, off + (uint32_t)(r * G::NA * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = conjg(cmul(v[r], f[r]));
  }
};
template <int RB, int KN, bool INV, int ABL = 0>
struct C6Out {
  using G = C6Geo<RB>;
  rsrc_t rch, rout;
  uint32_t off;
  double scale;
  cd f[KN];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < KN; ++r)
      f[r] = (ABL & 4) ? cd{1.0 - 1e-3 * r, (double)off * 1e-9} : buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      cd y = cmul(conjg(v[r]), f[r]);
      if constexpr (INV) y = {y.x * scale, -y.y * scale};
      buf_st_nt(rout, off + (uint32_t)(r * G::NA * 16), y);
    }
  }
};

// One FFT_M of the thread's registers v[r] = element t + NA r, in place
// (natural order in and out), then epi. ZIN: inputs r >= ZIN are zero (pass
// A pruned); first: no exchange precedes this one in the kernel. tw: the pass
// twiddle bases, W_{16 RB}^k (k < 16, pass B) then W_M^k (k < NA, pass C).
// Threads t >= NA (M = 6144: none) sit out passes A and C, threads t >= 256
// (M = 3072: none) pass B; all take part in the barriers.
// ABL (development ablations, results wrong): bit 3 drops the exchanges'
// barriers (a race, timing only)
// bit 6 (64, not an ablation): a barrier fencing LDS only. With an LDS-DMA in
// flight the compiler still waits vmcnt(0) at it (the DMA is a pending LDS
// write); the bare form (s_waitcnt lgkmcnt(0) + s_barrier between compiler
// memory barriers) keeps the DMA in flight but spilled 26 VGPRs in
// chirpz6k_x2_kernel and ran 5 % slower (profiles/r04/chirpz6k_ablation.txt)
template <int ABL>
__device__ __forceinline__ void c6_sync() {
  if constexpr (ABL & 64) {
    // (sched_barrier: nothing is scheduled across it, as across
    // __syncthreads; without, 22 VGPRs spill at 128)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  else if constexpr (!(ABL & 8)) __syncthreads();
}

// Hooks into c6_fft for the LDS-DMA-prefetching persistent kernel: after the
// first barrier of exchange 1, and between the last exchange and pass C (pa:
// this thread takes part in pass C); tw_b / tw_c give the pass twiddle bases
// (from registers where a load's wait would drain an LDS-DMA in flight).
struct C6NoHook {
  __device__ __forceinline__ void after_first(cd (&)[16]) {}
  __device__ __forceinline__ cd tw_b(const cd *tw, int t) const { return tw[t & 15]; }
  __device__ __forceinline__ cd tw_c(const cd *tw, int t) const { return tw[16 + t]; }
  __device__ __forceinline__ void before_c(const cd *, int, bool) {}
};

template <int RB, int ZIN, class EPI, int ABL = 0, class HOOK = C6NoHook>
__device__ __forceinline__ void c6_fft(cd (&v)[16], int t, const cd *__restrict__ tw, double *lds,
                                       bool first, EPI &epi, HOOK hk = {}) {
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
  if (!first) c6_sync<ABL>();
  hk.after_first(v);
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].x;
  }
  c6_sync<ABL>();
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) u[r].x = lds[ra + kC6B * r];
  }
  c6_sync<ABL>();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].y;
  }
  c6_sync<ABL>();
  // pass B
  const int wbo = (t >> 4) * (16 * RB) + (t & 15);
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) u[r].y = lds[ra + kC6B * r];
    c6_twiddle<RB>(u, hk.tw_b(tw, t));
    dft3x<RB>(u);
  }
  c6_sync<ABL>();
  // exchange 2: write (t / 16) 16 RB + t % 16 + 16 r, read t + NA r
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) lds[wbo + 16 * r] = u[r].x;
  }
  c6_sync<ABL>();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].x = lds[t + G::NA * r];
  }
  c6_sync<ABL>();
  if (pb) {
#pragma unroll
    for (int r = 0; r < RB; ++r) lds[wbo + 16 * r] = u[r].y;
  }
  c6_sync<ABL>();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r].y = lds[t + G::NA * r];
  }
  hk.before_c(tw, t, pa);
  if (pa) {
    // pass C: twiddle W_M^(t r), DFT_16, the epilogue
    c6_twiddle<16>(v, hk.tw_c(tw, t));
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
// ABL: development ablations (timing only, results wrong; 0 in the product):
// 1 = x and chirp premultiply loads replaced by constants, 2 = bhat loads,
// 4 = the output chirp loads, 8 = no exchange barriers, 16 = x only, 32 = the
// premultiply chirp only
//
// One transform (row g) of the workgroup: premultiply, FFT 1, bhat, FFT 2,
// postmultiply and store. first: no exchange of this workgroup precedes it.
// touch (persistent kernel): the next row's bytes, one 128-B line per thread,
// loaded into L2 right after this row's loads issue (its result is held in one
// register to the end of the transform, so no wait ever lands on it early).
// XD: the row comes in by LDS-DMA (buffer_load ... lds) into the exchange
// buffer, idle at the transform's start, and is read from there (an
// all-DMA prologue: MI355X_MICROARCH.md's prologue-burst row, ~12-13 against
// ~11 B/cycle/CU for register loads); bytes past the row land as zeros.
template <int RB, bool INV, int KN, bool REAL, int ABL, bool XD = false>
__device__ __forceinline__ void c6_transform(const void *__restrict__ in, cd *__restrict__ out,
                                             int64_t n, int64_t g, int t, const cd *tw,
                                             const cd *chirp, const cd *bhat, double scale,
                                             double *lds, bool first, int64_t touch_row) {
  using G = C6Geo<RB>;
  const uint32_t off = (uint32_t)t * 16u;
  const int64_t rowb = n * 16;
  const int64_t inb = REAL ? n * 8 : rowb;
  cd v[16];
  unsigned touched = 0u;
  if constexpr (XD) {
    constexpr int NW = G::T / 64;            // waves
    constexpr int PIECES = G::M * 8 / 1024;  // 1-KiB pieces of the buffer
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const rsrc_t rin = make_rsrc(static_cast<const char *>(in) + g * inb, inb);
    const uint32_t lane16 = (uint32_t)(t & 63) * 16u;
    if (!first) __syncthreads();  // the previous transform's last exchange reads are done
#pragma unroll
    for (int i = 0; i < (PIECES + NW - 1) / NW; ++i) {
      const int p = w + i * NW;
      if (p < PIECES)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rin, (__attribute__((address_space(3))) void *)((char *)lds + p * 1024), 16,
            (uint32_t)p * 1024u + lane16, 0, 0, 0);
    }
    cd cv[KN];
    if (G::NA == G::T || t < G::NA) {
      const rsrc_t rch = make_rsrc(chirp, rowb);
#pragma unroll
      for (int r = 0; r < KN; ++r) cv[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (G::NA == G::T || t < G::NA) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r < KN) {
          cd x;
          if constexpr (REAL) x = {lds[t + r * G::NA], 0.0};
          else x = reinterpret_cast<const cd *>(lds)[t + r * G::NA];
          if constexpr (INV) x.y = -x.y;
          v[r] = cmul(x, cv[r]);
        } else {
          v[r] = {0.0, 0.0};
        }
      }
    }
    first = false;  // the exchange below must wait for every read of the row
  } else if (G::NA == G::T || t < G::NA) {
    const rsrc_t rin =
        make_rsrc(static_cast<const char *>(in) + g * inb, inb);
    const rsrc_t rch = make_rsrc(chirp, rowb);
    cd xv[KN], cv[KN];
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      if constexpr (ABL & 1) {
        xv[r] = {(double)(off + r) * 1e-7, (double)g * 1e-9};
        cv[r] = {1.0 - 1e-4 * r, 1e-5 * r};
      } else if constexpr (ABL & 16) {
        xv[r] = {(double)(off + r) * 1e-7, (double)g * 1e-9};
        cv[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
      } else if constexpr (ABL & 32) {
        xv[r] = buf_ld(rin, off + (uint32_t)(r * G::NA * 16));
        cv[r] = {1.0 - 1e-4 * r, 1e-5 * r};
      } else {
        if constexpr (REAL)
          xv[r] = {buf_ld1(rin, (uint32_t)t * 8u + (uint32_t)(r * G::NA * 8)), 0.0};
        else
          xv[r] = buf_ld(rin, off + (uint32_t)(r * G::NA * 16));
        cv[r] = buf_ld(rch, off + (uint32_t)(r * G::NA * 16));
      }
    }
    if (touch_row >= 0) {
      const rsrc_t rnx = make_rsrc(static_cast<const char *>(in) + touch_row * inb, inb);
      touched = __builtin_amdgcn_raw_buffer_load_b32(rnx, (uint32_t)t * 128u, 0, 0);
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
  C6Bhat<RB, ABL> be{make_rsrc(bhat, (int64_t)G::M * 16), off, {}};
  c6_fft<RB, KN, C6Bhat<RB, ABL>, ABL>(v, t, tw, lds, first, be);
  // the second FFT must not share the first one's addresses (opaque copies:
  // otherwise the compiler keeps them live across both)
  const int t2 = opaque_int(t);
  C6Out<RB, KN, INV, ABL> oe{make_rsrc(opaque_ptr(chirp), rowb), make_rsrc(out + g * n, rowb),
                             (uint32_t)t2 * 16u, scale, {}};
  c6_fft<RB, 0, C6Out<RB, KN, INV, ABL>, ABL>(v, t2, opaque_ptr(tw), lds, false, oe);
  if (touch_row >= 0) asm volatile("" ::"v"(touched));
}

// TA: touch into L2 the row of the block TA places later in dispatch order
// (the same XCD when TA is a multiple of 8; it should start after this block
// ends, so TA >= the resident blocks, 2 per CU)
template <int RB, bool INV, int KN, bool REAL = false, int ABL = 0, int TA = 0, bool XD = false>
__global__ __launch_bounds__(C6Geo<RB>::T) __attribute__((amdgpu_waves_per_eu(RB == 24 ? 4 : 3))) void chirpz6k_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ tw, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale) {
  using G = C6Geo<RB>;
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  __shared__ double lds[G::M];
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  if (g >= batch) return;  // (grid = batch: never taken)
  int64_t touch = -1;
  if constexpr (TA > 0) {
    const int64_t bn = (int64_t)blockIdx.x + TA;
    if (bn < (int64_t)gridDim.x) touch = xcd_remap(bn, gridDim.x);
  }
  c6_transform<RB, INV, KN, REAL, ABL, XD>(in, out, n, g, (int)threadIdx.x, tw, chirp, bhat,
                                           scale, lds, true, touch);
}

// Persistent form: one workgroup per resident slot, each over a contiguous
// run of rows, touching its next row into L2 while the current one runs (the
// one-transform-per-workgroup kernel waits on each row's HBM loads with
// nothing else to do: 16 % of its time, profiles/r04/chirpz6k_ablation.txt).
template <int RB, bool INV, int KN, bool REAL = false>
__global__ __launch_bounds__(C6Geo<RB>::T) __attribute__((amdgpu_waves_per_eu(RB == 24 ? 4 : 3))) void chirpz6k_persist_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    int64_t rows_per_wg, const cd *__restrict__ tw, const cd *__restrict__ chirp,
    const cd *__restrict__ bhat, double scale) {
  using G = C6Geo<RB>;
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  __shared__ double lds[G::M];
  const int64_t g0 = (int64_t)blockIdx.x * rows_per_wg;
  const int64_t g1 = g0 + rows_per_wg < batch ? g0 + rows_per_wg : batch;
  for (int64_t g = g0; g < g1; ++g) {
    // laundered per row: nothing address-like is hoisted out of the loop and
    // kept live across it (the compiler would, 59 spilled VGPRs at 128)
    c6_transform<RB, INV, KN, REAL, 0>(opaque_ptr(in), opaque_ptr(out), n, g,
                                       opaque_int((int)threadIdx.x), opaque_ptr(tw),
                                       opaque_ptr(chirp), opaque_ptr(bhat), scale, lds, g == g0,
                                       GDSP_C6_TOUCH ? (g + 1 < g1 ? g + 1 : -1) : -1);
  }
}

// Two rows per workgroup, straight-line (development build, GDSP_C6_X2=1):
// row A as the one-shot kernel while its FFTs bring row B in by LDS-DMA, then
// row B from LDS. Bytes [0, LZ) of row B (the whole row for float64 input)
// go to a landing zone of their own, issued after FFT 1's pass A of row A
// (the zone is idle), bytes [LZ, 16 n) to the same offsets of the exchange
// buffer, issued after FFT 2's last exchange (the buffer is idle from there
// to row B). While a DMA is in flight the compiler waits vmcnt(0) at the next
// use of any ordinary load (cdna_hip_programming.md, "Pipelining across
// barriers"), so row A's barriers fence LDS only (c6_sync<64>) and the pass
// twiddle bases come from an LDS copy (ds_read: lgkmcnt) — the first waits
// on a DMA are then FFT 1's bhat (part 1) and FFT 2's output chirp (part 2).
// Held in registers instead, the bases cost 38 spilled VGPRs at the 128 two
// workgroups per CU need; a persistent loop over rows spilled 27-112 (the
// compiler keeps loop-invariant addresses live across the loop), so this is
// two rows, not a loop. LDS per workgroup: 48 KiB exchange + 6.25 KiB
// twiddles + 24 KiB landing zone (dynamic, so the compiler's LDS occupancy
// model keeps the 4-waves register cap): two per CU.
template <int RB>
struct C6Dma {
  using G = C6Geo<RB>;
  static constexpr int LZ = G::M * 4;      // landing zone bytes (half the buffer)
  static constexpr int NTW = 16 + G::NA;   // twiddle bases in LDS
  static constexpr int DYN = NTW * 16 + LZ;
  static constexpr int NW = G::T / 64;
  // bytes [b0, b0 + 1024 P) of the row to dst + b0 - d0
  template <int P>
  __device__ __forceinline__ static void part(rsrc_t rin, char *dst, uint32_t b0, int w,
                                              uint32_t lane16) {
#pragma unroll
    for (int i = 0; i < (P + NW - 1) / NW; ++i) {
      const int p = w + i * NW;
      if (p < P)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rin, (__attribute__((address_space(3))) void *)(dst + p * 1024), 16, lane16,
            __builtin_amdgcn_readfirstlane(b0 + p * 1024), 0, 0);
    }
  }
};
struct C6LdsTw {  // twiddle bases from the LDS copy
  const cd *ltw;
  __device__ __forceinline__ void after_first(cd (&)[16]) {}
  __device__ __forceinline__ cd tw_b(const cd *, int t) const { return ltw[t & 15]; }
  __device__ __forceinline__ cd tw_c(const cd *, int t) const { return ltw[16 + t]; }
  __device__ __forceinline__ void before_c(const cd *, int, bool) {}
};
template <int RB>
struct C6DmaHook1 : C6LdsTw {  // FFT 1: row B's bytes [0, LZ) into the landing zone
  rsrc_t rnx;
  char *lz;
  int w;
  uint32_t lane16;
  bool go;
  __device__ __forceinline__ void after_first(cd (&v)[16]) {
    // pass A's results (so every use of row A's loads) complete before the
    // DMA issues: otherwise the arithmetic sinks below it and the first use
    // of a row-A load waits vmcnt(0), draining the DMA at once
#pragma unroll
    for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(v[r].x), "+v"(v[r].y)::"memory");
    if (go) C6Dma<RB>::template part<C6Dma<RB>::LZ / 1024>(rnx, lz, 0u, w, lane16);
  }
};
template <int RB, bool REAL>
struct C6DmaHook2 : C6LdsTw {  // FFT 2: the rest of row B into the exchange buffer
  rsrc_t rnx;
  char *xb;
  int w;
  uint32_t lane16;
  bool go;
  __device__ __forceinline__ void before_c(const cd *, int, bool) {
    if constexpr (!REAL) {
      c6_sync<64>();  // every read of the exchange buffer is done
      constexpr int P = (C6Geo<RB>::M * 8 - C6Dma<RB>::LZ) / 1024;
      if (go) C6Dma<RB>::template part<P>(rnx, xb + C6Dma<RB>::LZ, (uint32_t)C6Dma<RB>::LZ, w, lane16);
    }
  }
};

template <int RB, bool INV, int KN, bool REAL = false>
__global__ __launch_bounds__(C6Geo<RB>::T) __attribute__((amdgpu_waves_per_eu(4))) void chirpz6k_x2_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ tw, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale) {
  using G = C6Geo<RB>;
  using D = C6Dma<RB>;
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  static_assert(!REAL || G::M * 4 <= D::LZ, "float64 rows land whole");
  static_assert(REAL || G::NA * 4 * 16 == D::LZ, "complex rows split at r = 4");
  __shared__ double lds[G::M];
  extern __shared__ double dyn[];  // D::DYN bytes: twiddle bases, landing zone
  cd *const ltw = reinterpret_cast<cd *>(dyn);
  char *const lz = reinterpret_cast<char *>(dyn) + D::NTW * 16;
  const int t = threadIdx.x;
  const bool pa = G::NA == G::T || t < G::NA;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t rowb = n * 16;
  const int64_t inb = REAL ? n * 8 : rowb;
  const int64_t ga = 2 * xcd_remap(blockIdx.x, gridDim.x);
  if (ga >= batch) return;
  const bool hasb = ga + 1 < batch;
  const rsrc_t rnx = make_rsrc(static_cast<const char *>(in) + (hasb ? ga + 1 : ga) * inb, inb);
  for (int i = t; i < D::NTW; i += G::T) ltw[i] = tw[i];  // (first read after 2 barriers)
  // row A: registers, as the one-shot kernel
  {
    const uint32_t off = (uint32_t)t * 16u;
    cd v[16];
    if (pa) {
      const rsrc_t rin = make_rsrc(static_cast<const char *>(in) + ga * inb, inb);
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
    const uint32_t lane16 = (uint32_t)(t & 63) * 16u;
    C6Bhat<RB> be{make_rsrc(bhat, (int64_t)G::M * 16), off, {}};
    C6DmaHook1<RB> h1{{ltw}, rnx, lz, w, lane16, hasb};
    c6_fft<RB, KN, C6Bhat<RB>, 64, C6DmaHook1<RB>>(v, t, tw, lds, true, be, h1);
    const int t2 = opaque_int(t);
    C6Out<RB, KN, INV> oe{make_rsrc(opaque_ptr(chirp), rowb), make_rsrc(out + ga * n, rowb),
                          (uint32_t)t2 * 16u, scale, {}};
    C6DmaHook2<RB, REAL> h2{{ltw}, rnx, (char *)lds, w, (uint32_t)(t2 & 63) * 16u, hasb};
    c6_fft<RB, 0, C6Out<RB, KN, INV>, 64, C6DmaHook2<RB, REAL>>(v, t2, tw, lds, false, oe, h2);
  }
  if (!hasb) return;
  // row B: from the landing zone and the exchange buffer
  const int tb = opaque_int(t);
  const uint32_t offb = (uint32_t)tb * 16u;
  cd v[16];
  cd cv[KN];
  if (pa) {
    const rsrc_t rch = make_rsrc(opaque_ptr(chirp), rowb);
#pragma unroll
    for (int r = 0; r < KN; ++r) cv[r] = buf_ld(rch, offb + (uint32_t)(r * G::NA * 16));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // row B's DMA has landed
  __syncthreads();
  if (pa) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r < KN) {
        const int e = tb + r * G::NA;
        cd x;
        if constexpr (REAL) x = {reinterpret_cast<const double *>(lz)[e], 0.0};
        else if (r < 4) x = reinterpret_cast<const cd *>(lz)[e];
        else x = reinterpret_cast<const cd *>(lds)[e];
        if constexpr (INV) x.y = -x.y;
        v[r] = cmul(x, cv[r]);
      } else {
        v[r] = {0.0, 0.0};
      }
    }
  }
  C6LdsTw hb{ltw};
  C6Bhat<RB> be{make_rsrc(opaque_ptr(bhat), (int64_t)G::M * 16), offb, {}};
  c6_fft<RB, KN, C6Bhat<RB>, 0, C6LdsTw>(v, tb, tw, lds, false, be, hb);
  const int t2 = opaque_int(tb);
  C6Out<RB, KN, INV> oe{make_rsrc(opaque_ptr(chirp), rowb),
                        make_rsrc(opaque_ptr(out) + (ga + 1) * n, rowb), (uint32_t)t2 * 16u,
                        scale, {}};
  c6_fft<RB, 0, C6Out<RB, KN, INV>, 0, C6LdsTw>(v, t2, tw, lds, false, oe, hb);
}

// The convolution length for n (0: neither size applies)
int chirpz6k_m(int64_t n) {
  if (n >= 2049 && 2 * n - 1 <= 6144) return 6144;
  if (n >= 1025 && 2 * n - 1 <= 3072) return 3072;
  return 0;
}

template <int RB>
static hipError_t launch_c6(bool inv, int load, const void *in, cd *out, int64_t n, int64_t batch,
                            const cd *tw, const cd *chirp, const cd *bhat, double scale,
                            hipStream_t s) {
  const dim3 grid((unsigned)batch), block(C6Geo<RB>::T);
#ifdef GDSP_DEV_BUILD
  if constexpr (RB == 24) {
    // ablation timings (GDSP_C6_ABL = 1..15, forward complex only; wrong results)
    if (const char *e = dev_switch("GDSP_C6_ABL"); e && !inv && load != LOAD_REAL) {
      switch (atoi(e)) {
#define GDSP_C6A(A)                                                                              \
  case A:                                                                                        \
    hipLaunchKernelGGL((chirpz6k_kernel<24, false, 8, false, A>), grid, block, 0, s, in, out, n, \
                       batch, tw, chirp, bhat, scale);                                           \
    return hipGetLastError();
        GDSP_C6A(1) GDSP_C6A(2) GDSP_C6A(4) GDSP_C6A(7) GDSP_C6A(8) GDSP_C6A(15) GDSP_C6A(16) GDSP_C6A(32) GDSP_C6A(64)
#undef GDSP_C6A
        default: break;
      }
    }
  }
#endif
#ifdef GDSP_DEV_BUILD
  if (const char *e = dev_switch("GDSP_C6_TA"); e && !inv && load != LOAD_REAL) {
    switch (atoi(e)) {
#define GDSP_C6T(D)                                                                             \
  case D:                                                                                       \
    hipLaunchKernelGGL((chirpz6k_kernel<RB, false, 8, false, 0, D>), grid, block, 0, s, in, out, \
                       n, batch, tw, chirp, bhat, scale);                                       \
    return hipGetLastError();
      GDSP_C6T(256) GDSP_C6T(512) GDSP_C6T(768) GDSP_C6T(1024) GDSP_C6T(2048)
#undef GDSP_C6T
      default: break;
    }
  }
  if (const char *e = dev_switch("GDSP_C6_XDMA"); e && e[0] == '1') {
    if (load == LOAD_REAL)
      hipLaunchKernelGGL((chirpz6k_kernel<RB, false, 8, true, 0, 0, true>), grid, block, 0, s, in,
                         out, n, batch, tw, chirp, bhat, scale);
    else if (inv)
      hipLaunchKernelGGL((chirpz6k_kernel<RB, true, 8, false, 0, 0, true>), grid, block, 0, s, in,
                         out, n, batch, tw, chirp, bhat, scale);
    else
      hipLaunchKernelGGL((chirpz6k_kernel<RB, false, 8, false, 0, 0, true>), grid, block, 0, s, in,
                         out, n, batch, tw, chirp, bhat, scale);
    return hipGetLastError();
  }
  if (const char *e = dev_switch("GDSP_C6_X2"); RB == 24 && e && e[0] == '1') {
    const dim3 g2((unsigned)((batch + 1) / 2));
    if (load == LOAD_REAL)
      hipLaunchKernelGGL((chirpz6k_x2_kernel<RB, false, 8, true>), g2, block, C6Dma<RB>::DYN, s, in,
                         out, n, batch, tw, chirp, bhat, scale);
    else if (inv)
      hipLaunchKernelGGL((chirpz6k_x2_kernel<RB, true, 8>), g2, block, C6Dma<RB>::DYN, s, in, out, n,
                         batch, tw, chirp, bhat, scale);
    else
      hipLaunchKernelGGL((chirpz6k_x2_kernel<RB, false, 8>), g2, block, C6Dma<RB>::DYN, s, in, out,
                         n, batch, tw, chirp, bhat, scale);
    return hipGetLastError();
  }
  if (const char *e = dev_switch("GDSP_C6_PERSIST"); e && e[0] == '1') {
    // one workgroup per resident slot (occupancy x CUs of the current device)
    static int slots_per_cu = 0, cus = 0;
    if (!slots_per_cu) {
      int dev = 0, nb = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &nb, reinterpret_cast<const void *>(&chirpz6k_persist_kernel<RB, false, 8>),
          C6Geo<RB>::T, 0);
      slots_per_cu = nb > 0 ? nb : 1;
    }
    const int64_t slots = (int64_t)slots_per_cu * (cus > 0 ? cus : 1);
    const int64_t nwg = batch < slots ? batch : slots;
    const int64_t rpw = (batch + nwg - 1) / nwg;
    const dim3 pg((unsigned)((batch + rpw - 1) / rpw));
    if (load == LOAD_REAL)
      hipLaunchKernelGGL((chirpz6k_persist_kernel<RB, false, 8, true>), pg, block, 0, s, in, out, n,
                         batch, rpw, tw, chirp, bhat, scale);
    else if (inv)
      hipLaunchKernelGGL((chirpz6k_persist_kernel<RB, true, 8>), pg, block, 0, s, in, out, n,
                         batch, rpw, tw, chirp, bhat, scale);
    else
      hipLaunchKernelGGL((chirpz6k_persist_kernel<RB, false, 8>), pg, block, 0, s, in, out, n,
                         batch, rpw, tw, chirp, bhat, scale);
    return hipGetLastError();
  }
#endif
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

hipError_t launch_chirpz6k(int64_t m, bool inv, int load, const void *in, cd *out, int64_t n,
                           int64_t batch, const cd *tw, const cd *chirp, const cd *bhat,
                           double scale, hipStream_t s) {
  if (chirpz6k_m(n) != m || batch < 0 || batch > 0x7fffffff || (inv && load == LOAD_REAL))
    return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  if (m == 6144) return launch_c6<24>(inv, load, in, out, n, batch, tw, chirp, bhat, scale, s);
  return launch_c6<12>(inv, load, in, out, n, batch, tw, chirp, bhat, scale, s);
}

}  // namespace gdsp
