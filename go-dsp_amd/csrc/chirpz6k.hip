// chirpz6k.hip — fused chirp-z (Bluestein, fft/bluestein.go:68-94) on the
// convolution length M = 6144 = 16 * 24 * 16 for 2049 <= n <= 3072.
//
// bluestein.go:70 pads the circular convolution to NextPowerOf2(2n - 1) =
// 8192 for these n because its FFT is radix 2. Any M >= 2n - 1 gives the
// same linear convolution, hence the same DFT; 6144 = 3 * 2^11 is a quarter
// fewer points, and its exchange buffer (6144 doubles, 48 KiB) and a
// 16-point-per-thread register set let two 384-thread workgroups share a CU
// at three waves per SIMD, where the M = 8192 kernel (bluestein_kernel<13>,
// 32 points per thread, 256 VGPRs) runs two.
//
// One workgroup per transform, 384 threads (thread t):
//   premultiply  a[t + 384 r] = x * conj(w), r < KN (n <= 384 KN; rest zero)
//   FFT 1        pass A  R = 16, NS = 1:   DFT_16 of t + 384 r (pruned input)
//                pass B  R = 24, NS = 16:  t < 256, inputs t + 256 r
//                pass C  R = 16, NS = 384: outputs t + 384 r (natural order)
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

namespace gdsp {

// (kernel and helpers outside an anonymous namespace, so profiler kernel
// names read gdsp::chirpz6k_kernel<...>)
constexpr int kC6M = 6144, kC6T = 384, kC6B = 256;  // points, threads, pass-B butterflies

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

// DFT_24 = DFT_8 over n1 (n = 3 n1 + n2), twiddles W_24^(n2 k1), DFT_3 over
// n2 (k = k1 + 8 k2)
__device__ __forceinline__ void dft24(cd (&a)[24]) {
  cd y[3][8];
#pragma unroll
  for (int n2 = 0; n2 < 3; ++n2) {
    cd tmp[8];
#pragma unroll
    for (int n1 = 0; n1 < 8; ++n1) tmp[n1] = a[3 * n1 + n2];
    Dft<8>::run(tmp);
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) y[n2][k1] = tmp[k1];
  }
#pragma unroll
  for (int k1 = 0; k1 < 8; ++k1) {
    const cd a0 = y[0][k1], a1 = rot24(y[1][k1], k1), a2 = rot24(y[2][k1], 2 * k1);
    // DFT_3: X1 = a0 - (a1 + a2)/2 - i sin(2 pi/3) (a1 - a2), X2 its mirror
    const cd s = a1 + a2, d = a1 - a2;
    const cd m = {fma(-0.5, s.x, a0.x), fma(-0.5, s.y, a0.y)};
    a[k1] = a0 + s;
    a[k1 + 8] = {fma(GDSP_C12, d.y, m.x), fma(-GDSP_C12, d.x, m.y)};
    a[k1 + 16] = {fma(-GDSP_C12, d.y, m.x), fma(GDSP_C12, d.x, m.y)};
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
struct C6Bhat {
  rsrc_t rb;
  uint32_t off;
  cd f[16];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < 16; ++r) f[r] = buf_ld(rb, off + (uint32_t)(r * kC6T * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = conjg(cmul(v[r], f[r]));
  }
};
template <int KN, bool INV>
struct C6Out {
  rsrc_t rch, rout;
  uint32_t off;
  double scale;
  cd f[KN];
  __device__ __forceinline__ void issue() {
#pragma unroll
    for (int r = 0; r < KN; ++r) f[r] = buf_ld(rch, off + (uint32_t)(r * kC6T * 16));
  }
  __device__ __forceinline__ void apply(cd (&v)[16]) const {
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      cd y = cmul(conjg(v[r]), f[r]);
      if constexpr (INV) y = {y.x * scale, -y.y * scale};
      buf_st_nt(rout, off + (uint32_t)(r * kC6T * 16), y);
    }
  }
};

// One FFT_6144 of the thread's registers v[r] = element t + 384 r, in place
// (natural order in and out), then epi. ZIN: inputs r >= ZIN are zero (pass
// A pruned); first: no exchange precedes this one in the kernel. tw: the pass
// twiddle bases, W_384^k (k < 16, pass B) then W_6144^k (k < 384, pass C).
template <int ZIN, class EPI>
__device__ __forceinline__ void c6_fft(cd (&v)[16], int t, const cd *__restrict__ tw, double *lds,
                                       bool first, EPI &epi) {
  // (the twiddle bases are read where they are used: read a pass ahead,
  // 3.2-3.3 against 2.37 ms)
  // pass A
  if constexpr (ZIN > 0 && ZIN <= 8) dft_half_in<16, ZIN>(v);
  else Dft<16>::run(v);
  // exchange 1: write 16 t + r, read t + 256 r (t < 256)
  const bool pb = t < kC6B;
  const int wa = 16 * t, ma = t & 15;
  const int ra = t ^ ((t >> 4) & 15);
  cd u[24];
  if (!first) __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].x;
  __syncthreads();
  if (pb) {
#pragma unroll
    for (int r = 0; r < 24; ++r) u[r].x = lds[ra + kC6B * r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) lds[wa + (r ^ ma)] = v[r].y;
  __syncthreads();
  // pass B (waves 0-3; waves 4-5 only take part in the barriers)
  const int wbo = (t >> 4) * 384 + (t & 15);
  if (pb) {
#pragma unroll
    for (int r = 0; r < 24; ++r) u[r].y = lds[ra + kC6B * r];
    c6_twiddle<24>(u, tw[t & 15]);
    dft24(u);
  }
  __syncthreads();
  // exchange 2: write (t / 16) 384 + t % 16 + 16 r, read t + 384 r
  if (pb) {
#pragma unroll
    for (int r = 0; r < 24; ++r) lds[wbo + 16 * r] = u[r].x;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r].x = lds[t + kC6T * r];
  __syncthreads();
  if (pb) {
#pragma unroll
    for (int r = 0; r < 24; ++r) lds[wbo + 16 * r] = u[r].y;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r].y = lds[t + kC6T * r];
  // pass C: twiddle W_6144^(t r), DFT_16, the epilogue
  c6_twiddle<16>(v, tw[16 + t]);
  Dft<16>::run(v);
  epi.issue();
  epi.apply(v);
}

// Two workgroups of 6 waves share a CU. Held to 128 VGPRs (4 waves per SIMD
// of room): at 144 (3 per SIMD) the second workgroup's waves did not fit
// beside the first's 2-2-1-1 placement and the kernel ran 3.13 against
// 2.43 ms (profiles/r03/chirpz6k_ab.txt)
// KN: n <= 384 KN (inputs and wanted outputs at r < KN)
// REAL: float64 input rows (fft.FFTReal, fft/fft.go:25-27), read directly
// (no complex copy of the input first)
template <bool INV, int KN, bool REAL = false>
__global__ __launch_bounds__(kC6T) __attribute__((amdgpu_waves_per_eu(4))) void chirpz6k_kernel(
    const void *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ tw, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale) {
  static_assert(KN >= 1 && KN <= 8, "n <= M/2");
  __shared__ double lds[kC6M];
  const int t = (int)threadIdx.x;
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  if (g >= batch) return;  // (grid = batch: never taken)
  const uint32_t off = (uint32_t)t * 16u;
  const int64_t rowb = n * 16;
  const rsrc_t rin =
      REAL ? make_rsrc(static_cast<const double *>(in) + g * n, n * 8)
           : make_rsrc(static_cast<const cd *>(in) + g * n, rowb);
  const rsrc_t rch = make_rsrc(chirp, rowb);
  cd v[16];
  {
    cd xv[KN], cv[KN];
#pragma unroll
    for (int r = 0; r < KN; ++r) {
      if constexpr (REAL)
        xv[r] = {buf_ld1(rin, (uint32_t)t * 8u + (uint32_t)(r * kC6T * 8)), 0.0};
      else
        xv[r] = buf_ld(rin, off + (uint32_t)(r * kC6T * 16));
      cv[r] = buf_ld(rch, off + (uint32_t)(r * kC6T * 16));
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
  C6Bhat be{make_rsrc(bhat, (int64_t)kC6M * 16), off, {}};
  c6_fft<KN>(v, t, tw, lds, true, be);
  // the second FFT must not share the first one's addresses (opaque copies:
  // otherwise the compiler keeps them live across both)
  const int t2 = opaque_int(t);
  C6Out<KN, INV> oe{make_rsrc(opaque_ptr(chirp), rowb), make_rsrc(out + g * n, rowb),
                    (uint32_t)t2 * 16u, scale, {}};
  c6_fft<0>(v, t2, opaque_ptr(tw), lds, false, oe);
}

bool chirpz6k_fits(int64_t n) { return n >= 2049 && 2 * n - 1 <= kC6M; }

hipError_t launch_chirpz6k(bool inv, int load, const void *in, cd *out, int64_t n, int64_t batch,
                           const cd *tw, const cd *chirp, const cd *bhat, double scale,
                           hipStream_t s) {
  if (!chirpz6k_fits(n) || batch < 0 || batch > 0x7fffffff || (inv && load == LOAD_REAL))
    return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  const dim3 grid((unsigned)batch), block(kC6T);
  if (load == LOAD_REAL)
    hipLaunchKernelGGL((chirpz6k_kernel<false, 8, true>), grid, block, 0, s, in, out, n, batch,
                       tw, chirp, bhat, scale);
  else if (inv)
    hipLaunchKernelGGL((chirpz6k_kernel<true, 8>), grid, block, 0, s, in, out, n, batch, tw, chirp,
                       bhat, scale);
  else
    hipLaunchKernelGGL((chirpz6k_kernel<false, 8>), grid, block, 0, s, in, out, n, batch, tw,
                       chirp, bhat, scale);
  return hipGetLastError();
}

}  // namespace gdsp
