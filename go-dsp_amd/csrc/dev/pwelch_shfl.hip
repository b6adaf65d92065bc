// pwelch_shfl.hip — fused Welch accumulation for NFFT = 4096, Noverlap = 2048,
// Pad = NFFT (the BASELINE configuration; spectral/pwelch.go:104-122) with a
// wavefront-shuffle exchange.
//
// Same scheme as pwelch_half_kernel (fft_kernels.hip): persistent workers over
// packed segment pairs z = w x_s + i w x_{s+1}, one sample load per sample (a
// carried half), |Z_k|^2 summed per bin in registers. The FFT-4096 differs: a
// decimation-in-frequency radix-16 x 3 whose digits are placed so that only
// ONE of its two exchanges crosses waves:
//   element e = D0 + 16 D1 + 256 D2; thread (wave w, lane l) holds D2 in its
//   16 registers, D0 = lane bits 2-5, D1 = lane bits 0-1 + 4 w (a wave's
//   sample loads still cover 64 consecutive doubles, permuted over lanes);
//   pass 1: DFT_16 over D2 -> K0, times W_4096^((D0 + 16 D1) K0);
//   exchange 1 (LDS, real then imaginary half): D1 into the registers, K0
//   into lane bits 0-1 + wave, D0 stays in lane bits 2-5;
//   pass 2: DFT_16 over D1 -> K1, times W_256^(D0 K1);
//   exchange 2 (inside the wave, no LDS, no barrier): register bits 0-3 (K1)
//   <-> lane bits 2-5 (D0), one bit at a time: lane bits 2 and 3 by DPP row
//   shifts whose bank mask keeps the lanes that stay (one v_mov_b32_dpp per
//   dword), lane bits 4 and 5 by v_permlane16_swap / v_permlane32_swap (one
//   per dword pair);
//   pass 3: DFT_16 over D0 -> K2; bin K = K0 + 16 K1 + 256 K2.
// Four workgroup barriers per pair instead of eight.
#include "dev.hpp"
#include "shfl.hpp"

namespace gdsp {

namespace {

constexpr int kPsN = 4096;
// exchange-1 slot of (D0, D1, K0): D1 stride 20 (>= 16 D0 values, = 4 mod 16:
// the 16-lane write groups cover d0 + 4 c), K0 stride 328 (>= 16 x 20, = 8
// mod 32: the 32-lane read groups cover d0 + 8 c); both conflict-free
__host__ __device__ __forceinline__ constexpr int ps_slot(int d0, int d1, int k0) {
  return k0 * 328 + d1 * 20 + d0;
}
constexpr int kPsXSlots = ps_slot(15, 15, 15) + 1;  // 5236 doubles
// window slot: bit 3 of i flipped where bit 5 is set (a permutation of each
// 64-slot block), so the reads at D0 + 16 D1 + 256 k are conflict-free within
// 32-lane groups
__host__ __device__ __forceinline__ constexpr int ps_wslot(int i) {
  return i ^ (((i >> 5) & 1) << 3);
}
constexpr int kPsWSlots = kPsN;

// u[r] *= w^r, r = 1..15: two interleaved power chains (as pass_compute)
__device__ __forceinline__ void twiddle16(cd (&u)[16], cd w) {
  u[1] = cmul(u[1], w);
  const cd w2 = cmul(w, w);
  cd wo = w, we = w2;
  u[2] = cmul(u[2], w2);
#pragma unroll
  for (int r = 3; r < 16; ++r) {
    if (r & 1) {
      wo = cmul(wo, w2);
      u[r] = cmul(u[r], wo);
    } else {
      we = cmul(we, w2);
      u[r] = cmul(u[r], we);
    }
  }
}

// register bits 0-3 <-> lane bits 2-5 (exchange 2): afterwards register r
// holds D0 = r and lane bits 2-5 hold the former register index
__device__ __forceinline__ void swap_reg_lane(cd (&v)[16]) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!(r & 1)) {
      dpp_swap<4>(v[r].x, v[r | 1].x);
      dpp_swap<4>(v[r].y, v[r | 1].y);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!(r & 2)) {
      dpp_swap<8>(v[r].x, v[r | 2].x);
      dpp_swap<8>(v[r].y, v[r | 2].y);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!(r & 4)) {
      perm_swap<true>(v[r].x, v[r | 4].x);
      perm_swap<true>(v[r].y, v[r | 4].y);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!(r & 8)) {
      perm_swap<false>(v[r].x, v[r | 8].x);
      perm_swap<false>(v[r].y, v[r | 8].y);
    }
  }
}

}  // namespace

__global__ __launch_bounds__(256) void pwelch4096_shfl_kernel(
    const double *__restrict__ x, int64_t seg_begin, int64_t seg_end, int64_t pairs_per_worker,
    const double *__restrict__ win, const cd *__restrict__ tw, double *__restrict__ partial) {
  constexpr int E = 16, H = 8, T = 256, N = kPsN;
  constexpr int64_t STRIDE = N / 2;
  __shared__ double lds[kPsXSlots + kPsWSlots + 2 * 256];
  double *lx = lds;                                             // exchange 1
  double *wl = lds + kPsXSlots;                                 // window
  cd *twl = reinterpret_cast<cd *>(lds + kPsXSlots + kPsWSlots);  // T_4096[0 .. 256)
  const int lt = threadIdx.x, lane = lt & 63, wv = lt >> 6;
  const int d0 = lane >> 2, d1 = (lane & 3) + 4 * wv;
  const int base = d0 + 16 * d1;  // this thread's elements: base + 256 k
  const int64_t worker = blockIdx.x;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  for (int i = lt; i < N; i += T) wl[ps_wslot(i)] = win[i];
  for (int i = lt; i < 256; i += T) twl[i] = tw[i];
  __syncthreads();
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  const int64_t p0 = worker * pairs_per_worker;
  // carried samples: the first half of the next pair's first segment
  double carry[H];
  {
    const int64_t s0 = seg_begin + 2 * (p0 < npairs ? p0 : 0);
    const double *b = x + s0 * STRIDE + base;
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = (p0 < npairs) ? b[k * T] : 0.0;
  }
  auto load_pair = [&](int64_t p, double (&a2)[H], double (&c2)[H]) {
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * p;
    const bool has1 = active && (s0 + 1 < seg_end);
    const double *b = opaque_ptr(x) + s0 * STRIDE + base;
#pragma unroll
    for (int k = 0; k < H; ++k) {
      a2[k] = active ? b[(H + k) * T] : 0.0;
      c2[k] = has1 ? b[(E + k) * T] : 0.0;
    }
  };
  double na2[H], nc2[H];  // the next pair's samples, in flight
  load_pair(p0, na2, nc2);
  // exchange-1 addresses: write (D0, D1, K0 = r), read (D0, D1 = r, K0 = d1)
  const int wbase = ps_slot(d0, d1, 0), rbase = ps_slot(d0, 0, d1);
  for (int64_t it = 0; it < pairs_per_worker; ++it) {
    const int64_t p = p0 + it;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * p;
    const bool has1 = active && (s0 + 1 < seg_end);
    double a2[H], c2[H];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      a2[k] = na2[k];
      c2[k] = nc2[k];
    }
    if (it + 1 < pairs_per_worker) load_pair(p + 1, na2, nc2);
    const int bo = opaque_int(base);
    cd v[E];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      const double w0 = wl[ps_wslot(bo + k * T)], w1 = wl[ps_wslot(bo + (H + k) * T)];
      // an unpaired last segment (odd count) has a zero partner
      v[k] = {carry[k] * w0, has1 ? a2[k] * w0 : 0.0};
      v[H + k] = {a2[k] * w1, c2[k] * w1};
    }
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = c2[k];
    // pass 1: DFT_16 over D2 -> K0, times W_4096^(base K0)
    Dft<16>::run(v);
    twiddle16(v, twl[bo]);
    // exchange 1 through LDS, real then imaginary half
    {
      const int wb = opaque_int(wbase), rb = opaque_int(rbase);
      if (it) __syncthreads();  // the previous pair's reads are done
#pragma unroll
      for (int r = 0; r < E; ++r) lx[wb + ps_slot(0, 0, r)] = v[r].x;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < E; ++r) v[r].x = lx[rb + ps_slot(0, r, 0)];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < E; ++r) lx[wb + ps_slot(0, 0, r)] = v[r].y;
      __syncthreads();
#pragma unroll
      for (int r = 0; r < E; ++r) v[r].y = lx[rb + ps_slot(0, r, 0)];
    }
    // pass 2: DFT_16 over D1 -> K1, times W_256^(D0 K1) = W_4096^(16 D0 K1)
    Dft<16>::run(v);
    twiddle16(v, twl[16 * (bo & 15)]);
    // exchange 2 inside the wave, then pass 3: DFT_16 over D0 -> K2
    swap_reg_lane(v);
    Dft<16>::run(v);
    if (active) {
#pragma unroll
      for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  }
  if (p0 < npairs) {
    // bin K0 + 16 K1 + 256 K2: K0 = d1, K1 = lane bits 2-5 (= d0), K2 = k
    double *dst = partial + worker * N + d1 + 16 * d0;
#pragma unroll
    for (int k = 0; k < E; ++k) dst[256 * k] = acc[k];
  }
}

hipError_t launch_pwelch4096_shfl(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                  int64_t nworkers, const double *win, const cd *tw,
                                  double *partial, hipStream_t s) {
  hipLaunchKernelGGL(pwelch4096_shfl_kernel, dim3((unsigned)nworkers), dim3(256), 0, s, x,
                     seg_begin, seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

}  // namespace gdsp
