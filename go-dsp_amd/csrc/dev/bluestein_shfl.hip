// bluestein_shfl.hip — fused chirp-z for M = 8192 (fft/bluestein.go:68-94 with
// Convolve, fft/fft.go:55-69; 2049 <= n <= 4096 at the reference's M) whose
// two FFTs each keep one of their two exchanges inside the wave.
//
// Same work as bluestein_kernel<13, E = 32> (fft_kernels.hip): 256 threads,
// 32 complex128 per thread, radices 32 * 32 * 8, premultiply, FFT, x bhat,
// IFFT as conj(FFT(conj .)), postmultiply. The FFTs differ:
//   element e = D0 + 8 D1 + 256 D2: thread (wave w, lane l) holds D2 in its 32
//   registers, D0 = lane bits 3-5, D1 = lane bits 0-2 + 8 w (a wave's loads
//   still cover 64 consecutive elements, permuted over lanes);
//   FFT 1, decimation in frequency (natural order in, K = K0 + 32 K1 + 1024 K2
//   out): P1 DFT_32 over D2 -> K0, T1 x W_8192^((D0 + 8 D1) K0), X1 (LDS:
//   D1 into the registers, K0 into lane bits 0-2 + wave), P2 DFT_32 over
//   D1 -> K1, T2 x W_256^(D0 K1), X2 (inside the wave: register bits 0-2 <->
//   lane bits 3-5, by a DPP row shift and v_permlane16/32_swap), P3 DFT_8
//   over D0 -> K2;
//   x conj(bhat) in that order (bhat permuted at plan time);
//   FFT 2 is the transpose of FFT 1 (every pass and twiddle is symmetric,
//   the exchanges are involutions): P3, X2, T2, P2, X1 back, T1, P1, so it
//   takes the digit order FFT 1 leaves and returns natural order.
// Two LDS exchanges and eight workgroup barriers per transform instead of
// four and sixteen. Measured slower (chirp-z 3000: 3.53 against 3.32 ms; the
// DPP and permlane moves take VALU issue slots the block kernel spends on
// nothing); the development build runs it through gdsp_dev_fft_batch_chirpz_shfl.
#include "dev.hpp"
#include "shfl.hpp"

namespace gdsp {

namespace {

constexpr int kBsM = 8192, kBsT = 256;
// exchange slot of (D0, D1, K0): D0 stride 1064 (= 8 mod 16 and 8 mod 32),
// D1 stride 33, K0 stride 1: the writes (16-lane groups: 8 D0 + lane bits
// 0-2) and the reads (32-lane groups: 8 D0 + lane bits 0-2) are
// conflict-free in both directions
__host__ __device__ constexpr int bs_slot(int d0, int d1, int k0) {
  return d0 * 1064 + d1 * 33 + k0;
}
constexpr int kBsSlots = bs_slot(7, 31, 31) + 1;  // 8503 doubles

// u[r] *= w^r, r = 1..31: two interleaved power chains (as pass_compute)
__device__ __forceinline__ void twiddle32(cd (&u)[32], cd w) {
  u[1] = cmul(u[1], w);
  const cd w2 = cmul(w, w);
  cd wo = w, we = w2;
  u[2] = cmul(u[2], w2);
#pragma unroll
  for (int r = 3; r < 32; ++r) {
    if (r & 1) {
      wo = cmul(wo, w2);
      u[r] = cmul(u[r], wo);
    } else {
      we = cmul(we, w2);
      u[r] = cmul(u[r], we);
    }
  }
}

// keeps the scheduler from interleaving neighbouring stages (register pressure)
__device__ __forceinline__ void stage_fence() { __builtin_amdgcn_sched_barrier(0); }

// X2: register bits 0-2 <-> lane bits 3-5
__device__ __forceinline__ void swap_x2(cd (&v)[32]) {
#pragma unroll
  for (int r = 0; r < 32; ++r)
    if (!(r & 1)) {
      dpp_swap<8>(v[r].x, v[r | 1].x);
      dpp_swap<8>(v[r].y, v[r | 1].y);
    }
#pragma unroll
  for (int r = 0; r < 32; ++r)
    if (!(r & 2)) {
      perm_swap<true>(v[r].x, v[r | 2].x);
      perm_swap<true>(v[r].y, v[r | 2].y);
    }
#pragma unroll
  for (int r = 0; r < 32; ++r)
    if (!(r & 4)) {
      perm_swap<false>(v[r].x, v[r | 4].x);
      perm_swap<false>(v[r].y, v[r | 4].y);
    }
}

// P3: DFT_8 over register bits 0-2, four groups
__device__ __forceinline__ void dft8x4(cd (&v)[32]) {
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    cd u[8];
#pragma unroll
    for (int d = 0; d < 8; ++d) u[d] = v[8 * h + d];
    Dft<8>::run(u);
#pragma unroll
    for (int d = 0; d < 8; ++d) v[8 * h + d] = u[d];
  }
}

// X1 through LDS (real then imaginary half): write at wr + the register's
// offset, read at rd + the register's offset. Forward: (wr, WS, rd, RS) =
// (slot(D0, m, 0), 1, slot(D0, 0, m), 33); back: the two swapped.
template <int WS, int RS>
__device__ __forceinline__ void exchange_x1(cd (&v)[32], double *lx, int wr, int rd, bool first) {
  if (!first) __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) lx[wr + WS * r] = v[r].x;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) v[r].x = lx[rd + RS * r];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) lx[wr + WS * r] = v[r].y;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 32; ++r) v[r].y = lx[rd + RS * r];
}

}  // namespace

// bhatp[r * 256 + t] = bhat[K(t, r)] / (the 1/M of the IFFT is in bhat),
// K = K0 + 32 K1 + 1024 K2 with K0 = lane bits 0-2 + 8 w, K1 = lane bits 3-5
// + 8 (r >> 3), K2 = r & 7 (gdsp_api.hip builds it).
template <bool INV>
__global__ __launch_bounds__(256, 2) void bluestein_shfl_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ twm, const cd *__restrict__ chirp, const cd *__restrict__ bhatp,
    double scale) {
  __shared__ double lx[kBsSlots];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int d0 = lane >> 3, m = (lane & 7) + 8 * w;
  const int base = d0 + 8 * m;  // this thread's elements: base + 256 k
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x);
  const bool valid = g < batch;
  const int xw = bs_slot(d0, m, 0), xr = bs_slot(d0, 0, m);
  cd v[32];
  {
    const cd *src = in + (valid ? g : 0) * n;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int e = base + kBsT * k;
      v[k] = {0.0, 0.0};
      if (k < 16 && valid && e < n) {  // n <= 4096: registers 16..31 stay zero
        cd x = ld_nt(&src[e]);
        if constexpr (INV) x.y = -x.y;
        v[k] = cmul(x, chirp[e]);
      }
    }
  }
  // FFT 1 (decimation in frequency)
  {
    const cd *tw = opaque_ptr(twm);
    const int b = opaque_int(base), dd = opaque_int(d0);
    Dft<32>::run(v);                 // P1
    stage_fence();
    twiddle32(v, tw[b]);             // T1: W_8192^(base K0)
    stage_fence();
    exchange_x1<1, 33>(v, lx, opaque_int(xw), opaque_int(xr), true);
    stage_fence();
    Dft<32>::run(v);                 // P2
    stage_fence();
    twiddle32(v, tw[32 * dd]);       // T2: W_256^(D0 K1)
    stage_fence();
    swap_x2(v);                      // X2
    stage_fence();
    dft8x4(v);                       // P3
    stage_fence();
  }
  {
    const cd *bh = opaque_ptr(bhatp) + opaque_int(t);
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = conjg(cmul(v[r], bh[kBsT * r]));
    stage_fence();
  }
  // FFT 2: the transpose of FFT 1
  {
    const cd *tw = opaque_ptr(twm);
    const int b = opaque_int(base), dd = opaque_int(d0);
    dft8x4(v);                       // P3
    stage_fence();
    swap_x2(v);                      // X2
    stage_fence();
    twiddle32(v, tw[32 * dd]);       // T2
    stage_fence();
    Dft<32>::run(v);                 // P2
    stage_fence();
    exchange_x1<33, 1>(v, lx, opaque_int(xr), opaque_int(xw), false);
    stage_fence();
    twiddle32(v, tw[b]);             // T1
    stage_fence();
    Dft<32>::run(v);                 // P1
    stage_fence();
  }
  if (valid) {
    const cd *ch = opaque_ptr(chirp);
    const int b = opaque_int(base);
    cd *dst = out + g * n;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = b + kBsT * k;
      if (e < n) {
        cd y = cmul(conjg(v[k]), ch[e]);
        if constexpr (INV) y = {y.x * scale, -y.y * scale};
        st_nt(&dst[e], y);
      }
    }
  }
}

// bin of (thread t, register r) after FFT 1 (see the kernel)
int bluestein_shfl_bin(int t, int r) {
  const int lane = t & 63, w = t >> 6;
  return ((lane & 7) + 8 * w) + 32 * ((lane >> 3) + 8 * (r >> 3)) + 1024 * (r & 7);
}

hipError_t launch_bluestein_shfl(bool inv, const cd *in, cd *out, int64_t n, int64_t batch,
                                 const cd *twm, const cd *chirp, const cd *bhatp, double scale,
                                 hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  if (n > kBsM / 2) return hipErrorInvalidValue;
  if (inv)
    hipLaunchKernelGGL(bluestein_shfl_kernel<true>, dim3((unsigned)batch), dim3(kBsT), 0, s, in,
                       out, n, batch, twm, chirp, bhatp, scale);
  else
    hipLaunchKernelGGL(bluestein_shfl_kernel<false>, dim3((unsigned)batch), dim3(kBsT), 0, s, in,
                       out, n, batch, twm, chirp, bhatp, scale);
  return hipGetLastError();
}

}  // namespace gdsp
