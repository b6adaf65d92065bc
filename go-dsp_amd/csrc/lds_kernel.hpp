// lds_kernel.hpp — the one-kernel power-of-2 transform (fft_lds_kernel,
// fft/radix2.go:80-154) and its launch templates, shared by fft_kernels.hip
// and fft_lds12.hip (the N = 4096 instantiation in its own translation unit).
#pragma once
#include "fft_device.hpp"
#include "launch.hpp"

namespace gdsp {

// ----------------------------------------------------------------------------
// One-kernel transform: each workgroup owns TPW whole transforms in registers
// (16 complex128 per thread) and LDS (exchange between radix-16 passes).
// N >= 8192: 512+ threads per transform, so <= 128 VGPRs is what lets two
// workgroups share a CU (measured 1.27 -> 1.21 ms on the FFT2 8192^2 step).
// Short transforms (fewer than 16 threads per transform, N <= 128): a
// wave-instruction of the register layout t + k*T would touch 64 / T rows in
// runs of only T*16 bytes, so the workgroup's TPW*N contiguous elements are
// staged through LDS instead: coalesced 16-B-per-lane HBM streams on both
// sides, real and imaginary halves in turn through one padded buffer
// (slot = i + i/E keeps the stride-E reads conflict-free). N = 8 went from
// 1.5 to ~6 TB/s.
template <int LOG2N>
struct Stage {
  using G = Geo<LOG2N>;
  static constexpr bool ON = G::T < 16 && G::TPW > 1;
  static constexpr int DOUBLES = ON ? G::WG * (G::E + 1) : 1;
  __device__ __forceinline__ static int pad(int i) { return i + i / G::E; }
};

template <int LOG2N, bool INV, int LOAD, bool SPLIT, int LOG2E = 4>
__global__ __launch_bounds__((Geo<LOG2N, LOG2E>::WG),
                             (LOG2N >= 13 && SPLIT ? (LOG2E == 4 ? 4 : 2) : 1)) void
fft_lds_kernel(const void *__restrict__ in, cd *__restrict__ out, int64_t batch,
               const cd *__restrict__ tw, double scale) {
  using G = Geo<LOG2N, LOG2E>;
  using S = Stage<LOG2N>;
  constexpr int XD = (SPLIT ? 1 : 2) * G::LDS_DOUBLES;
  __shared__ double lds[XD > S::DOUBLES ? XD : S::DOUBLES];
  const int lt = threadIdx.x;
  const int slot = lt / G::T;
  const int t = lt & (G::T - 1);
  const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t g = blk * G::TPW + slot;
  // Only the last workgroup can hold slots past the batch (TPW > 1); they
  // load a valid row (clamped) and skip the store, so loads stay
  // branch-free and the whole workgroup reaches every barrier.
  const bool valid = G::TPW == 1 || g < batch;
  const int64_t gl = G::TPW == 1 ? g : (g < batch ? g : batch - 1);
  double *lre = lds + slot * G::STRIDE;
  double *lim = SPLIT ? lre : lds + G::LDS_DOUBLES + slot * G::STRIDE;
  cd v[G::E];
  if constexpr (S::ON) {
    // element i of the block's chunk is row blk*TPW + i/N, column i%N;
    // thread (slot, t) owns chunk elements slot*N + t + k*T
    const int64_t base = blk * G::TPW * G::N, total = batch * G::N;
    double tmp[2][G::E];
#pragma unroll
    for (int q = 0; q < G::E; ++q) {
      const int64_t idx = base + lt + q * G::WG;
      cd x = {0.0, 0.0};
      if (idx < total) {
        if constexpr (LOAD == LOAD_COMPLEX) x = ld_nt(reinterpret_cast<const cd *>(in) + idx);
        else x = {ld_nt(reinterpret_cast<const double *>(in) + idx), 0.0};
      }
      tmp[0][q] = x.x;
      tmp[1][q] = INV ? -x.y : x.y;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (LOAD == LOAD_REAL && h == 1) {
#pragma unroll
        for (int k = 0; k < G::E; ++k) v[k].y = 0.0;
        break;
      }
      if (h) __syncthreads();
#pragma unroll
      for (int q = 0; q < G::E; ++q) lds[S::pad(lt + q * G::WG)] = tmp[h][q];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < G::E; ++k) {
        const double d = lds[S::pad(slot * G::N + t + k * G::T)];
        if (h) v[k].y = d;
        else v[k].x = d;
      }
    }
    __syncthreads();  // the exchanges below reuse the buffer
  } else if constexpr (LOAD == LOAD_COMPLEX) {
    const cd *src = reinterpret_cast<const cd *>(in) + gl * G::N;
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
      v[k] = ld_nt(&src[t + k * G::T]);
      if constexpr (INV) v[k].y = -v[k].y;
    }
  } else {
    const double *src = reinterpret_cast<const double *>(in) + gl * G::N;
#pragma unroll
    for (int k = 0; k < G::E; ++k) v[k] = {ld_nt(&src[t + k * G::T]), 0.0};
  }
  fft_regs<LOG2N, SPLIT, 0, LOG2E>(v, t, tw, lre, lim, true);
  if constexpr (S::ON) {
    const int64_t base = blk * G::TPW * G::N, total = batch * G::N;
    double tmp[2][G::E];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // the last exchange's (or the previous half's) reads are done
#pragma unroll
      for (int k = 0; k < G::E; ++k) {
        double o = h ? v[k].y : v[k].x;
        if constexpr (INV) o = h ? -o * scale : o * scale;
        lds[S::pad(slot * G::N + t + k * G::T)] = o;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < G::E; ++q) tmp[h][q] = lds[S::pad(lt + q * G::WG)];
    }
#pragma unroll
    for (int q = 0; q < G::E; ++q) {
      const int64_t idx = base + lt + q * G::WG;
      if (idx < total) st_nt(out + idx, cd{tmp[0][q], tmp[1][q]});
    }
  } else if (valid) {
    cd *dst = out + g * G::N;
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
      cd o = v[k];
      if constexpr (INV) o = {o.x * scale, -o.y * scale};
      st_nt(&dst[t + k * G::T], o);
    }
  }
}

// ============================================================================
// Launch templates
// ============================================================================
template <int LOG2N, bool INV, int LOAD, bool SPLIT>
inline hipError_t launch_lds_t(const void *in, cd *out, int64_t batch, const cd *tw,
                               double scale, hipStream_t s) {
  // N = 16384: one 139 KiB workgroup per CU either way; 32 points per thread
  // (512 threads, three passes) 0.918-0.930 against 0.966-0.969 ms per 2^27
  // samples for 16 (1024 threads, four passes), alternating runs
  if constexpr (LOG2N == 14) {
    using G5 = Geo<LOG2N, 5>;
    const int64_t nb5 = (batch + G5::TPW - 1) / G5::TPW;
    hipLaunchKernelGGL((fft_lds_kernel<LOG2N, INV, LOAD, SPLIT, 5>), dim3((unsigned)nb5),
                       dim3(G5::WG), 0, s, in, out, batch, tw, scale);
    return hipGetLastError();
  }
  using G = Geo<LOG2N>;
  const int64_t nblk = (batch + G::TPW - 1) / G::TPW;
  hipLaunchKernelGGL((fft_lds_kernel<LOG2N, INV, LOAD, SPLIT>), dim3((unsigned)nblk),
                     dim3(G::WG), 0, s, in, out, batch, tw, scale);
  return hipGetLastError();
}

template <int LOG2N, bool INV, int LOAD>
inline hipError_t launch_lds_s(const void *in, cd *out, int64_t batch, const cd *tw,
                               double scale, bool split, hipStream_t s) {
  // the two-buffer exchange is only instantiated where it still fits LDS
  if constexpr (LOG2N <= 13) {
    if (!split) return launch_lds_t<LOG2N, INV, LOAD, false>(in, out, batch, tw, scale, s);
  }
  return launch_lds_t<LOG2N, INV, LOAD, true>(in, out, batch, tw, scale, s);
}

}  // namespace gdsp
