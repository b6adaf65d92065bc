// pwelch_row3.hip — (development build) the NFFT 4096 / 50 % Pwelch row
// kernel (pwelch_row.hip; spectral/pwelch.go:104-122) reshaped for three
// workgroups per CU, the design VERDICT r04 asked to be built or ruled out:
//  - the next pair's 4096 new samples come in by LDS-DMA (buffer_load ... lds,
//    16 B per lane) into a 32 KiB stage while this pair's FFT runs, instead of
//    32 prefetch VGPRs; a partnerless last pair's descriptor ends after its
//    first segment, so the hardware zero-fills the partner;
//  - the two exchanges go through a half-size buffer (17 KiB): each component
//    in two rounds, the writers of round h being waves 2h and 2h + 1 (the
//    outputs of threads 128 h .. 128 h + 127 are exactly half h of the
//    transform in both exchanges), every thread reading its elements of that
//    half; the first round's reads go to 8 temporaries, since the second
//    round's writers still need their own values;
//  - the window is read from L1/L2 per pair (issued before the DMA, so its
//    wait does not drain the DMA: vmcnt is in order) instead of a 32 KiB table;
//  - every barrier is bare (s_waitcnt lgkmcnt(0) + s_barrier): a workgroup
//    fence would also wait for the DMA in flight (a pending LDS write).
// LDS 49 KiB, and amdgpu_waves_per_eu(3) caps the VGPRs at 168: three 4-wave
// workgroups per CU. Same carry, packing, twiddles (RegTw, recurrence) and
// |Z|^2 accumulation as pwelch_row_kernel<12>; gdsp_dev_pwelch4096_row3_
// accumulate runs it against the oracle.
#include "dev.hpp"

namespace gdsp {

namespace {
constexpr int kR3N = 4096, kR3T = 256, kR3E = 16, kR3H = 8;
constexpr int kR3Half = 8 * 272;  // half-buffer slots (LAYOUT 2 of one half)
constexpr int kR3Stage = 4096;    // staged samples (doubles)

__device__ __forceinline__ void bare_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One component of the exchange after pass (R = 16, NS) through the half
// buffer; c[k] holds element k of the thread's registers (pass output r = k).
// NS = 1: writes 16 t + (r ^ (t & 15)), reads (t ^ ((t >> 4) & 15)) + 256 k;
// NS = 16: writes (t / 16) 272 + t % 16 + 16 r, reads t + 272 k (LAYOUT 2).
template <int NS>
__device__ __forceinline__ void r3_part(double (&c)[kR3E], int t, double *buf) {
  const int h1 = t >= 128;  // this thread writes in round h1 (wave-uniform)
  double tmp[kR3H];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bare_sync();  // the previous reads of the buffer are done
    if (h1 == h) {
      const int tl = t - 128 * h;
#pragma unroll
      for (int r = 0; r < kR3E; ++r) {
        const int slot = NS == 1 ? 16 * tl + (r ^ (t & 15)) : (tl / 16) * 272 + (tl & 15) + 16 * r;
        buf[slot] = c[r];
      }
    }
    bare_sync();
#pragma unroll
    for (int k = 0; k < kR3H; ++k) {
      const int slot = NS == 1 ? (t ^ ((t >> 4) & 15)) + 256 * k : t + 272 * k;
      if (h == 0) tmp[k] = buf[slot];
      else c[kR3H + k] = buf[slot];
    }
  }
#pragma unroll
  for (int k = 0; k < kR3H; ++k) c[k] = tmp[k];
}

template <int NS>
__device__ __forceinline__ void r3_exchange(cd (&v)[kR3E], int t, double *buf) {
  double c[kR3E];
#pragma unroll
  for (int k = 0; k < kR3E; ++k) c[k] = v[k].x;
  r3_part<NS>(c, t, buf);
#pragma unroll
  for (int k = 0; k < kR3E; ++k) {
    v[k].x = c[k];
    c[k] = v[k].y;
  }
  r3_part<NS>(c, t, buf);
#pragma unroll
  for (int k = 0; k < kR3E; ++k) v[k].y = c[k];
}

// the 32 KiB of pair p's new samples (rows 8 .. 23 of the pair) into the
// stage: 32 wave-instructions of 1 KiB, 8 per wave
__device__ __forceinline__ void r3_dma(const double *x, int64_t seg_begin, int64_t p, bool partner,
                                       double *stage, int t) {
  const int64_t base = (seg_begin + 2 * p) * 2048 + 2048;
  const rsrc_t r = make_rsrc(x + base, (int64_t)(partner ? 4096 : 2048) * 8);
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t lane16 = (uint32_t)(t & 63) * 16u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int piece = w + 4 * i;  // 1 KiB piece
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r, (__attribute__((address_space(3))) void *)((char *)stage + piece * 1024), 16,
        (uint32_t)piece * 1024u + lane16, 0, 0, 0);  // (soffset is not range-checked)
  }
}
}  // namespace

// FOLD (register count only: tools/pwelch_fold_probe.hip,
// profiles/r06/pw4096_fold_resusage.txt): 8 folded |Z_k|^2 + |Z_F-k|^2 sums
// (+ thread 0's bin 2048) instead of 16, through the half buffer per pair, as
// pwelch_row_kernel's FOLD.
template <bool FOLD = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void pwelch_row3_kernel(
    const double *__restrict__ x, int64_t seg_begin, int64_t seg_end, int64_t pairs_per_worker,
    const double *__restrict__ win, const cd *__restrict__ tw, double *__restrict__ partial) {
  __shared__ double lds[kR3Half + kR3Stage];
  double *const buf = lds;
  double *const stage = lds + kR3Half;
  const int t = threadIdx.x;
  using RT = RegTw<3>;
  RT rtw;
  rtw.base[0] = {1.0, 0.0};
  rtw.base[1] = pass_base<kR3N, 16, 16>(tw, t);
  rtw.base[2] = pass_base<kR3N, 16, 256>(tw, t);
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t nfull = (seg_end - seg_begin) / 2;
  const int64_t p0 = (int64_t)blockIdx.x * pairs_per_worker;
  const int64_t pend = p0 + pairs_per_worker < npairs ? p0 + pairs_per_worker : npairs;
  if (p0 >= pend) return;  // whole workgroup (uniform)
  double carry[kR3H];
  {
    const double *b = x + (seg_begin + 2 * p0) * 2048 + t;
#pragma unroll
    for (int k = 0; k < kR3H; ++k) carry[k] = b[k * kR3T];
  }
  r3_dma(x, seg_begin, p0, p0 < nfull, stage, t);
  constexpr int NACC = FOLD ? kR3H + 1 : kR3E;
  double acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = 0.0;
  for (int64_t p = p0; p < pend; ++p) {
    const int tt = opaque_int(t);
    const double *wp = opaque_ptr(win);
    double wv[kR3E];
#pragma unroll
    for (int k = 0; k < kR3E; ++k) wv[k] = wp[tt + k * kR3T];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this pair's DMA (and the window) landed
    bare_sync();
    double a2[kR3H], c2[kR3H];
#pragma unroll
    for (int k = 0; k < kR3H; ++k) {
      a2[k] = stage[k * kR3T + tt];
      c2[k] = stage[(kR3H + k) * kR3T + tt];
    }
    bare_sync();  // every thread has read the stage
    if (p + 1 < pend) r3_dma(x, seg_begin, p + 1, p + 1 < nfull, stage, tt);
    const bool partner = p < nfull;  // (else the second segment is zeros: c2 by the descriptor)
    cd v[kR3E];
#pragma unroll
    for (int k = 0; k < kR3H; ++k) {
      v[k] = {carry[k] * wv[k], partner ? a2[k] * wv[k] : 0.0};
      v[kR3H + k] = {a2[k] * wv[kR3H + k], c2[k] * wv[kR3H + k]};
      carry[k] = c2[k];
    }
    RT rl = rtw;
    rl.base[1] = opaque_cd(rl.base[1]);
    rl.base[2] = opaque_cd(rl.base[2]);
    pass_compute<kR3N, kR3E, kR3T, 16, 1, 0, NoEpi, false, 0, RT, true>(v, tt, rl);
    r3_exchange<1>(v, tt, buf);
    pass_compute<kR3N, kR3E, kR3T, 16, 16, 0, NoEpi, false, 1, RT, true>(v, tt, rl);
    r3_exchange<16>(v, tt, buf);
    pass_compute<kR3N, kR3E, kR3T, 16, 256, 0, NoEpi, false, 2, RT, true>(v, tt, rl);
    if constexpr (FOLD) {
      double pw[kR3E];
#pragma unroll
      for (int k = 0; k < kR3E; ++k) pw[k] = fma(v[k].y, v[k].y, v[k].x * v[k].x);
      bare_sync();  // the last exchange's reads are done
#pragma unroll
      for (int k = kR3H; k < kR3E; ++k) buf[tt * kR3H + (k - kR3H)] = pw[k];
      bare_sync();
      if (tt == 0) {
        acc[0] += pw[0];
#pragma unroll
        for (int m = 1; m < kR3H; ++m) acc[m] += pw[m] + buf[kR3H - m];
        acc[kR3H] += buf[0];
      } else {
        const int tp = kR3T - tt;
#pragma unroll
        for (int m = 0; m < kR3H; ++m) acc[m] += pw[m] + buf[tp * kR3H + (kR3H - 1 - m)];
      }
    } else {
#pragma unroll
      for (int k = 0; k < kR3E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  }
  double *dst = partial + blockIdx.x * (int64_t)kR3N;
#pragma unroll
  for (int k = 0; k < kR3E; ++k) {
    if constexpr (FOLD)
      dst[t + k * kR3T] = k < kR3H ? acc[k] : (t == 0 && k == kR3H ? acc[kR3H] : 0.0);
    else
      dst[t + k * kR3T] = acc[k];
  }
}

hipError_t launch_pwelch4096_row3(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                  int64_t nworkers, const double *win, const cd *tw,
                                  double *partial, hipStream_t s) {
  hipLaunchKernelGGL(pwelch_row3_kernel<false>, dim3((unsigned)nworkers), dim3(256), 0, s, x, seg_begin,
                     seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

}  // namespace gdsp
