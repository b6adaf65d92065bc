// pwelch_row.hip — the fused Pwelch kernel of the BASELINE configuration
// (NFFT 4096, Noverlap 2048, Pad = NFFT; spectral/pwelch.go:104-122). Its own
// translation unit so it can be compiled with the max-ILP scheduler
// (Makefile): 2.81 against 2.85-2.89 ms with the default scheduler, at the
// same 246-248 VGPRs (the other kernels keep the default: the chirp-z kernel
// would lose a wave per SIMD to it).
#include "fft_device.hpp"
#include "launch.hpp"

namespace gdsp {

// Half-overlap Pwelch with one worker per workgroup (TPW = 1: F >= 4096, the
// BASELINE configuration). Same packing, carry and accumulation as
// pwelch_half_kernel, arranged so that the loop's bookkeeping costs no
// vector instructions:
//  - the worker's pair range, segment offsets and the has-partner test are
//    wave-uniform (scalar registers and branches); the loop runs over the
//    worker's own pairs only, full pairs first, then at most one pair whose
//    second segment does not exist (odd count: zero partner, its own body);
//  - each sample row is a scalar base pointer plus the lane's 32-bit offset
//    (global_load saddr: no 64-bit address arithmetic per load);
//  - the next pair's samples are loaded into the registers this pair's
//    samples just left (copied into the transform's registers), so they are
//    in flight during the FFT with no double buffer to copy between;
//  - each pass's twiddle base (the same for every pair) is read once per
//    kernel into registers (no LDS table, no bank conflicts on it); pass 1's
//    powers from an LDS table instead of each pair's chain measured slower
//    (2.99-3.01 against 2.86-2.87 ms: LDS, not the vector unit, is the
//    scarcer resource here);
//  - the twiddle powers of both twiddled passes by the three-term recurrence
//    (pass_compute CHEB: two FMAs per power instead of a complex product):
//    2.70-2.72 against 2.75-2.82 ms, parity 1.58e-15 against 1.16e-15;
//  - LAYOUT 2 exchange slots (fft_device.hpp): every LDS address a per-thread
//    base plus a compile-time offset (2.81-2.84 against 2.94-2.97 ms with
//    XOR-swizzled slots throughout).
// (Measured and not kept: the exchange through two unpadded buffers, real
// and imaginary parts at once with two barriers per exchange instead of
// four, and half the (symmetric) window in LDS to keep 80 KiB and two
// workgroups per CU: 3.10-3.17 against 2.83 ms.)
// Also measured and not kept: E = 8 (4 passes of radix 8, 512 threads,
// 116 VGPRs, four waves per SIMD; XOR exchange slots, table twiddles):
// 3.18-3.29 against 2.76 ms; re-measured in round 4 on this kernel, 3.17-3.18
// against 2.61 ms (profiles/r04/pwelch_rowx_ab.txt). And the window folded into pass 0's first radix-2
// stage as FMAs (w_j z_j +- w_(j+8) z_(j+8): 16 fewer FP64 instructions per
// thread and pair), 2.92 against 2.74 ms — the weights stay live in 32 more
// registers through the first DFT.
// And for a third wave per SIMD (scripts/archive/gpu_r03_occ.sh): the exchange through
// a buffer of half a transform (each component in two rounds, 17 KiB: three
// workgroups per CU by LDS) with the VGPRs capped at 168 spills 106-186
// registers, 5.95 ms without the next pair's samples in flight (touching its
// lines one pair ahead instead), 10.4 with them; without them at two waves,
// 3.02 against 2.73-2.77 ms.
//
// FOLD (measured by register count only, tools/
// pwelch_fold_probe.hip, profiles/r06/pw4096_fold_resusage.txt): finalise
// uses only acc[k] + acc[F - k], and the partner of the thread's bin
// k = t + T m is bin F - k = (T - t) + T (E - 1 - m) of thread T - t, so after
// each pair's last pass a thread hands its upper-half |Z|^2 to its partner
// through LDS and keeps E / 2 folded sums (+ one for the self-mirrored bin
// F / 2 of thread 0), 14 fewer VGPRs, at 8 LDS writes, 8 reads and a barrier
// per pair. Not instantiated in the library: it does not reach three waves
// per SIMD.
template <int LOG2F, int LOG2E = 4, bool REGTW = true, int LAYOUT = 2, bool FOLD = false>
__global__ __launch_bounds__((Geo<LOG2F, LOG2E>::WG)) void pwelch_row_kernel(
    const double *__restrict__ x, int64_t seg_begin, int64_t seg_end, int64_t pairs_per_worker,
    const double *__restrict__ win, const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F, LOG2E>;
  static_assert(G::TPW == 1, "one worker per workgroup");
  static_assert(!REGTW || (G::E == G::EMAX && G::NPE == G::NPASS && G::NPASS <= 4),
                "register twiddles need radix-E passes with one butterfly per thread");
  constexpr int E = G::E, H = E / 2, T = G::T;
  constexpr int64_t STRIDE = G::N / 2;
  __shared__ double lds[G::LDS_DOUBLES + G::N];
  double *const lx = lds;                   // exchange (real / imaginary halves in turn)
  double *const wl = lds + G::LDS_DOUBLES;  // window
  const int t = threadIdx.x;
  const uint32_t lane = (uint32_t)t;
  for (int i = t; i < G::N; i += G::WG) wl[i] = win[i];
  using RT = RegTw<G::NPASS>;
  RT rtw;
#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) rtw.base[p] = {1.0, 0.0};
  if constexpr (REGTW) {
    if constexpr (G::NPASS > 1) rtw.base[1] = pass_base<G::N, G::EMAX, G::ns(1)>(tw, t);
    if constexpr (G::NPASS > 2) rtw.base[2] = pass_base<G::N, G::EMAX, G::ns(2)>(tw, t);
    if constexpr (G::NPASS > 3) rtw.base[3] = pass_base<G::N, G::EMAX, G::ns(3)>(tw, t);
  }
  __syncthreads();
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;  // pairs, the last maybe partnerless
  const int64_t nfull = (seg_end - seg_begin) / 2;       // pairs with both segments
  const int64_t p0 = (int64_t)blockIdx.x * pairs_per_worker;
  const int64_t pend = p0 + pairs_per_worker < npairs ? p0 + pairs_per_worker : npairs;
  const int64_t fend = pend < nfull ? pend : nfull;
  if (p0 >= pend) return;  // whole workgroup (uniform): no barrier follows
  // row r of a pair's samples: x[(seg_begin + 2p) STRIDE + r T + lane]; the
  // rows a pair needs beyond its carry are H .. 2E-1 ... as scalar pointers
  auto row = [&](int64_t p, int r) -> const double * {
    return opaque_ptr(x + (seg_begin + 2 * p) * STRIDE + (int64_t)r * T);
  };
  double carry[H], a2[H], c2[H];
#pragma unroll
  for (int k = 0; k < H; ++k) carry[k] = row(p0, k)[lane];
  // samples of pair p: a = (carry, a2) is segment s0, (a2, c2) segment s0+1;
  // c2 of a partnerless pair is not read (its rows are clamped onto a2's)
  auto issue = [&](int64_t p) {
    const int cr = p < nfull ? E : H;
#pragma unroll
    for (int k = 0; k < H; ++k) {
      a2[k] = row(p, H + k)[lane];
      c2[k] = row(p, cr + k)[lane];
    }
  };
  issue(p0);
  constexpr int NACC = FOLD ? H + 1 : E;  // FOLD: E / 2 folded sums + thread 0's bin F / 2
  double acc[NACC];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = 0.0;
  auto pair = [&](int64_t p, bool first, bool partner) {
    const int tt = opaque_int(t);
    cd v[E];
    double wv[E];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      wv[k] = wl[tt + k * T];
      wv[H + k] = wl[tt + (H + k) * T];
      v[k] = {carry[k], partner ? a2[k] : 0.0};
      v[H + k] = {a2[k], partner ? c2[k] : 0.0};
    }
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = c2[k];
    if (p + 1 < pend) issue(p + 1);
    RT rl = rtw;
#pragma unroll
    for (int q = 1; q < G::NPASS; ++q) rl.base[q] = opaque_cd(rl.base[q]);
    // the window multiply after the next pair's loads are issued
#pragma unroll
    for (int k = 0; k < E; ++k) v[k] = {v[k].x * wv[k], v[k].y * wv[k]};
    if constexpr (REGTW)
      fft_regs<LOG2F, true, 2, LOG2E, 0, 0, RT, LAYOUT, false, NoEpi, 0, 16>(v, tt, rl, lx, lx,
                                                                          first);
    else
      fft_regs<LOG2F, true, 1, LOG2E, 0, 0, const cd *, LAYOUT>(v, tt, tw, lx, lx, first);
    if constexpr (FOLD) {
      double pw[E];
#pragma unroll
      for (int k = 0; k < E; ++k) pw[k] = fma(v[k].y, v[k].y, v[k].x * v[k].x);
      __syncthreads();  // the last exchange's reads are done
#pragma unroll
      for (int k = H; k < E; ++k) lx[tt * H + (k - H)] = pw[k];
      __syncthreads();
      if (tt == 0) {  // bins T m, mirrors T (E - m): 0 and F / 2 are their own
        acc[0] += pw[0];
#pragma unroll
        for (int m = 1; m < H; ++m) acc[m] += pw[m] + lx[H - m];
        acc[H] += lx[0];
      } else {
        const int tp = T - tt;
#pragma unroll
        for (int m = 0; m < H; ++m) acc[m] += pw[m] + lx[tp * H + (H - 1 - m)];
      }
    } else {
#pragma unroll
      for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  };
  int64_t p = p0;
  for (; p < fend; ++p) pair(p, p == p0, true);
  if (p < pend) pair(p, p == p0, false);  // the odd count's last segment, zero partner
  double *dst = partial + blockIdx.x * (int64_t)G::N;
  if constexpr (FOLD) {
#pragma unroll
    for (int k = 0; k < E; ++k)
      dst[t + k * T] = k < H ? acc[k] : (t == 0 && k == H ? acc[H] : 0.0);
  } else {
#pragma unroll
    for (int k = 0; k < E; ++k) dst[t + k * T] = acc[k];
  }
}


hipError_t launch_pwelch_row4096(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                 int64_t nworkers, const double *win, const cd *tw,
                                 double *partial, hipStream_t s) {
  hipLaunchKernelGGL((pwelch_row_kernel<12>), dim3((unsigned)nworkers), dim3(Geo<12>::WG), 0, s,
                     x, seg_begin, seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

// Any other overlap at F = 4096 with Pad = NFFT (Noverlap 0 among them): the
// same worker, twiddles, exchanges and accumulation, without the carry —
// segment s0 + 1 shares no register-aligned half with s0, so both segments of
// a pair are loaded whole (32 loads), each row a scalar base plus the lane's
// offset, at the top of the pair. (The next pair's 32 samples in flight during
// this pair's FFT, as the half-overlap kernel does with its 16, take 256
// VGPRs + 12 AGPRs: one wave per SIMD.) Per 2^28 samples against
// pwelch_kernel<12>: 4096 / 0 0.436 against 0.522 ms, 4096 / 1024 0.580
// against 0.695.
template <int LOG2F, int LOG2E = 4, int LAYOUT = 2>
__global__ __launch_bounds__((Geo<LOG2F, LOG2E>::WG)) void pwelch_rowg_kernel(
    const double *__restrict__ x, int64_t stride, int64_t seg_begin, int64_t seg_end,
    int64_t pairs_per_worker, const double *__restrict__ win, const cd *__restrict__ tw,
    double *__restrict__ partial) {
  using G = Geo<LOG2F, LOG2E>;
  static_assert(G::TPW == 1 && G::E == G::EMAX && G::NPE == G::NPASS && G::NPASS <= 4,
                "one worker per workgroup, register twiddles");
  constexpr int E = G::E, T = G::T;
  __shared__ double lds[G::LDS_DOUBLES + G::N];
  double *const lx = lds;
  double *const wl = lds + G::LDS_DOUBLES;
  const int t = threadIdx.x;
  const uint32_t lane = (uint32_t)t;
  for (int i = t; i < G::N; i += G::WG) wl[i] = win[i];
  using RT = RegTw<G::NPASS>;
  RT rtw;
#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) rtw.base[p] = {1.0, 0.0};
  if constexpr (G::NPASS > 1) rtw.base[1] = pass_base<G::N, G::EMAX, G::ns(1)>(tw, t);
  if constexpr (G::NPASS > 2) rtw.base[2] = pass_base<G::N, G::EMAX, G::ns(2)>(tw, t);
  if constexpr (G::NPASS > 3) rtw.base[3] = pass_base<G::N, G::EMAX, G::ns(3)>(tw, t);
  __syncthreads();
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t nfull = (seg_end - seg_begin) / 2;
  const int64_t p0 = (int64_t)blockIdx.x * pairs_per_worker;
  const int64_t pend = p0 + pairs_per_worker < npairs ? p0 + pairs_per_worker : npairs;
  const int64_t fend = pend < nfull ? pend : nfull;
  if (p0 >= pend) return;  // whole workgroup (uniform): no barrier follows
  auto row = [&](int64_t seg, int k) -> const double * {
    return opaque_ptr(x + seg * stride + (int64_t)k * T);
  };
  double a[E], b[E];
  // pair p's samples; a partnerless pair's second row is clamped onto its
  // first (not used)
  auto issue = [&](int64_t p) {
    const int64_t s0 = seg_begin + 2 * p, s1 = p < nfull ? s0 + 1 : s0;
#pragma unroll
    for (int k = 0; k < E; ++k) {
      a[k] = row(s0, k)[lane];
      b[k] = row(s1, k)[lane];
    }
  };
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  auto pair = [&](int64_t p, bool first, bool partner) {
    issue(p);
    const int tt = opaque_int(t);
    cd v[E];
#pragma unroll
    for (int k = 0; k < E; ++k) v[k] = {a[k], partner ? b[k] : 0.0};
    RT rl = rtw;
#pragma unroll
    for (int q = 1; q < G::NPASS; ++q) rl.base[q] = opaque_cd(rl.base[q]);
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const double wk = wl[tt + k * T];
      v[k] = {v[k].x * wk, v[k].y * wk};
    }
    fft_regs<LOG2F, true, 2, LOG2E, 0, 0, RT, LAYOUT, false, NoEpi, 0, 16>(v, tt, rl, lx, lx,
                                                                        first);
#pragma unroll
    for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
  };
  int64_t p = p0;
  for (; p < fend; ++p) pair(p, p == p0, true);
  if (p < pend) pair(p, p == p0, false);  // the odd count's last segment, zero partner
  double *dst = partial + blockIdx.x * (int64_t)G::N;
#pragma unroll
  for (int k = 0; k < E; ++k) dst[t + k * T] = acc[k];
}

hipError_t launch_pwelch_rowg4096(const double *x, int64_t stride, int64_t seg_begin,
                                  int64_t seg_end, int64_t ppw, int64_t nworkers,
                                  const double *win, const cd *tw, double *partial,
                                  hipStream_t s) {
  hipLaunchKernelGGL((pwelch_rowg_kernel<12>), dim3((unsigned)nworkers),
                     dim3(Geo<12>::WG), 0, s, x, stride, seg_begin, seg_end, ppw, win, tw,
                     partial);
  return hipGetLastError();
}

}  // namespace gdsp
