// pwelch_wave.hip — the fused Pwelch accumulation (spectral/pwelch.go:104-122)
// for FFT lengths F = max(Pad, NFFT) from 64 to 1024, where a packed segment
// pair's transform (16 points per thread, T = F / 16 threads) fits inside one
// 64-lane wave. Same arithmetic as pwelch_half_kernel / pwelch_kernel: z =
// w x_s + i w x_(s+1), Z = FFT_F(z), each thread accumulating |Z_k|^2 of its
// own bins in registers; the k / F - k fold is done once in finalise.
//
// What is different is the synchronisation. Those kernels run 256-thread
// workgroups of several transforms and meet at a workgroup barrier around
// every exchange, so all four waves of a workgroup stall together at each
// LDS round trip. Here every transform lives in one wave and exchanges
// through an LDS region of its own, so an exchange needs no barrier (xsync:
// a wave's LDS instructions execute in order) and the waves of a SIMD
// interleave freely. Each wave is a persistent worker over a contiguous range
// of pair groups: the S = 64 / T slots of the wave take S consecutive pairs
// per iteration, so a worker's pair range, its loop and its tests are wave-
// uniform. With HALF (Noverlap = NFFT / 2, Pad = NFFT) segment s + 1's first
// half is segment s's second half: 24 loads per pair instead of 32 (the
// half-block a slot shares with its neighbour comes from L2). PF: the next
// group's samples are loaded into registers while this group's FFT runs.
#include "fft_device.hpp"
#include "launch.hpp"

namespace gdsp {

constexpr int kPwWaves = 4;  // waves per workgroup

// Workers: with T <= 64 a wave (S = 64 / T transforms side by side, four
// waves per workgroup, wave-synchronised exchanges); with T = 128 (F = 2048)
// a two-wave workgroup of one transform, whose barriers meet only its own two
// waves (pwelch_half_kernel's 256-thread workgroups meet four).
template <int LOG2F>
struct PwwGeo {
  using G = Geo<LOG2F>;
  static constexpr int T = G::T;
  static constexpr bool WAVE = T <= 64;
  static constexpr int S = WAVE ? 64 / T : 1;       // transforms (pairs) per worker
  static constexpr int WPB = WAVE ? kPwWaves : 1;   // workers per workgroup
  static constexpr int BLOCK = WAVE ? 64 * kPwWaves : T;
  // twiddle bases the passes read: T_F[k], k < F / (last radix)
  static constexpr int TWN = G::N / G::radix(G::NPASS - 1);
};

template <int LOG2F, bool HALF, bool PF>
__global__ __launch_bounds__((PwwGeo<LOG2F>::BLOCK)) void pwelch_wave_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t groups_per_wave, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F>;
  using W = PwwGeo<LOG2F>;
  constexpr int E = G::E, T = G::T, F = G::N, H = E / 2;
  static_assert(E == 16 && (T <= 64 ? 64 % T == 0 : T == 128), "one transform per wave or two waves");
  constexpr int S = W::S;
  constexpr int XS = G::STRIDE;  // exchange doubles per transform
  // LDS: the exchange regions, the window, and the twiddle bases (from LDS,
  // so the samples in flight are the loop's only global loads: a global
  // twiddle read's wait, vmcnt being in order, would also wait for the next
  // group's samples)
  __shared__ double lds[W::WPB * S * XS + F + 2 * W::TWN];
  const int lt = (int)threadIdx.x;
  const int w = W::WAVE ? lt >> 6 : 0, lane = W::WAVE ? lt & 63 : lt;
  const int s = lane / T, t = lane % T;
  double *const lre = lds + (w * S + s) * XS;
  double *const wl = lds + W::WPB * S * XS;
  cd *const twl = reinterpret_cast<cd *>(wl + F);
  for (int i = lt; i < F; i += W::BLOCK) wl[i] = win[i];
  for (int i = lt; i < W::TWN; i += W::BLOCK) twl[i] = tw[i];
  __syncthreads();
  // the worker and its group range: uniform over its waves
  const int64_t wave = (int64_t)blockIdx.x * W::WPB + __builtin_amdgcn_readfirstlane(w);
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t ngroups = (npairs + S - 1) / S;
  const int64_t g0 = wave * groups_per_wave;
  const int64_t gend = g0 + groups_per_wave < ngroups ? g0 + groups_per_wave : ngroups;
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  // samples of group g for this slot: a[k] = segment s0's element t + k T,
  // b[k] = segment s0 + 1's (HALF: b[k] = a[k + H] for k < H, so only b[H..E)
  // is loaded); zero past the signal's segments and past nfft (Pad > NFFT)
  constexpr int NB = HALF ? H : E;
  // Every load is unconditional, from a clamped address (a slot past the
  // pairs reads the last pair, a missing partner reads segment s0 again,
  // elements past nfft read element nfft - 1), and the mask is applied where
  // the samples are used, not where they are loaded: a load inside a per-lane
  // branch is waited for inside that branch (s_waitcnt vmcnt(0) per element,
  // serialising them all), and a select right after a prefetch waits for it.
  auto seg0 = [&](int64_t g, bool &active, bool &has1) {
    const int64_t p = g * S + s;
    active = g < gend && p < npairs;
    const int64_t s0 = seg_begin + 2 * (active ? p : npairs - 1);
    has1 = active && s0 + 1 < seg_end;
    return s0;
  };
  auto load = [&](int64_t g, double (&a)[E], double (&b)[NB]) {
    bool active, has1;
    const int64_t s0 = seg0(g, active, has1);
    const double *xa = opaque_ptr(x) + s0 * stride;
    const double *xb = has1 ? xa + stride : xa;
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int i = t + k * T;
      a[k] = xa[HALF || i < nfft ? i : nfft - 1];
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int i = t + (HALF ? k + H : k) * T;
      b[k] = xb[HALF || i < nfft ? i : nfft - 1];
    }
  };
  double na[E], nb[NB];
  if constexpr (PF) load(g0, na, nb);
  for (int64_t g = g0; g < gend; ++g) {
    double a[E], b[NB];
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < E; ++k) a[k] = na[k];
#pragma unroll
      for (int k = 0; k < NB; ++k) b[k] = nb[k];
      if (g + 1 < gend) load(g + 1, na, nb);
    } else {
      load(g, a, b);
    }
    bool active, has1;
    (void)seg0(g, active, has1);
    const int tt = opaque_int(t);
    cd v[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      // (HALF: a partnerless last pair, odd segment count, takes zeros for
      // its second segment's first half too, not segment s0's second half)
      const int i = t + k * T;
      const bool ina = active && (HALF || i < nfft);
      const bool inb = has1 && (HALF || i < nfft);
      const double wk = wl[tt + k * T];
      const double ak = ina ? a[k] : 0.0;
      const double bk = inb ? (HALF ? (k < H ? a[k + H] : b[k - H]) : b[k]) : 0.0;
      v[k] = {ak * wk, bk * wk};
    }
    fft_regs<LOG2F, true, 2, 4, 0, 0, const cd *, 0, 0, NoEpi, 0, 16, W::WAVE>(v, tt, twl, lre,
                                                                              lre, g == g0);
    if (active) {
#pragma unroll
      for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  }
  // every slot writes its row (zeros for a slot with no pairs): the reduce
  // sums all of them
  double *dst = partial + (wave * S + s) * (int64_t)F;
#pragma unroll
  for (int k = 0; k < E; ++k) dst[t + k * T] = acc[k];
}

template <int LOG2F, bool HALF, bool PF>
static hipError_t launch_pww_t(const double *x, int64_t nfft, int64_t stride, int64_t seg_begin,
                               int64_t seg_end, int64_t gpw, int64_t nblk, const double *win,
                               const cd *tw, double *partial, hipStream_t s) {
  hipLaunchKernelGGL((pwelch_wave_kernel<LOG2F, HALF, PF>), dim3((unsigned)nblk),
                     dim3(PwwGeo<LOG2F>::BLOCK), 0, s, x, nfft, stride, seg_begin, seg_end, gpw,
                     win, tw, partial);
  return hipGetLastError();
}

// Geometry of a launch: pairs per group (S), groups per worker, workgroups,
// and the partial rows the reduce sums (one per transform slot).
bool pwelch_wave_applies(int log2f) { return log2f >= 6 && log2f <= 11; }

void pwelch_wave_geometry(int log2f, int64_t nsegs, int64_t *gpw, int64_t *nblk,
                          int64_t *nrows) {
  const int T = (1 << log2f) / 16;
  const bool wave = T <= 64;
  const int S = wave ? 64 / T : 1, wpb = wave ? kPwWaves : 1;
  const int64_t npairs = (nsegs + 1) / 2;
  const int64_t ngroups = (npairs + S - 1) / S;
  // about 2048 waves in all (8 per CU: two per SIMD, the kernel's register
  // budget): 2048 one-wave workers, or 1024 two-wave ones
  const int64_t target = wave ? 2048 : 1024;
  const int64_t g = ngroups < 1 ? 1 : (ngroups + target - 1) / target;
  const int64_t workers = ngroups < 1 ? 1 : (ngroups + g - 1) / g;
  *gpw = g;
  *nblk = (workers + wpb - 1) / wpb;
  *nrows = *nblk * wpb * S;
}

hipError_t launch_pwelch_wave(int log2f, bool half, const double *x, int64_t nfft, int64_t stride,
                              int64_t seg_begin, int64_t seg_end, int64_t gpw, int64_t nblk,
                              const double *win, const cd *tw, double *partial, hipStream_t s) {
  if (nblk < 1 || nblk > 0x7fffffff) return hipErrorInvalidValue;
  switch (log2f) {
// PF for the half-overlap case only: there it measured 0.571 against 0.58
// ms (256 / 128), 0.664 against 0.69 (1024 / 512) and 0.53 against 0.56 (64 /
// 32) per 2^28 samples; without overlap all 32 samples of a pair are new and
// the prefetch costs more registers than it hides (1024 / 0: 0.454 against
// 0.43 ms; at F = 2048 it leaves one wave per SIMD)
#define GDSP_PWW(L)                                                                           \
  case L:                                                                                   \
    return half ? launch_pww_t<L, true, true>(x, nfft, stride, seg_begin, seg_end, gpw, nblk, \
                                              win, tw, partial, s)                          \
                : launch_pww_t<L, false, false>(x, nfft, stride, seg_begin, seg_end, gpw,     \
                                                nblk, win, tw, partial, s);
    GDSP_PWW(6) GDSP_PWW(7) GDSP_PWW(8) GDSP_PWW(9) GDSP_PWW(10) GDSP_PWW(11)
#undef GDSP_PWW
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gdsp
