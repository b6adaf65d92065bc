// pwelch_wave.hip — the fused Pwelch accumulation (spectral/pwelch.go:104-122)
// for FFT lengths F = max(Pad, NFFT) from 64 to 1024, where a packed segment
// pair's transform (16 points per thread, T = F / 16 threads) fits inside one
// 64-lane wave, and F = 2048 in two-wave workgroups. Same arithmetic as pwelch_half_kernel / pwelch_kernel: z =
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
// half-block a slot shares with its neighbour comes from L2).
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
  // waves per SIMD the registers are held to: three for the half-overlap
  // wave kernels (twice the FFTs per sample: latency-bound), whose full-group
  // loop fits 168 VGPRs (the compiler's 35-44 spills from F = 256 are all in
  // the masked tail loop); the others at their natural 170-250 VGPRs, two per
  // SIMD (three cost F = 1024 56 spills and 35 % of its time)
  static constexpr int wpe(bool half) { return WAVE && half ? 3 : 1; }
};

template <int LOG2F, bool HALF, bool PAD>
__global__ __launch_bounds__((PwwGeo<LOG2F>::BLOCK))
__attribute__((amdgpu_waves_per_eu(PwwGeo<LOG2F>::wpe(HALF)))) void pwelch_wave_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t groups_per_wave, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F>;
  using W = PwwGeo<LOG2F>;
  constexpr int E = G::E, T = G::T, F = G::N, H = E / 2;
  static_assert(E == 16 && (T <= 64 ? 64 % T == 0 : T == 128), "one transform per wave or two waves");
  static_assert(!(HALF && PAD), "half overlap implies Pad = NFFT");
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
  // [g0, gm): full groups (each of the S pairs exists and has its partner),
  // run without masks; [gm, gend): at most the signal's last group, masked
  const int64_t gfull = (seg_end - seg_begin) / 2 / S;
  const int64_t gm = PAD ? g0 : (gend < gfull ? gend : (g0 > gfull ? g0 : gfull));
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  constexpr int NB = HALF ? H : E;  // second-segment samples loaded (HALF: its new half)
  // the packed pair of this slot from samples a (segment s0) and b (segment
  // s0 + 1; HALF: b[k] = a[k + H] for k < H, only b[H..E) loaded), windowed,
  // then transformed and summed as |Z_k|^2
  auto run = [&](const double (&a)[E], const double (&b)[NB], bool ina_all, bool inb_all,
                 bool active, bool has1) {
    const int tt = opaque_int(t);
    cd v[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int i = t + k * T;
      const double wk = wl[tt + k * T];
      double ak = a[k], bk = HALF ? (k < H ? a[k + H] : b[k - H]) : b[k];
      if (!ina_all) ak = active && (!PAD || i < nfft) ? ak : 0.0;
      if (!inb_all) bk = has1 && (!PAD || i < nfft) ? bk : 0.0;
      v[k] = {ak * wk, bk * wk};
    }
    // (every exchange but the kernel's first waits for the previous
    // transform's reads: a fence inside a wave, a barrier across two.) The
    // exchange slots are linear padded (LAYOUT 1, i + i / 16: per-thread base
    // plus compile-time offsets, paired ds_read2 / ds_write2) where T >= 32:
    // 1024 / 512 0.566 against 0.534 ms per 2^28 samples with XOR-swizzled
    // slots, 512 / 256 0.529 / 0.516, 2048 / 0 0.390 / 0.379 (the loop's non-
    // FP64 VALU 150 -> 28 at F = 1024; profiles/r05/pwelch_layout_ab.txt)
    fft_regs<LOG2F, true, 2, 4, 0, 0, const cd *, 1, 0, NoEpi, 0, 16, W::WAVE>(v, tt, twl, lre,
                                                                              lre, false);
#pragma unroll
    for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
  };
  // Full groups: each group's S pairs are 2 S consecutive segments from one
  // wave-uniform base, so every load is a buffer load from a scalar
  // descriptor, the lane's loop-invariant offset and a compile-time one — no
  // address arithmetic, clamps or masks in the vector unit.
  const uint32_t loff = (uint32_t)((2 * s * stride + t) * 8);
  auto load_full = [&](int64_t g, double (&a)[E], double (&b)[NB]) {
    const rsrc_t r = make_rsrc(x + (seg_begin + 2 * g * S) * stride, 0x7fffffff);
    const int sb = (int)(stride * 8);
    // (a constant offset past the 12-bit immediate goes to the scalar offset)
#pragma unroll
    for (int k = 0; k < E; ++k) {
      constexpr int kMaxImm = 4095;
      const int c = k * T * 8;
      a[k] = buf_ld1s(r, loff + (c <= kMaxImm ? c : 0), c <= kMaxImm ? 0 : c);
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      constexpr int kMaxImm = 4095;
      const int c = (HALF ? k + H : k) * T * 8;
      b[k] = buf_ld1s(r, loff + (c <= kMaxImm ? c : 0), sb + (c <= kMaxImm ? 0 : c));
    }
  };
  // (Loading the next group into registers while this one's FFT runs was
  // measured with the half-overlap kernels, per 2^28 samples: at two waves
  // per SIMD it lost to three waves without it, 128 / 64 0.452 against 0.419
  // ms, 512 / 256 0.564 against 0.534, 1024 / 512 0.604 against 0.554; at F =
  // 2048, two waves either way, 0.778 against 0.752.)
  if constexpr (!PAD) {
    for (int64_t g = g0; g < gm; ++g) {
      double a[E], b[NB];
      load_full(g, a, b);
      run(a, b, true, true, true, true);
    }
  }
  // The masked groups. Every load is unconditional, from a clamped address
  // (a slot past the pairs reads the last pair, a missing partner reads
  // segment s0 again, elements past nfft read element nfft - 1), and the mask
  // is applied where the samples are used, not where they are loaded: a load
  // inside a per-lane branch is waited for inside that branch (s_waitcnt
  // vmcnt(0) per element, serialising them all).
  for (int64_t g = gm; g < gend; ++g) {
    const int64_t p = g * S + s;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * (active ? p : npairs - 1);
    const bool has1 = active && s0 + 1 < seg_end;
    const double *xa = opaque_ptr(x) + s0 * stride;
    const double *xb = has1 ? xa + stride : xa;
    double a[E], b[NB];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int i = t + k * T;
      a[k] = xa[!PAD || i < nfft ? i : nfft - 1];
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int i = t + (HALF ? k + H : k) * T;
      b[k] = xb[!PAD || i < nfft ? i : nfft - 1];
    }
    // (HALF: a partnerless last pair, odd segment count, takes zeros for its
    // second segment's first half too, not segment s0's second half)
    run(a, b, false, false, active, has1);
  }
  // every slot writes its row (zeros for a slot with no pairs): the reduce
  // sums all of them
  double *dst = partial + (wave * S + s) * (int64_t)F;
#pragma unroll
  for (int k = 0; k < E; ++k) dst[t + k * T] = acc[k];
}

template <int LOG2F, bool HALF, bool PAD>
static hipError_t launch_pww_t(const double *x, int64_t nfft, int64_t stride, int64_t seg_begin,
                               int64_t seg_end, int64_t gpw, int64_t nblk, const double *win,
                               const cd *tw, double *partial, hipStream_t s) {
  hipLaunchKernelGGL((pwelch_wave_kernel<LOG2F, HALF, PAD>), dim3((unsigned)nblk),
                     dim3(PwwGeo<LOG2F>::BLOCK), 0, s, x, nfft, stride, seg_begin, seg_end, gpw,
                     win, tw, partial);
  return hipGetLastError();
}

// Geometry of a launch: pairs per group (S), groups per worker, workgroups,
// and the partial rows the reduce sums (one per transform slot).
bool pwelch_wave_applies(int log2f) { return log2f >= 6 && log2f <= 11; }

void pwelch_wave_geometry(int log2f, bool half, int64_t nsegs, int64_t *gpw, int64_t *nblk,
                          int64_t *nrows) {
  const int T = (1 << log2f) / 16;
  const bool wave = T <= 64;
  const int S = wave ? 64 / T : 1, wpb = wave ? kPwWaves : 1;
  const int64_t npairs = (nsegs + 1) / 2;
  const int64_t ngroups = (npairs + S - 1) / S;
  // waves in all: two per SIMD (2048: the kernels' register budget; 1024
  // two-wave workers at F = 2048 — with the window read from L1/L2 instead
  // of LDS, 21 KiB per workgroup and 168 VGPRs, three per SIMD measured
  // 0.712-0.743 against 0.707-0.723 ms per 2^28 samples at 2048 / 1024), three for the half-overlap wave kernels
  // from F = 128 (at F = 64 3072 workers measured 0.42 against 0.39 ms per
  // 2^28 samples for 2048)
  const int64_t target = !wave ? 1024 : half && log2f >= 7 ? 3072 : 2048;
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
#define GDSP_PWW(L)                                                                        \
  case L:                                                                                \
    return half ? launch_pww_t<L, true, false>(x, nfft, stride, seg_begin, seg_end, gpw, nblk, \
                                               win, tw, partial, s)                      \
           : nfft < (1 << L)                                                              \
               ? launch_pww_t<L, false, true>(x, nfft, stride, seg_begin, seg_end, gpw, nblk, \
                                              win, tw, partial, s)                       \
               : launch_pww_t<L, false, false>(x, nfft, stride, seg_begin, seg_end, gpw, nblk, \
                                               win, tw, partial, s);
    GDSP_PWW(6) GDSP_PWW(7) GDSP_PWW(8) GDSP_PWW(9) GDSP_PWW(10) GDSP_PWW(11)
#undef GDSP_PWW
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gdsp
