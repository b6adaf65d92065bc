// fft_kernels.hip — gfx950 kernels of the go-dsp FFT engine and their host
// launchers (declared in launch.hpp). See DESIGN.md for the roofline of each.
//
//   fft_lds_kernel       one launch, one HBM read + one HBM write per
//                        transform, power-of-2 N <= 16384 (fft/radix2.go:80-154,
//                        fft/fft.go:35-52 for the inverse)
//   stockham_global_pass multi-launch power-of-2 N > 16384 (radix-16 passes
//                        through HBM)
//   bluestein_kernel     fused chirp-z: premultiply, FFT_M, x FFT_M(b), IFFT_M,
//                        postmultiply in one launch (fft/bluestein.go:68-94 with
//                        Convolve fft/fft.go:55-69), M <= 16384
//   pwelch_kernel        fused window + two-real-segments-per-complex FFT +
//                        |X|^2 accumulation (spectral/pwelch.go:104-122)
//   transpose / elementwise helpers for FFT2 (fft/fft.go:123-154) and for the
//   composed Bluestein / materialised Pwelch paths.
#include "fft_device.hpp"
#include "launch.hpp"
#include "lds_kernel.hpp"

#include <stdlib.h>

namespace gdsp {

// ----------------------------------------------------------------------------
// Epilogues of the chirp-z kernel's two FFTs (fft_regs EPI): FFT 1 ends with
// v = conj(A * bhat), FFT 2 with the postmultiply and the store of the first
// n outputs; both load their factors ahead of each butterfly's arithmetic.
template <int T>
struct BhatEpi {
  const cd *m;  // bhat + t
  static constexpr bool on = true;
  __device__ static constexpr bool want(int) { return true; }
  __device__ cd load(int k) const { return m[k * T]; }
  template <int E>
  __device__ void apply(cd (&v)[E], int k, cd u, cd f) const { v[k] = conjg(cmul(u, f)); }
};
template <int T, int KH, bool INV>
struct ChirpOutEpi {
  const cd *chirp;
  cd *dst;  // the transform's output row, or null (a padding slot)
  int t;
  int64_t n;
  double scale;
  static constexpr bool on = true;
  __device__ static constexpr bool want(int k) { return k < KH; }
  __device__ cd load(int k) const {
    const int idx = t + k * T;
    return idx < n ? chirp[idx] : cd{0.0, 0.0};
  }
  template <int E>
  __device__ void apply(cd (&)[E], int k, cd u, cd f) const {
    const int idx = t + k * T;
    if (dst && idx < n) {
      cd y = cmul(conjg(u), f);
      if constexpr (INV) y = {y.x * scale, -y.y * scale};
      st_nt(&dst[idx], y);
    }
  }
};

// The same two epilogues for one transform per workgroup, through
// bounds-checked buffer descriptors (row, chirp, bhat): no per-element test,
// branch or 64-bit address (loads past n read 0, stores past n are dropped).
template <int T>
struct BhatBufEpi {
  rsrc_t m;      // bhat (M values)
  uint32_t off;  // the lane's byte offset, t * 16
  static constexpr bool on = true;
  __device__ static constexpr bool want(int) { return true; }
  __device__ cd load(int k) const { return buf_ld(m, off + (uint32_t)(k * T * 16)); }
  template <int E>
  __device__ void apply(cd (&v)[E], int k, cd u, cd f) const { v[k] = conjg(cmul(u, f)); }
};
template <int T, int KH, bool INV>
struct ChirpOutBufEpi {
  rsrc_t chirp, dst;  // n values each
  uint32_t off;
  double scale;
  static constexpr bool on = true;
  __device__ static constexpr bool want(int k) { return k < KH; }
  __device__ cd load(int k) const { return buf_ld(chirp, off + (uint32_t)(k * T * 16)); }
  template <int E>
  __device__ void apply(cd (&)[E], int k, cd u, cd f) const {
    cd y = cmul(conjg(u), f);
    if constexpr (INV) y = {y.x * scale, -y.y * scale};
    buf_st_nt(dst, off + (uint32_t)(k * T * 16), y);
  }
};

// Which chirp-z steps ride in an FFT's last pass (EPI): 2 both the bhat step
// and the output postmultiply, 1 the bhat step only, 0 neither. Chosen per M
// by occupancy and measurement (forced chirp-z, ms per 2^27 samples, 2 runs
// each, both / bhat only / neither): M = 2^4 (n 5, 7) 4.62, 5.43 / — / 4.80,
// 6.50; 2^5 (13) 4.33 / — / 4.10; 2^6 (29) 2.64 / — / 2.58; 2^7 (n 37) 1.76-1.86 / 1.86-1.93 /
// 2.04-2.11; 2^8 (101) 1.38-1.40 / 1.75-1.78 / 1.73-1.78; 2^10 (509, the
// fused steps cost a wave per SIMD) 1.68 / 1.71-1.72 / 1.46; 2^11 (1021) 1.57
// / 1.72 / 1.74; 2^12 (1201, 2039; both: 2 waves per SIMD, else 3) 2.65 /
// 2.23 / 2.24-2.27 and 1.83 / 1.76 / 1.77; 2^13 (3000, 4093) 2.16-2.18 /
// 2.17-2.19 / 2.24 and 1.83 / 1.91 / 1.98; 2^14 (8191) 2.35 / 2.27-2.28 / 2.26.
// Twiddle-base prefetch (fft_regs PREW) for passes with one base per thread;
// not at M = 2^10, where it costs that kernel a wave per SIMD
constexpr int kPwPrew = 1;
__host__ __device__ constexpr int blu_prew(int log2m) { return log2m == 10 ? 0 : 1; }
__host__ __device__ constexpr int blu_epi_mode(int log2m, int log2e) {
  // (the 16-points-per-thread kernels of M = 2^13 / 2^14: none; with both
  // chirpz3000 took 4.86 against 3.40 ms)
  return (log2m == 5 || log2m == 6 || log2m == 10 || (log2m >= 13 && log2e == 4)) ? 0
         : (log2m == 12 || log2m == 14)                                          ? 1
                                                                                 : 2;
}

// Fused Bluestein (chirp-z) for non-power-of-2 n with M = NextPowerOf2(2n-1):
//   a = x * conj(w) (zero-padded to M), A = FFT_M(a), C = A * bhat,
//   r = IFFT_M(C) = conj(FFT_M(conj(C))) (1/M folded into bhat),
//   X = r * conj(w), first n.  chirp[k] = conj(w_k) = exp(-i pi k^2/n).
// Inverse (fft.IFFT of non-power-of-2 length): conj in, conj + 1/n out.
//
// PARTS (n > M/2, where bluestein.go:70's M would exceed one kernel): the
// outputs are split into nparts parts of kpart, part p computing
// X[k0 + k], k < kpart, k0 = p * kpart, by its own circular
// convolution c_p[m mod M] = w_(k0 + m), m in [-(n-1), kpart-1], which does not
// wrap as long as n + kpart - 1 <= M (bhat + p * M holds FFT_M(c_p)/M).
// The input then fills more than half of M, so only the output side is pruned.
// Rows ahead a chirp-z block touches for its successor on the XCD (0: off).
// chirpz3000 2.95-3.05 -> 2.80-2.89 ms at 8-32, 2.84-2.85 at 48, 2.94-3.03 at
// 64-128 (scripts/archive/dev/blu_pf_ab.sh); blocks of several transforms (M <= 2048)
// touch the same slot's row kBluPf blocks on: primes 13..1021 10-22 %
// faster (scripts/archive/dev/blu_pfall_ab.sh)
constexpr int kBluPf = 16;
// Twiddle powers of the radix-8 passes by the three-term recurrence
// (pass_compute CHEB; one transform per workgroup): chirpz3000 2.65-2.67
// against 2.71-2.74 ms, parity 1.58e-15 against 1.56e-15 vs the oracle. The
// radix-32 passes keep complex products: the recurrence there bought 0.3 %
// for 5.5e-15 (scripts/archive/gpu_r03_cheb.sh)
constexpr int kBluChebR = 8;
constexpr int kBluPf14 = 4;     // M = 16384, one block per CU: 2-4 % faster than 8 or 16
constexpr int kBluPfParts = 2;  // PARTS: the row's part-0 block touches 2 rows on
constexpr int kBluPfShift = 7;  // touch granularity: one load per 2^7 bytes (a line)
// KN (one transform per workgroup, the buffer path): n <= KN T, so
// registers k >= KN hold no input to FFT 1 and no wanted output of FFT 2 —
// pass 0 of FFT 1 adds no zeros and the last pass of FFT 2 forms only the
// outputs below KN T (0: KN = E/2, what n <= M/2 guarantees for any n).
template <int LOG2M, bool INV, bool SPLIT, int LOG2E = 4, bool PARTS = false, int KN = 0>
__global__ __launch_bounds__((Geo<LOG2M, LOG2E>::WG))
__attribute__((amdgpu_waves_per_eu(LOG2M >= 13 && LOG2E == 4 ? 4 : 1))) void bluestein_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ twm, const cd *__restrict__ chirp, const cd *__restrict__ bhat,
    double scale, int64_t kpart, int nparts) {
  using G = Geo<LOG2M, LOG2E>;
  __shared__ double lds[(SPLIT ? 1 : 2) * G::LDS_DOUBLES];
  const int lt = threadIdx.x;
  const int slot = lt / G::T;
  const int t = lt & (G::T - 1);
  // PARTS: the parts of a row are adjacent block indices (after the XCD
  // remap, so on one XCD at about the same time), and its 2nd..nth reads of
  // the row hit L2 instead of HBM (the part-major grid was 3-9 % slower)
  int64_t gb = xcd_remap(blockIdx.x, gridDim.x);
  int part = 0;
  if constexpr (PARTS) {
    const int64_t q = gb / nparts;
    part = (int)(gb - q * nparts);
    gb = q;
  }
  const int64_t g = gb * G::TPW + slot;
  const bool valid = g < batch;
  double *lre = lds + slot * G::STRIDE;
  double *lim = SPLIT ? lre : lds + G::LDS_DOUBLES + slot * G::STRIDE;
  // n <= M/2 (M is a power of 2 >= 2n - 1): registers k >= E/2 hold no input
  // and no output, so the first pass of FFT 1 and the last of FFT 2 are pruned
  static_assert(KN == 0 || (KN >= 1 && KN <= G::E / 2 && !PARTS), "KN within the first half");
  constexpr int KH = KN > 0 ? KN : (G::E > 1 ? G::E / 2 : G::E);
  constexpr int KIN = PARTS ? G::E : KH;
  // pass 0 of FFT 1: the nonzero inputs per butterfly (0: no pruning)
  constexpr int ZIN = G::E >= 4 && !PARTS ? KH : 0;
  // this block's outputs: X[k0 + k], k < nout
  int64_t nout = n;
  const cd *ochirp = chirp;
  cd *orow = valid ? out + g * n : nullptr;
  if constexpr (PARTS) {
    const int64_t k0 = (int64_t)part * kpart;
    nout = n - k0 < kpart ? n - k0 : kpart;
    ochirp += k0;
    if (orow) orow += k0;
    bhat += (int64_t)part * G::N;
  }
  cd v[G::E];
  constexpr int EPI = blu_epi_mode(LOG2M, LOG2E);
  if constexpr (G::TPW == 1 && !PARTS && EPI == 2) {
    // one transform per workgroup: the row, its successor (touch-ahead), the
    // chirp and bhat through wave-uniform buffer descriptors, every load
    // issued before the first use
    const int64_t gu = gb;
    const uint32_t off = (uint32_t)t * 16u;
    const int64_t rowb = n * 16;
    const rsrc_t rin = make_rsrc(in + gu * n, rowb);
    const rsrc_t rch = make_rsrc(chirp, rowb);
    const int64_t gp = gu + (LOG2M == 14 ? kBluPf14 : kBluPf);
    const rsrc_t rpf = make_rsrc(in + (gp < batch ? gp : gu) * n, gp < batch ? rowb : 0);
    constexpr int SH = kBluPfShift, NPF = (G::E * 8 >> SH) > 0 ? (G::E * 8 >> SH) : 1;
    double pf[NPF];
#pragma unroll
    for (int k = 0; k < NPF; ++k) pf[k] = buf_ld1(rpf, ((uint32_t)t + (uint32_t)(k * G::T)) << SH);
    cd xv[KIN], cv[KIN];
#pragma unroll
    for (int k = 0; k < KIN; ++k) {
      xv[k] = buf_ld(rin, off + (uint32_t)(k * G::T * 16));
      cv[k] = buf_ld(rch, off + (uint32_t)(k * G::T * 16));
    }
#pragma unroll
    for (int k = 0; k < NPF; ++k) asm volatile("" ::"v"(pf[k]));
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
      if (k < KIN) {
        cd x = xv[k];
        if constexpr (INV) x.y = -x.y;
        v[k] = cmul(x, cv[k]);
      } else {
        v[k] = {0.0, 0.0};
      }
    }
    const BhatBufEpi<G::T> be{make_rsrc(bhat, (int64_t)G::N * 16), off};
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, ZIN, BhatBufEpi<G::T>,
             blu_prew(LOG2M), kBluChebR>(v, t, twm, lre, lim, true, be);
    const ChirpOutBufEpi<G::T, KH, INV> oe{make_rsrc(opaque_ptr(chirp), rowb),
                                           make_rsrc(out + gu * n, rowb), (uint32_t)opaque_int(t) * 16u,
                                           scale};
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, false,
             ChirpOutBufEpi<G::T, KH, INV>, blu_prew(LOG2M), kBluChebR>(v, t, twm, lre,
                                                                                 lim, false, oe);
    return;
  }
  const cd *src = in + g * n;
  // touch every 128-B line of the row the block kBluPf places later on
  // this XCD will take (xcd_remap keeps an XCD's rows contiguous), so that
  // block's row loads hit L2 / MALL instead of waiting on HBM
  // (n <= M/2 = T*E/2, so a row is at most T*E*16/2^SH pieces of 2^SH bytes:
  // E*8/2^SH per thread of the transform's T)
  // (PARTS: n <= M, twice the pieces; the row's part-0 block touches the row
  // kBluPfParts rows on)
  constexpr int SH = kBluPfShift,
                NPF = ((PARTS ? 2 : 1) * G::E * 8 >> SH) > 0 ? ((PARTS ? 2 : 1) * G::E * 8 >> SH) : 1;
  double pf[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) pf[k] = 0.0;
  {
    const int64_t gp = g + (PARTS ? (int64_t)kBluPfParts
                                  : (int64_t)(LOG2M == 14 ? kBluPf14 : kBluPf) * G::TPW);
    if (valid && gp < batch && part == 0) {
      const char *prow = reinterpret_cast<const char *>(in + gp * n);
      const int pieces = (int)((n * 16 + (1 << SH) - 1) >> SH);
#pragma unroll
      for (int k = 0; k < NPF; ++k)
        if (t + k * G::T < pieces)
          pf[k] = *reinterpret_cast<const double *>(prow + ((int64_t)(t + k * G::T) << SH));
    }
  }
#pragma unroll
  for (int k = 0; k < G::E; ++k) {
    const int idx = t + k * G::T;
    v[k] = {0.0, 0.0};
    if (k < KIN && valid && idx < n) {
      cd x = ld_nt(&src[idx]);
      if constexpr (INV) x.y = -x.y;
      v[k] = cmul(x, chirp[idx]);
    }
  }
  // the prefetches were issued before the row loads the premultiply waited
  // for (loads return in order), so consuming them here costs no wait
#pragma unroll
  for (int k = 0; k < NPF; ++k) asm volatile("" ::"v"(pf[k]));
  if constexpr (EPI >= 1) {
    // x bhat, conj: fused into FFT 1's last pass, each butterfly's factors
    // loaded ahead of its arithmetic
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, ZIN, BhatEpi<G::T>, blu_prew(LOG2M)>(
        v, t, twm, lre, lim, true, BhatEpi<G::T>{bhat + t});
  } else {
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, ZIN, NoEpi, blu_prew(LOG2M)>(
        v, t, twm, lre, lim, true);
#pragma unroll
    for (int k = 0; k < G::E; ++k) v[k] = conjg(cmul(v[k], bhat[t + k * G::T]));
  }
  if constexpr (EPI == 2) {
    // postmultiply and store: fused into FFT 2's last pass the same way
    const ChirpOutEpi<G::T, KH, INV> oe{opaque_ptr(ochirp), orow, opaque_int(t), nout, scale};
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, false,
             ChirpOutEpi<G::T, KH, INV>, blu_prew(LOG2M)>(v, t, twm, lre, lim, false, oe);
  } else {
    fft_regs<LOG2M, SPLIT, true, LOG2E, 0, 0, const cd *, true, false, NoEpi, blu_prew(LOG2M)>(
        v, t, twm, lre, lim, false);
    ochirp = opaque_ptr(ochirp);
    const int to = opaque_int(t);
    if (orow) {
      cd *dst = orow;
#pragma unroll
      for (int k = 0; k < KH; ++k) {
        const int idx = to + k * G::T;
        if (idx < nout) {
          cd y = cmul(conjg(v[k]), ochirp[idx]);
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          st_nt(&dst[idx], y);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------
// One radix-R Stockham pass through HBM (large power-of-2 N). One thread per
// butterfly; loads are coalesced across j.
template <int R, bool CONJ_IN, int LOAD, bool CONJ_SCALE_OUT>
__global__ __launch_bounds__(256) void stockham_global_pass(
    const void *__restrict__ in, cd *__restrict__ out, const cd *__restrict__ tw, int log2n,
    int log2ns, int64_t batch, double scale) {
  const int64_t nr = ((int64_t)1 << log2n) / R;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= batch * nr) return;
  const int64_t g = tid / nr;
  const int64_t j = tid - g * nr;
  const int64_t N = (int64_t)1 << log2n;
  const int64_t NS = (int64_t)1 << log2ns;
  cd u[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (LOAD == LOAD_COMPLEX) {
      u[r] = ld_nt(reinterpret_cast<const cd *>(in) + g * N + j + r * nr);
      if constexpr (CONJ_IN) u[r].y = -u[r].y;
    } else {
      u[r] = {ld_nt(reinterpret_cast<const double *>(in) + g * N + j + r * nr), 0.0};
    }
  }
  if (NS > 1) {
    const cd w = tw[(j & (NS - 1)) * (N / (NS * R))];
    cd wr = w;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      u[r] = cmul(u[r], wr);
      wr = cmul(wr, w);
    }
  }
  Dft<R>::run(u);
  const int64_t base = g * N + (j >> log2ns) * (NS * R) + (j & (NS - 1));
#pragma unroll
  for (int r = 0; r < R; ++r) {
    cd o = u[r];
    if constexpr (CONJ_SCALE_OUT) o = {o.x * scale, -o.y * scale};
    st_nt(&out[base + r * NS], o);
  }
}

// ----------------------------------------------------------------------------
// Fused Welch periodogram accumulation over packed segment pairs:
// z = w*x_s0 + i*w*x_s1, Z = FFT(z); |X_s0,k|^2 + |X_s1,k|^2 =
// (|Z_k|^2 + |Z_{F-k}|^2)/2, so each thread accumulates |Z_k|^2 for its own
// bins across all pairs of its worker, in registers; the k / F-k fold is done
// once in gdsp_pwelch_finalize.
template <int LOG2F, bool SPLIT, int LOG2E = 4>
__global__ __launch_bounds__((Geo<LOG2F, LOG2E>::WG)) void pwelch_kernel(
    const double *__restrict__ x, int64_t nfft, int64_t stride, int64_t seg_begin,
    int64_t seg_end, int64_t pairs_per_worker, const double *__restrict__ win,
    const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F, LOG2E>;
  __shared__ double lds[(SPLIT ? 1 : 2) * G::LDS_DOUBLES];
  const int lt = threadIdx.x;
  const int slot = lt / G::T;
  const int t = lt & (G::T - 1);
  const int64_t worker = (int64_t)blockIdx.x * G::TPW + slot;
  double *lre = lds + slot * G::STRIDE;
  double *lim = SPLIT ? lre : lds + G::LDS_DOUBLES + slot * G::STRIDE;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  double acc[G::E];
#pragma unroll
  for (int k = 0; k < G::E; ++k) acc[k] = 0.0;
  for (int64_t it = 0; it < pairs_per_worker; ++it) {
    const int64_t p = worker * pairs_per_worker + it;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * p;
    const bool has1 = active && (s0 + 1 < seg_end);
    const double *x0 = x + s0 * stride;
    const double *x1 = x0 + stride;
    // the window is re-read every iteration (L1/L2 hits) instead of being
    // held in 2*E registers across the loop
    const double *w = opaque_ptr(win);
    const int tt = opaque_int(t);
    cd v[G::E];
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
      const int i = tt + k * G::T;
      const bool in_seg = i < nfft;
      const double wk = w[i];
      const double a = (active && in_seg) ? x0[i] : 0.0;
      const double b = (has1 && in_seg) ? x1[i] : 0.0;
      v[k] = {a * wk, b * wk};
    }
    fft_regs<LOG2F, SPLIT, true, LOG2E>(v, tt, tw, lre, lim, it == 0);
    if (active) {
#pragma unroll
      for (int k = 0; k < G::E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  }
  if (worker * pairs_per_worker < npairs) {
    double *dst = partial + worker * G::N;
#pragma unroll
    for (int k = 0; k < G::E; ++k) dst[t + k * G::T] = acc[k];
  }
}

// Half-overlap specialisation (Noverlap = NFFT/2, Pad = NFFT: the BASELINE
// configuration and Welch's usual choice). With stride = F/2 and thread t
// owning samples t + k*T of a segment, segment s0+1's element k is segment
// s0's element k + E/2, and the next pair's first segment starts where
// s0+1's second half does. So per pair a thread loads only E new samples and
// carries E/2 across iterations: every sample is read from HBM/L2 once, and
// the window stays in registers.
// WMODE: where the window lives — 0 registers, 1 re-read from global (L1/L2)
// every iteration, 2 an LDS table shared by the workgroup.
// Measured at F = 4096 (2^30 samples): E = 16 with the LDS window 3.19 ms;
// E = 8 (LOG2E = 3: 104 VGPRs, twice the waves, one more exchange) 3.67 ms;
// E = 16 forced to 168 / 128 VGPRs (MINW 3 / 4) spills: 4.85 / 6.07 ms;
// window re-read from L1/L2 (WMODE 1) with the split exchange 3.48 ms, with
// a complex (two-buffer) exchange 3.45 ms.
// Exchange slot layout of the half-overlap kernels: the linear padded layout
// (slot i + i / E: a per-thread base plus compile-time offsets, and paired
// ds_read2 / ds_write2, at the cost of 2-way conflicted reads at E = 16).
// Against XOR-swizzled slots (conflict-free, an address computation per
// element) it measured slower on the round-2 NFFT 4096 kernel (3.08-3.09
// against 3.03-3.05 ms) and faster on the ones left here in round 5: 16384 /
// 8192 1.88 against 2.01 ms per 2^28 samples, 8192 / 4096 equal
// (profiles/r05/pwelch_layout_ab.txt). NFFT 4096 runs on the row kernels
// (XOR for the first exchange, a block-padded layout for the second: LAYOUT
// 2, fft_device.hpp), 64 ... 2048 on the wave kernels (pwelch_wave.hip).
constexpr int kPwLinear = 1;
// PF: the pass twiddle bases (T_N[0 .. N/R_last)) live in LDS, so the only
// global loads in the loop are the samples, and the next pair's samples are
// prefetched while this pair's FFT runs (vmcnt then covers only them)
template <int LOG2F, int WMODE = 2, int MINW = 1, int LOG2E = 4, bool SPLIT = true,
          bool PF = false>
__global__ __launch_bounds__((Geo<LOG2F, LOG2E>::WG), MINW) void pwelch_half_kernel(
    const double *__restrict__ x, int64_t seg_begin, int64_t seg_end, int64_t pairs_per_worker,
    const double *__restrict__ win, const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F, LOG2E>;
  constexpr int E = G::E, H = E / 2;
  constexpr int64_t STRIDE = G::N / 2;
  constexpr int XD = (SPLIT ? 1 : 2) * G::LDS_DOUBLES;  // exchange buffer(s)
  constexpr int TWN = PF ? G::N / G::radix(G::NPASS - 1) : 0;
  __shared__ double lds[XD + (WMODE == 2 ? G::N : 0) + 2 * TWN];
  const int lt = threadIdx.x;
  // one worker per workgroup (TPW = 1, F >= 4096): the worker index, its
  // pairs, their segment offsets and the active / has-partner tests are
  // wave-uniform (scalar registers and branches), and the sample loads are
  // a scalar row base plus the lane's 32-bit offset
  const int slot = G::TPW == 1 ? 0 : lt / G::T;
  const int t = lt & (G::T - 1);
  const int64_t worker = (int64_t)blockIdx.x * G::TPW + slot;
  double *lre = lds + slot * G::STRIDE;
  double *lim = SPLIT ? lre : lre + G::LDS_DOUBLES;
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  double wv[E];
  double *wl = lds + XD;
  if constexpr (WMODE == 0) {
#pragma unroll
    for (int k = 0; k < E; ++k) wv[k] = win[t + k * G::T];
  } else if constexpr (WMODE == 2) {
    for (int i = lt; i < G::N; i += G::WG) wl[i] = win[i];
  }
  cd *twl = reinterpret_cast<cd *>(lds + XD + (WMODE == 2 ? G::N : 0));
  if constexpr (PF) {
    for (int i = lt; i < TWN; i += G::WG) twl[i] = tw[i];
  }
  if constexpr (WMODE == 2 || PF) __syncthreads();
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  const int64_t p0 = worker * pairs_per_worker;
  // carried samples: the first half of the next pair's first segment
  double carry[H];
  {
    const int64_t s0 = seg_begin + 2 * (p0 < npairs ? p0 : 0);
    const double *b = x + s0 * STRIDE + t;
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = (p0 < npairs) ? b[k * G::T] : 0.0;
  }
  // samples of pair p: a[0..H) = carry, a[H..E) (shared with seg s0+1),
  // c[0..H) = second half of seg s0+1 (= first half of the next pair)
  auto load_pair = [&](int64_t p, double (&a2)[H], double (&c2)[H]) {
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * p;
    const bool has1 = active && (s0 + 1 < seg_end);
    if constexpr (G::TPW == 1) {
      const double *b = opaque_ptr(x) + s0 * STRIDE;
      const uint32_t lane = (uint32_t)t;
      if (active) {
#pragma unroll
        for (int k = 0; k < H; ++k) a2[k] = (b + (H + k) * G::T)[lane];
      } else {
#pragma unroll
        for (int k = 0; k < H; ++k) a2[k] = 0.0;
      }
      if (has1) {
#pragma unroll
        for (int k = 0; k < H; ++k) c2[k] = (b + (E + k) * G::T)[lane];
      } else {
#pragma unroll
        for (int k = 0; k < H; ++k) c2[k] = 0.0;
      }
    } else {
      const double *b = opaque_ptr(x) + s0 * STRIDE + t;
#pragma unroll
      for (int k = 0; k < H; ++k) {
        a2[k] = active ? b[(H + k) * G::T] : 0.0;
        c2[k] = has1 ? b[(E + k) * G::T] : 0.0;
      }
    }
  };
  double na2[H], nc2[H];  // PF: the next pair's samples, in flight
  if constexpr (PF) load_pair(p0, na2, nc2);
  for (int64_t it = 0; it < pairs_per_worker; ++it) {
    const int64_t p = p0 + it;
    const bool active = p < npairs;
    const int64_t s0 = seg_begin + 2 * p;
    const bool has1 = active && (s0 + 1 < seg_end);
    double a2[H], c2[H];
    if constexpr (PF) {
#pragma unroll
      for (int k = 0; k < H; ++k) {
        a2[k] = na2[k];
        c2[k] = nc2[k];
      }
      if (it + 1 < pairs_per_worker) load_pair(p + 1, na2, nc2);
    } else {
      load_pair(p, a2, c2);
    }
    if constexpr (WMODE == 1) {
      const double *w = opaque_ptr(win) + t;
#pragma unroll
      for (int k = 0; k < E; ++k) wv[k] = w[k * G::T];
    } else if constexpr (WMODE == 2) {
      const int tw2 = opaque_int(t);
#pragma unroll
      for (int k = 0; k < E; ++k) wv[k] = wl[tw2 + k * G::T];
    }
    cd v[E];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      // an unpaired last segment (odd count) has a zero partner
      v[k] = {carry[k] * wv[k], has1 ? a2[k] * wv[k] : 0.0};
      v[H + k] = {a2[k] * wv[H + k], c2[k] * wv[H + k]};
    }
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = c2[k];
    if constexpr (PF)
      fft_regs<LOG2F, SPLIT, 2, LOG2E, 0, 0, const cd *, kPwLinear, false, NoEpi, kPwPrew>(
          v, opaque_int(t), (const cd *)twl, lre, lim, it == 0);
    else
      fft_regs<LOG2F, SPLIT, 1, LOG2E, 0, 0, const cd *, kPwLinear>(v, opaque_int(t), tw, lre,
                                                                    lim, it == 0);
    if (active) {
#pragma unroll
      for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
    }
  }
  if (p0 < npairs) {
    double *dst = partial + worker * G::N;
#pragma unroll
    for (int k = 0; k < E; ++k) dst[t + k * G::T] = acc[k];
  }
}

// Deterministic two-level reduction of the per-worker partial spectra:
// level 1 sums fixed chunks of workers per bin (grid: bins x chunks), level 2
// sums the chunk results in chunk order and adds into acc.
constexpr int kReduceChunk = 64;
__global__ void reduce_partials_l1(const double *__restrict__ partial, int64_t nworkers,
                                   int64_t F, double *__restrict__ chunk_sums) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (k >= F) return;
  const int64_t w0 = c * kReduceChunk;
  const int64_t w1 = w0 + kReduceChunk < nworkers ? w0 + kReduceChunk : nworkers;
  const double *p = partial + w0 * F + k;
  double s = 0.0;
  if (w1 - w0 == kReduceChunk) {
    // a full chunk: every load in flight at once, the sum in the same order
    double v[kReduceChunk];
#pragma unroll
    for (int i = 0; i < kReduceChunk; ++i) v[i] = p[i * F];
#pragma unroll
    for (int i = 0; i < kReduceChunk; ++i) s += v[i];
  } else {
    for (int64_t w = w0; w < w1; ++w, p += F) s += *p;
  }
  chunk_sums[c * F + k] = s;
}

__global__ void reduce_partials_l2(const double *__restrict__ chunk_sums, int64_t nchunks,
                                   int64_t F, double *__restrict__ acc) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= F) return;
  double s = 0.0;
  int64_t c = 0;
  for (; c + 8 <= nchunks; c += 8) {  // eight loads in flight, summed in order
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = chunk_sums[(c + i) * F + k];
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
  }
  for (; c < nchunks; ++c) s += chunk_sums[c * F + k];
  acc[k] += s;
}

// Materialised Pwelch path (any segment length): windowed, zero-padded real
// segments as complex rows.
// Materialised Pwelch: row r of buf = windowed segments seg0 + 2r (real part)
// and seg0 + 2r + 1 (imaginary part, zero past seg_end), zero-padded to flen
// — the same packed pairs as the fused kernels.
__global__ void segments_to_complex_kernel(const double *__restrict__ x, int64_t nfft,
                                           int64_t flen, int64_t stride, int64_t seg0,
                                           int64_t seg_end, int64_t nrows,
                                           const double *__restrict__ win,
                                           cd *__restrict__ buf) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nrows * flen) return;
  const int64_t r = tid / flen;
  const int64_t i = tid - r * flen;
  const int64_t s = seg0 + 2 * r;
  double a = 0.0, b = 0.0;
  if (i < nfft) {
    a = x[s * stride + i] * win[i];
    if (s + 1 < seg_end) b = x[(s + 1) * stride + i] * win[i];
  }
  buf[tid] = {a, b};
}

// partial[c][k] = sum over rows [c*rpp, (c+1)*rpp) of |buf[row][k]|^2
// (grid: bins x parts; reduced in fixed order by reduce_partials)
__global__ void power_partials_kernel(const cd *__restrict__ buf, int64_t nrows, int64_t flen,
                                      int64_t rpp, double *__restrict__ partial) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (k >= flen) return;
  const int64_t r0 = c * rpp, r1 = r0 + rpp < nrows ? r0 + rpp : nrows;
  double s = 0.0;
  for (int64_t r = r0; r < r1; ++r) {
    const cd z = buf[r * flen + k];
    s += z.x * z.x + z.y * z.y;
  }
  partial[c * flen + k] = s;
}

// ----------------------------------------------------------------------------
// FFT2 column pass on tiles of L rows x CW columns of a row-major matrix with
// row length C (fft/fft.go:138-147 without the gather/scatter copies). Thread
// (c, t), c fastest, owns column blockIdx.x*CW + c and tile elements
// j = t + k*T, so every load/store wave-instruction covers whole 128..1024-B
// row segments. Tile row j of row group q is matrix row q*step + j*stride
// (in and out separately), which expresses both steps of the four-step split
// R = R1*R2 used for long columns:
//   A: q = n2 < R2, rows n2 + R2*j, DFT_R1, times W_R^(n2*k1), in place;
//   B: q = k1 < R1, rows R2*k1 + j, DFT_R2, out rows k1 + R1*k2.
// TWIDDLE: 0 none; 1 times W_R^(q*j) (FFT2 four-step, q = row group);
// 2 times W_R^(col*j) (1-D four-step: the column is the n2 index).
template <int LOG2L, bool CONJ_IN, int TWIDDLE, bool CONJ_SCALE_OUT, int WGT = 256>
__global__ __launch_bounds__(WGT) void colfft_tile_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t C, int64_t in_step,
    int64_t in_stride, int64_t out_step, int64_t out_stride, const cd *__restrict__ twl,
    const cd *__restrict__ twr, int log2r, double scale, int64_t mat_stride, int64_t twn) {
  using G = Geo<LOG2L>;
  static_assert(G::T <= 256, "tile column length too large");
  in += (int64_t)blockIdx.z * mat_stride;
  out += (int64_t)blockIdx.z * mat_stride;
  constexpr int CW = WGT / G::T;
  __shared__ double lds[G::NPASS > 1 ? CW * G::N : 1];
  const int lt = threadIdx.x;
  const int c = lt & (CW - 1);
  const int t = lt / CW;
  const int64_t col = (int64_t)blockIdx.x * CW + c;
  const int64_t cl = col < C ? col : C - 1;  // partial last block: load a valid column
  const int64_t q = blockIdx.y;
  const cd *src = in + q * in_step * C + cl;
  cd v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; ++k) {
    v[k] = ld_nt(&src[(int64_t)(t + k * G::T) * in_stride * C]);
    if constexpr (CONJ_IN) v[k].y = -v[k].y;
  }
  fft_regs<LOG2L, true, false, 4, CW>(v, t, twl, lds + c, lds + c);
  if (col < C) {
    cd *dst = out + q * out_step * C + col;
    // W_R^(m*j), m = q (mode 1) or col (mode 2), for j = t + k*T: the base
    // W^(m*t) and the step W^(m*T) from the table, the rest by recurrence
    // (two table reads per thread instead of E scattered ones: for N = 2^20
    // the table is 16 MiB and the scattered reads missed L2)
    // table index m*j mod N: a mask for power-of-2 N, else twn = N (the
    // power-of-2-column mixed four-step)
    const int64_t mask = ((int64_t)1 << log2r) - 1;
    const int64_t m = TWIDDLE == 1 ? q : col;
    cd w = {1.0, 0.0}, wstep = {1.0, 0.0};
    if constexpr (TWIDDLE != 0) {
      w = twr[twn ? (m * t) % twn : (m * t) & mask];
      wstep = twr[twn ? (m * G::T) % twn : (m * G::T) & mask];
    }
#pragma unroll
    for (int k = 0; k < G::E; ++k) {
      const int64_t j = t + k * G::T;
      cd o = v[k];
      if constexpr (TWIDDLE != 0) {
        o = cmul(o, w);
        if (k + 1 < G::E) w = cmul(w, wstep);
      }
      if constexpr (CONJ_SCALE_OUT) o = {o.x * scale, -o.y * scale};
      st_nt(&dst[j * out_stride * C], o);
    }
  }
}

// The composed chirp-z's first column pass with the premultiply folded in
// (as colfft_tile_kernel, TWIDDLE 2, on a = x * chirp zero-padded to M =
// R * C): element (j, col) of the R x C view is a[j C + col] = x[e] chirp[e]
// for e = j C + col < n (x conjugated for an inverse), 0 past n (not loaded).
// x rows of n per transform (blockIdx.z), out rows of M.
template <int LOG2L, bool CONJ_IN, int WGT>
__global__ __launch_bounds__(WGT) void colfft_chirp_kernel(
    const cd *__restrict__ x, cd *__restrict__ out, int64_t C, int64_t n,
    const cd *__restrict__ chirp, const cd *__restrict__ twl, const cd *__restrict__ twr) {
  using G = Geo<LOG2L>;
  constexpr int CW = WGT / G::T;
  __shared__ double lds[G::NPASS > 1 ? CW * G::N : 1];
  const int lt = threadIdx.x;
  const int c = lt & (CW - 1);
  const int t = lt / CW;
  const int64_t col = (int64_t)blockIdx.x * CW + c;  // C is a multiple of CW
  const int64_t M = (int64_t)G::N * C;
  x += (int64_t)blockIdx.z * n;
  out += (int64_t)blockIdx.z * M;
  cd v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; ++k) {
    const int64_t e = (int64_t)(t + k * G::T) * C + col;
    cd a = {0.0, 0.0};
    if (e < n) {
      cd xe = ld_nt(&x[e]);
      if constexpr (CONJ_IN) xe.y = -xe.y;
      a = cmul(xe, chirp[e]);
    }
    v[k] = a;
  }
  fft_regs<LOG2L, true, false, 4, CW>(v, t, twl, lds + c, lds + c);
  // times W_M^(col j), j = t + k T: base and step from the table, then the
  // recurrence (as colfft_tile_kernel's TWIDDLE 2)
  cd w = twr[(col * t) & (M - 1)];
  const cd wstep = twr[(col * G::T) & (M - 1)];
  cd *dst = out + col;
#pragma unroll
  for (int k = 0; k < G::E; ++k) {
    st_nt(&dst[(int64_t)(t + k * G::T) * C], cmul(v[k], w));
    if (k + 1 < G::E) w = cmul(w, wstep);
  }
}

hipError_t launch_colfft_chirp(int log2l, bool conj_in, const cd *x, cd *out, int64_t C,
                               int64_t n, const cd *chirp, const cd *twl, const cd *twr,
                               int64_t batch, hipStream_t s) {
  if (batch < 1 || batch > 65535 || C <= 0 || (C & (C - 1)) || n < 1 || n > (C << log2l))
    return hipErrorInvalidValue;
#define GDSP_CCH(L, WGT)                                                                       \
  if (log2l == L) {                                                                            \
    constexpr int CW = WGT / Geo<L>::T;                                                        \
    if (C % CW) return hipErrorInvalidValue;                                                   \
    const dim3 grid((unsigned)(C / CW), 1, (unsigned)batch);                                   \
    if (conj_in)                                                                               \
      hipLaunchKernelGGL((colfft_chirp_kernel<L, true, WGT>), grid, dim3(WGT), 0, s, x, out, C, \
                         n, chirp, twl, twr);                                                  \
    else                                                                                       \
      hipLaunchKernelGGL((colfft_chirp_kernel<L, false, WGT>), grid, dim3(WGT), 0, s, x, out,  \
                         C, n, chirp, twl, twr);                                               \
    return hipGetLastError();                                                                  \
  }
  GDSP_CCH(7, 256)
  GDSP_CCH(8, 256)
  GDSP_CCH(9, 512)
  GDSP_CCH(10, 512)
#undef GDSP_CCH
  return hipErrorInvalidValue;
}

// Row pass of the two-pass four-steps (N = R*C, C = 2^LOG2C, 16 ... 1024): DFT_C
// along TPW = 4096 / C consecutive rows k1 of the R x C matrix Y (rows of the
// column pass's output), with the transpose X[k1 + R*k2] = Y[k1][k2] fused
// into the store. The workgroup stages its TPW rows through LDS so that
// every store wave-instruction writes, for 64 / TPW output indices k2, TPW
// consecutive k1: 16 * TPW-byte segments (4 KiB at C = 16 ... 64 B at 1024),
// where the row-per-workgroup form of this fusion wrote 16-B pieces R * 16 B
// apart (DESIGN.md §3 "Four-step": slower than a separate transpose). R is
// any length (log2r >= 0: a power of 2, shifts instead of divisions); `rows`
// = batch * R, the last workgroup's rows past it load a valid row and store
// nothing.
// MODE 0: X as is; 1: the inverse's conj and 1/N on the way out; 2 and 3
// (the composed chirp-z's two FFT_M, as transpose_blu_kernel's modes 1 and
// 2): 2 stores conj(X[k] tab[k]) (tab = b-hat), 3 stores the k < n outputs
// conj(X[k]) tab[k] (tab = chirp; inv: conj and scale) into rows of n.
template <int LOG2C, int MODE, bool P2R>
__global__ __launch_bounds__(256) void rowfft_t_kernel(const cd *__restrict__ in,
                                                       cd *__restrict__ out, int64_t R,
                                                       int log2r, int64_t rows,
                                                       const cd *__restrict__ tw, double scale,
                                                       const cd *__restrict__ tab, int64_t n,
                                                       int inv) {
  using G = Geo<LOG2C>;
  static_assert(G::WG == 256 && G::TPW >= 4, "rows of 16 to 1024");
  constexpr int TPW = G::TPW, T = G::T, E = G::E, C = G::N;
  constexpr int SD = C * (TPW + 1);  // staging: element a of row slot at a (TPW + 1) + slot
  __shared__ double lds[G::LDS_DOUBLES > SD ? G::LDS_DOUBLES : SD];
  const int lt = threadIdx.x, slot = lt / T, t = lt & (T - 1);
  const int64_t g0 = xcd_remap(blockIdx.x, gridDim.x) * TPW;
  const int64_t gl = g0 + slot < rows ? g0 + slot : rows - 1;
  const cd *src = in + gl * C;
  cd v[E];
#pragma unroll
  for (int k = 0; k < E; ++k) v[k] = ld_nt(&src[t + k * T]);
  double *lre = lds + slot * G::STRIDE;
  fft_regs<LOG2C, true, 0, 4>(v, t, tw, lre, lre);
  // store lane lt: row g0 + s (s fastest), outputs a = a0 + q T
  const int s = lt % TPW, a0 = lt / TPW;
  const int64_t g = g0 + s;
  const int64_t b = P2R ? g >> log2r : g / R;
  const int64_t k1 = g - b * R;
  cd *dst = out + b * (MODE == 3 ? n : R * C) + k1;
  const bool valid = g < rows;
  double re[E];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();  // the last exchange's (or the real parts') reads are done
#pragma unroll
    for (int k = 0; k < E; ++k) lds[(t + k * T) * (TPW + 1) + slot] = h ? v[k].y : v[k].x;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < E; ++q) {
      const double d = lds[(a0 + q * T) * (TPW + 1) + s];
      if (h == 0) {
        re[q] = d;
      } else if (valid) {
        cd o = {re[q], d};
        const int64_t kk = (int64_t)(a0 + q * T) * R;  // k - k1
        if constexpr (MODE == 1) o = {o.x * scale, -o.y * scale};
        if constexpr (MODE == 2) o = conjg(cmul(o, tab[kk + k1]));
        if constexpr (MODE == 3) {
          if (kk + k1 >= n) continue;
          o = cmul(conjg(o), tab[kk + k1]);
          if (inv) o = {o.x * scale, -o.y * scale};
        }
        st_nt(&dst[kk], o);
      }
    }
  }
}

hipError_t launch_rowfft_t(int log2c, int mode, const cd *in, cd *out, int64_t rows, int64_t R,
                           const cd *tw, double scale, hipStream_t s, const cd *tab, int64_t n,
                           bool inv) {
  if (rows <= 0 || R <= 0 || rows % R || mode < 0 || mode > 3 || (mode >= 2 && !tab))
    return hipErrorInvalidValue;
  int log2r = -1;
  if ((R & (R - 1)) == 0) {
    log2r = 0;
    while (((int64_t)1 << log2r) < R) ++log2r;
  }
#define GDSP_RTM(L, MO)                                                                          \
  do {                                                                                           \
    if (log2r >= 0)                                                                              \
      hipLaunchKernelGGL((rowfft_t_kernel<L, MO, true>), grid, dim3(256), 0, s, in, out, R,      \
                         log2r, rows, tw, scale, tab, n, (int)inv);                              \
    else                                                                                         \
      hipLaunchKernelGGL((rowfft_t_kernel<L, MO, false>), grid, dim3(256), 0, s, in, out, R,     \
                         log2r, rows, tw, scale, tab, n, (int)inv);                              \
  } while (0)
#define GDSP_RT(L)                                                  \
  if (log2c == L) {                                                 \
    constexpr int TPW = Geo<L>::TPW;                                \
    const int64_t nb = (rows + TPW - 1) / TPW;                      \
    if (nb > 0x7fffffff) return hipErrorInvalidValue;               \
    const dim3 grid((unsigned)nb);                                  \
    switch (mode) {                                                 \
      case 0: GDSP_RTM(L, 0); break;                                \
      case 1: GDSP_RTM(L, 1); break;                                \
      case 2: GDSP_RTM(L, 2); break;                                \
      default: GDSP_RTM(L, 3); break;                               \
    }                                                               \
    return hipGetLastError();                                       \
  }
  GDSP_RT(4)
  GDSP_RT(5)
  GDSP_RT(6)
  GDSP_RT(7)
  GDSP_RT(8)
  GDSP_RT(9)
  GDSP_RT(10)
#undef GDSP_RT
#undef GDSP_RTM
  return hipErrorInvalidValue;
}

// out[c*rows + r] = in[r*cols + c] through a 32x33 LDS tile (complex128),
// for `batch` consecutive matrices. Tiles of all matrices form one index
// space that a bounded grid strides over, so small matrices (the 210 x 210
// steps of a 44100-point four-step) do not cost a workgroup per tile.
// Options: conj + scale on the way out; times tw[r*c] (conjugated if
// tw_conj; the caller guarantees r*c < twn, as rows*cols = twn in the
// mixed four-step's W_N^(n2*k1) step).
template <int TR, int TC>
__global__ __launch_bounds__(256) void transpose_kernel(const cd *__restrict__ in,
                                                        cd *__restrict__ out, int64_t rows,
                                                        int64_t cols, int64_t batch,
                                                        int conj_scale, double scale,
                                                        const cd *__restrict__ tw, int64_t twn,
                                                        int tw_conj) {
  // TR rows x TC columns per tile: loads are TC * 16 B row segments, stores
  // TR * 16 B column segments; the LDS row stride TC + 1 is odd, so the
  // column reads are conflict-free
  constexpr int LY = 256 / TC, SY = 256 / TR;
  __shared__ cd tile[TR][TC + 1];
  const int64_t tiles_c = (cols + TC - 1) / TC;
  const int64_t tiles_r = (rows + TR - 1) / TR;
  const int64_t per = tiles_c * tiles_r;
  const int lx = threadIdx.x % TC, ly = threadIdx.x / TC;
  const int sx = threadIdx.x % TR, sy = threadIdx.x / TR;
  // (a register-prefetch variant, next tile's loads issued before this
  // tile's stores, measured 853 -> 1385 us on 2048 16x4096 matrices)
  for (int64_t tg = blockIdx.x; tg < per * batch; tg += gridDim.x) {
    const int64_t b = tg / per, tb = tg - b * per;
    const int64_t tr = tb / tiles_c, tc = tb - tr * tiles_c;
    const cd *src = in + b * rows * cols;
    cd *dst = out + b * rows * cols;
#pragma unroll
    for (int i = 0; i < TR; i += LY) {
      const int64_t r = tr * TR + ly + i, c = tc * TC + lx;
      if (r < rows && c < cols) tile[ly + i][lx] = ld_nt(&src[r * cols + c]);
    }
    __syncthreads();
    const int64_t r = tr * TR + sx;
    cd w = {1.0, 0.0}, ws = {1.0, 0.0};
    if (tw && r < rows) {  // W^(r*c) for c = c0 + sy + SY*i: two reads and a recurrence
      w = tw[r * (tc * TC + sy) % twn];
      ws = tw[r * SY % twn];
      if (tw_conj) {
        w.y = -w.y;
        ws.y = -ws.y;
      }
    }
#pragma unroll
    for (int i = 0; i < TC; i += SY) {
      const int64_t c = tc * TC + sy + i;
      if (r < rows && c < cols) {
        cd o = tile[sx][sy + i];
        if (tw) o = cmul(o, w);
        if (conj_scale) o = {o.x * scale, -o.y * scale};
        st_nt(&dst[c * rows + r], o);
      }
      if (tw && i + SY < TC) w = cmul(w, ws);
    }
    __syncthreads();
  }
}

// The final transpose of a composed chirp-z FFT_M (M = rows * cols, the
// four-step's output order), with the chirp-z step that follows folded in.
// Output index k = c * rows + r of matrix b:
//   mode 1: out[b*M + k] = conj(v * bhat[k])          (between the two FFTs)
//   mode 2: out[b*n + k] = conj(v) * chirp[k], k < n   (the result; an
//           inverse conjugates and scales it)
// Tiles of TR x TC as transpose_kernel; TR follows the row count (the
// four-step's column length, as short as 4 for a single-radix column split),
// so the load lanes of a tile are not mostly past the last row.
template <int TR, int TC>
__global__ __launch_bounds__(256) void transpose_blu_kernel(const cd *__restrict__ in,
                                                            cd *__restrict__ out, int64_t rows,
                                                            int64_t cols, int64_t batch, int mode,
                                                            int64_t n, const cd *__restrict__ tab,
                                                            int inv, double scale) {
  constexpr int LY = 256 / TC, SY = 256 / TR;
  __shared__ cd tile[TR][TC + 1];
  const int64_t M = rows * cols;
  const int64_t tiles_c = (cols + TC - 1) / TC, tiles_r = (rows + TR - 1) / TR;
  const int64_t per = tiles_c * tiles_r;
  const int lx = threadIdx.x % TC, ly = threadIdx.x / TC;
  const int sx = threadIdx.x % TR, sy = threadIdx.x / TR;
  for (int64_t tg = blockIdx.x; tg < per * batch; tg += gridDim.x) {
    const int64_t b = tg / per, tb = tg - b * per;
    const int64_t tr = tb / tiles_c, tc = tb - tr * tiles_c;
    const cd *src = in + b * M;
#pragma unroll
    for (int i = 0; i < TR; i += LY) {
      const int64_t r = tr * TR + ly + i, c = tc * TC + lx;
      if (r < rows && c < cols) tile[ly + i][lx] = ld_nt(&src[r * cols + c]);
    }
    __syncthreads();
    const int64_t r = tr * TR + sx;
#pragma unroll
    for (int i = 0; i < TC; i += SY) {
      const int64_t c = tc * TC + sy + i;
      if (r < rows && c < cols) {
        const int64_t k = c * rows + r;
        const cd v = tile[sx][sy + i];
        if (mode == 1) {
          st_nt(&out[b * M + k], conjg(cmul(v, tab[k])));
        } else if (k < n) {
          cd y = cmul(conjg(v), tab[k]);
          if (inv) y = {y.x * scale, -y.y * scale};
          st_nt(&out[b * n + k], y);
        }
      }
    }
    __syncthreads();
  }
}

__global__ void real_to_complex_kernel(const double *__restrict__ in, cd *__restrict__ out,
                                       int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = {in[i], 0.0};
}

// Composed Bluestein (n > 8192): premultiply into M-length rows.
__global__ void chirp_premul_kernel(const cd *__restrict__ in, cd *__restrict__ a, int64_t n,
                                    int64_t m, int64_t batch, const cd *__restrict__ chirp,
                                    int conj_in) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= batch * m) return;
  const int64_t g = tid / m, i = tid - g * m;
  cd v = {0.0, 0.0};
  if (i < n) {
    cd x = in[g * n + i];
    if (conj_in) x.y = -x.y;
    v = cmul(x, chirp[i]);
  }
  a[tid] = v;
}

// a = conj(a * bhat) (elementwise over batch rows of m)
__global__ void bhat_mul_conj_kernel(cd *__restrict__ a, int64_t m, int64_t batch,
                                     const cd *__restrict__ bhat) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= batch * m) return;
  a[tid] = conjg(cmul(a[tid], bhat[tid % m]));
}

__global__ void chirp_postmul_kernel(const cd *__restrict__ a, cd *__restrict__ out, int64_t n,
                                     int64_t m, int64_t batch, const cd *__restrict__ chirp,
                                     int inv, double scale) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= batch * n) return;
  const int64_t g = tid / n, k = tid - g * n;
  cd y = cmul(conjg(a[g * m + k]), chirp[k]);
  if (inv) y = {y.x * scale, -y.y * scale};
  out[tid] = y;
}

__global__ void pointwise_mul_kernel(const cd *__restrict__ a, const cd *__restrict__ b,
                                     cd *__restrict__ out, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = cmul(a[i], b[i]);
}

__global__ void scale_kernel(cd *__restrict__ a, int64_t count, double s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) a[i] = {a[i].x * s, a[i].y * s};
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ void fill_uniform_kernel(double *__restrict__ out, int64_t count, uint64_t seed,
                                    uint64_t offset) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t z = splitmix64(seed + (offset + (uint64_t)i + 1) * 0x9E3779B97F4A7C15ULL);
    out[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

// ============================================================================
// Host launchers
// ============================================================================
static inline unsigned blocks_for(int64_t work, int per) {
  return (unsigned)((work + per - 1) / per);
}

#define GDSP_LDS_CASE(L)                                                                   \
  case L:                                                                                  \
    if (load == LOAD_COMPLEX)                                                              \
      return inv ? launch_lds_s<L, true, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s) \
                 : launch_lds_s<L, false, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s); \
    return launch_lds_s<L, false, LOAD_REAL>(in, out, batch, tw, scale, split, s);

hipError_t launch_fft_lds(int log2n, bool inv, int load, bool split, const void *in, cd *out,
                          int64_t batch, const cd *tw, double scale, hipStream_t s) {
  if (load == LOAD_REAL && inv) return hipErrorInvalidValue;
  switch (log2n) {
    GDSP_LDS_CASE(1)
    GDSP_LDS_CASE(2)
    GDSP_LDS_CASE(3)
    GDSP_LDS_CASE(4)
    GDSP_LDS_CASE(5)
    GDSP_LDS_CASE(6)
    GDSP_LDS_CASE(7)
    GDSP_LDS_CASE(8)
    GDSP_LDS_CASE(9)
    GDSP_LDS_CASE(10)
    GDSP_LDS_CASE(11)
    case 12:  // fft_lds12.hip
      return launch_fft_lds12(inv, load, split, in, out, batch, tw, scale, s);
    GDSP_LDS_CASE(13)
    GDSP_LDS_CASE(14)
    default: return hipErrorInvalidValue;
  }
}

template <int LOG2M, bool INV>
static hipError_t launch_blu_t(const cd *in, cd *out, int64_t n, int64_t batch, const cd *twm,
                               const cd *chirp, const cd *bhat, double scale, hipStream_t s) {
  // M = 8192 / 16384: 32 points per thread (three passes, two exchanges, one
  // twiddle stage fewer; 254 VGPRs, 2 waves per SIMD) beat 16 (four passes,
  // 124 VGPRs, 4 waves per SIMD): chirp-z 3000 3.44 against 3.56 ms, primes
  // 4099..8191 (M = 16384) 2-5 %; round 3, with
  // the 16-point kernel held to 128 VGPRs (amdgpu_waves_per_eu: at 130 it ran
  // one 512-thread block per CU, 4.37 ms) and n-aware pruning (KN = 6):
  // 3.27-3.34 against 2.80 ms (scripts/archive/gpu_r03_e16.sh). The 32 points
  // alone hold 128 VGPRs, so a third wave per SIMD is out of reach: with the
  // exchange through half-size buffers (34 KiB of LDS) and 168 VGPRs the
  // kernel spills 206 registers, 6.20 against 2.62 ms (scripts/archive/gpu_r03_occ.sh)
  if constexpr (LOG2M == 13 || LOG2M == 14) {
    using G5 = Geo<LOG2M, 5>;
    const int64_t nb5 = (batch + G5::TPW - 1) / G5::TPW;
    if constexpr (LOG2M == 13) {
      // n <= 3072 = 12 T at M = 8192 (the BASELINE n = 3000): 12 of the 32
      // registers carry input and wanted output (2.87 -> 2.77 ms)
      if (n <= 12 * G5::T) {
        hipLaunchKernelGGL((bluestein_kernel<LOG2M, INV, true, 5, false, 12>), dim3((unsigned)nb5),
                           dim3(G5::WG), 0, s, in, out, n, batch, twm, chirp, bhat, scale,
                           (int64_t)0, 1);
        return hipGetLastError();
      }
    }
    hipLaunchKernelGGL((bluestein_kernel<LOG2M, INV, true, 5>), dim3((unsigned)nb5), dim3(G5::WG),
                       0, s, in, out, n, batch, twm, chirp, bhat, scale, (int64_t)0, 1);
    return hipGetLastError();
  }
  using G = Geo<LOG2M>;
  const int64_t nblk = (batch + G::TPW - 1) / G::TPW;
  hipLaunchKernelGGL((bluestein_kernel<LOG2M, INV, true>), dim3((unsigned)nblk), dim3(G::WG), 0,
                     s, in, out, n, batch, twm, chirp, bhat, scale, (int64_t)0, 1);
  return hipGetLastError();
}

// Output-split chirp-z on M = 8192 / 16384 (bluestein_kernel PARTS): `parts`
// launches' worth of blocks in one grid (the parts of a row adjacent), bhat holding
// parts * M.
template <int LOG2M>
static hipError_t launch_blu_parts_t(bool inv, const cd *in, cd *out, int64_t n, int64_t batch,
                                     int parts, int64_t kpart, const cd *twm, const cd *chirp,
                                     const cd *bhat, double scale, hipStream_t s) {
  using G = Geo<LOG2M, 5>;
  if (parts < 1 || parts > 65535 || kpart < 1 || kpart > G::N / 2 || n + kpart - 1 > G::N ||
      kpart * parts < n)
    return hipErrorInvalidValue;
  const int64_t nb = (batch + G::TPW - 1) / G::TPW * parts;
  if (nb > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nb);
  if (inv)
    hipLaunchKernelGGL((bluestein_kernel<LOG2M, true, true, 5, true>), grid, dim3(G::WG), 0, s,
                       in, out, n, batch, twm, chirp, bhat, scale, kpart, parts);
  else
    hipLaunchKernelGGL((bluestein_kernel<LOG2M, false, true, 5, true>), grid, dim3(G::WG), 0, s,
                       in, out, n, batch, twm, chirp, bhat, scale, kpart, parts);
  return hipGetLastError();
}

hipError_t launch_bluestein_parts(int log2m, bool inv, const cd *in, cd *out, int64_t n,
                                  int64_t batch, int parts, int64_t kpart, const cd *twm,
                                  const cd *chirp, const cd *bhat, double scale, hipStream_t s) {
  if (log2m == 13)
    return launch_blu_parts_t<13>(inv, in, out, n, batch, parts, kpart, twm, chirp, bhat, scale, s);
  if (log2m == 14)
    return launch_blu_parts_t<14>(inv, in, out, n, batch, parts, kpart, twm, chirp, bhat, scale, s);
  return hipErrorInvalidValue;
}

#define GDSP_BLU_CASE(L)                                                                     \
  case L:                                                                                    \
    return inv ? launch_blu_t<L, true>(in, out, n, batch, twm, chirp, bhat, scale, s)        \
               : launch_blu_t<L, false>(in, out, n, batch, twm, chirp, bhat, scale, s);

hipError_t launch_bluestein(int log2m, bool inv, const cd *in, cd *out, int64_t n,
                            int64_t batch, const cd *twm, const cd *chirp, const cd *bhat,
                            double scale, hipStream_t s) {
  switch (log2m) {
    GDSP_BLU_CASE(2)
    GDSP_BLU_CASE(3)
    GDSP_BLU_CASE(4)
    GDSP_BLU_CASE(5)
    GDSP_BLU_CASE(6)
    GDSP_BLU_CASE(7)
    GDSP_BLU_CASE(8)
    GDSP_BLU_CASE(9)
    GDSP_BLU_CASE(10)
    GDSP_BLU_CASE(11)
    GDSP_BLU_CASE(12)
    GDSP_BLU_CASE(13)
    GDSP_BLU_CASE(14)
    default: return hipErrorInvalidValue;
  }
}

template <int R>
static hipError_t launch_gpass_r(bool conj_in, int load, bool conj_scale_out, const void *in,
                                 cd *out, const cd *tw, int log2n, int log2ns, int64_t batch,
                                 double scale, hipStream_t s) {
  const int64_t work = batch * (((int64_t)1 << log2n) / R);
  const unsigned nb = blocks_for(work, 256);
#define GDSP_GP(CI, LD, CO)                                                                  \
  hipLaunchKernelGGL((stockham_global_pass<R, CI, LD, CO>), dim3(nb), dim3(256), 0, s, in, out, \
                     tw, log2n, log2ns, batch, scale)
  if (load == LOAD_REAL) {
    if (conj_scale_out) GDSP_GP(false, LOAD_REAL, true);
    else GDSP_GP(false, LOAD_REAL, false);
  } else if (conj_in) {
    if (conj_scale_out) GDSP_GP(true, LOAD_COMPLEX, true);
    else GDSP_GP(true, LOAD_COMPLEX, false);
  } else {
    if (conj_scale_out) GDSP_GP(false, LOAD_COMPLEX, true);
    else GDSP_GP(false, LOAD_COMPLEX, false);
  }
#undef GDSP_GP
  return hipGetLastError();
}

hipError_t launch_global_pass(int radix, bool conj_in, int load, bool conj_scale_out,
                              const void *in, cd *out, const cd *tw, int log2n, int log2ns,
                              int64_t batch, double scale, hipStream_t s) {
  switch (radix) {
    case 2: return launch_gpass_r<2>(conj_in, load, conj_scale_out, in, out, tw, log2n, log2ns, batch, scale, s);
    case 4: return launch_gpass_r<4>(conj_in, load, conj_scale_out, in, out, tw, log2n, log2ns, batch, scale, s);
    case 8: return launch_gpass_r<8>(conj_in, load, conj_scale_out, in, out, tw, log2n, log2ns, batch, scale, s);
    case 16: return launch_gpass_r<16>(conj_in, load, conj_scale_out, in, out, tw, log2n, log2ns, batch, scale, s);
    default: return hipErrorInvalidValue;
  }
}

template <int LOG2F>
static hipError_t launch_pw_t(const double *x, int64_t nfft, int64_t stride, int64_t seg_begin,
                              int64_t seg_end, int64_t ppw, int64_t nworkers, const double *win,
                              const cd *tw, double *partial, hipStream_t s) {
  using G = Geo<LOG2F>;
  const int64_t nblk = (nworkers + G::TPW - 1) / G::TPW;
  hipLaunchKernelGGL((pwelch_kernel<LOG2F, true>), dim3((unsigned)nblk), dim3(G::WG), 0, s, x,
                     nfft, stride, seg_begin, seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

template <int LOG2F, int WMODE = 2, int MINW = 1, int LOG2E = 4, bool SPLIT = true,
          bool PF = false>
static hipError_t launch_pwh_t(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                               int64_t nworkers, const double *win, const cd *tw, double *partial,
                               hipStream_t s) {
  using G = Geo<LOG2F, LOG2E>;
  if (G::TPW != Geo<LOG2F>::TPW) return hipErrorInvalidValue;  // workers per block
  const int64_t nblk = (nworkers + G::TPW - 1) / G::TPW;
  hipLaunchKernelGGL((pwelch_half_kernel<LOG2F, WMODE, MINW, LOG2E, SPLIT, PF>), dim3((unsigned)nblk), dim3(G::WG), 0, s,
                     x, seg_begin, seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

hipError_t launch_pwelch_half(int log2f, const double *x, int64_t seg_begin, int64_t seg_end,
                              int64_t ppw, int64_t nworkers, const double *win, const cd *tw,
                              double *partial, hipStream_t s) {
  // (F = 64 ... 2048 run on the wave kernels, pwelch_wave.hip, since round 5)
  switch (log2f) {
    case 5: return launch_pwh_t<5>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 12: {
      // the BASELINE configuration, on the row kernel: 2.81-2.84 against
      // 3.13-3.14 ms for pwelch_half_kernel<12> (which with twiddle bases in
      // LDS and the next pair prefetched had gone 3.16 -> 3.11 ms)
      return launch_pwelch_row4096(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    }
    // (F = 8192 held to four waves per SIMD with the window read from L1/L2,
    // two workgroups per CU at 128 VGPRs and 62 spilled: 1.64-1.65 against
    // 1.16-1.17 ms per 2^28 samples; scripts/archive/gpu_r05_h13.sh)
    case 13: return launch_pwh_t<13>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    // F = 16384: the exchange buffer alone takes 136 KiB, so the window is
    // re-read from L1/L2 instead of living in LDS
    case 14: {
      // 32 points per thread (512 threads): 2.25-2.27 against 2.37-2.40 ms at
      // 2^28 samples for 16 (1024 threads); both spill (re-measured at the end
      // of round 5 on the linear exchange slots: 256 VGPRs, 123 spilled, two
      // waves per SIMD, 1.91 ms, against 128 VGPRs, 67 spilled, four waves,
      // 2.00-2.01 ms; scripts/archive/gpu_r05_h16.sh)
      return launch_pwh_t<14, 1, 1, 5>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    }
    default: return hipErrorInvalidValue;
  }
}

int pwelch_workers_per_block(int log2f) {
  switch (log2f) {
#define GDSP_PWT(L) case L: return Geo<L>::TPW;
    GDSP_PWT(4) GDSP_PWT(5) GDSP_PWT(6) GDSP_PWT(7) GDSP_PWT(8) GDSP_PWT(9) GDSP_PWT(10)
    GDSP_PWT(11) GDSP_PWT(12) GDSP_PWT(13) GDSP_PWT(14)
#undef GDSP_PWT
    default: return 1;
  }
}

hipError_t launch_pwelch(int log2f, const double *x, int64_t nfft, int64_t stride,
                         int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                         const double *win, const cd *tw, double *partial, hipStream_t s) {
  // (F = 64 ... 2048 run on the wave kernels; 4096 with Pad = NFFT on the
  // row kernel's general-overlap form, pwelch_row.hip)
  switch (log2f) {
#define GDSP_PWC(L) \
  case L: return launch_pw_t<L>(x, nfft, stride, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    GDSP_PWC(4) GDSP_PWC(5) GDSP_PWC(12) GDSP_PWC(13) GDSP_PWC(14)
#undef GDSP_PWC
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_reduce_partials(const double *partial, int64_t nworkers, int64_t F, double *acc,
                                  double *scratch, hipStream_t s) {
  // scratch: ceil(nworkers / kReduceChunk) * F doubles
  const int64_t nchunks = (nworkers + kReduceChunk - 1) / kReduceChunk;
  hipLaunchKernelGGL(reduce_partials_l1, dim3(blocks_for(F, 256), (unsigned)nchunks), dim3(256), 0,
                     s, partial, nworkers, F, scratch);
  hipLaunchKernelGGL(reduce_partials_l2, dim3(blocks_for(F, 256)), dim3(256), 0, s, scratch,
                     nchunks, F, acc);
  return hipGetLastError();
}

int64_t reduce_scratch_doubles(int64_t nworkers, int64_t F) {
  return ((nworkers + kReduceChunk - 1) / kReduceChunk) * F;
}

hipError_t launch_segments_to_complex(const double *x, int64_t nfft, int64_t flen, int64_t stride,
                                      int64_t seg0, int64_t seg_end, int64_t nrows,
                                      const double *win, cd *buf, hipStream_t s) {
  hipLaunchKernelGGL(segments_to_complex_kernel, dim3(blocks_for(nrows * flen, 256)), dim3(256),
                     0, s, x, nfft, flen, stride, seg0, seg_end, nrows, win, buf);
  return hipGetLastError();
}

hipError_t launch_power_partials(const cd *buf, int64_t nrows, int64_t flen, int64_t rpp,
                                 double *partial, hipStream_t s) {
  const int64_t parts = (nrows + rpp - 1) / rpp;
  if (parts > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(power_partials_kernel, dim3(blocks_for(flen, 256), (unsigned)parts),
                     dim3(256), 0, s, buf, nrows, flen, rpp, partial);
  return hipGetLastError();
}

template <int LOG2L, int WGT>
static hipError_t launch_colfft_w(bool conj_in, int twiddle, bool conj_scale_out, const cd *in,
                                  cd *out, int64_t C, int64_t ngroups, int64_t in_step,
                                  int64_t in_stride, int64_t out_step, int64_t out_stride,
                                  const cd *twl, const cd *twr, int log2r, double scale,
                                  int64_t batch, int64_t mat_stride, int64_t twn, hipStream_t s) {
  constexpr int CW = WGT / Geo<LOG2L>::T;
  const dim3 grid((unsigned)((C + CW - 1) / CW), (unsigned)ngroups, (unsigned)batch);
#define GDSP_CF(A, B, D)                                                                      \
  hipLaunchKernelGGL((colfft_tile_kernel<LOG2L, A, B, D, WGT>), grid, dim3(WGT), 0, s, in, out, C, \
                     in_step, in_stride, out_step, out_stride, twl, twr, log2r, scale,         \
                     mat_stride, twn)
  if (twiddle == 1) {
    if (conj_in) GDSP_CF(true, 1, false);
    else GDSP_CF(false, 1, false);
  } else if (twiddle == 2) {
    if (conj_in) GDSP_CF(true, 2, false);
    else GDSP_CF(false, 2, false);
  } else if (conj_in) {
    if (conj_scale_out) GDSP_CF(true, 0, true);
    else GDSP_CF(true, 0, false);
  } else {
    if (conj_scale_out) GDSP_CF(false, 0, true);
    else GDSP_CF(false, 0, false);
  }
#undef GDSP_CF
  return hipGetLastError();
}


template <int LOG2L>
static hipError_t launch_colfft_t(bool conj_in, int twiddle, bool conj_scale_out, const cd *in,
                                  cd *out, int64_t C, int64_t ngroups, int64_t in_step,
                                  int64_t in_stride, int64_t out_step, int64_t out_stride,
                                  const cd *twl, const cd *twr, int log2r, double scale,
                                  int64_t batch, int64_t mat_stride, int64_t twn, hipStream_t s) {
  // 512-column-thread tiles for 512-point columns: 16 columns = 256-B row
  // segments instead of 128 (FFTN 512^3: 2.41-2.51 -> 2.28 ms); shorter
  // columns keep 256 threads (their segments are already 512 B - 1 KiB, and
  // 512 threads measured slower on the FFT2 8192^2 column tiles)
  if constexpr (LOG2L >= 9) {
    return launch_colfft_w<LOG2L, 512>(conj_in, twiddle, conj_scale_out, in, out, C, ngroups,
                                       in_step, in_stride, out_step, out_stride, twl, twr, log2r,
                                       scale, batch, mat_stride, twn, s);
  }
  return launch_colfft_w<LOG2L, 256>(conj_in, twiddle, conj_scale_out, in, out, C, ngroups,
                                     in_step, in_stride, out_step, out_stride, twl, twr, log2r,
                                     scale, batch, mat_stride, twn, s);
}

hipError_t launch_colfft(int log2l, bool conj_in, int twiddle, bool conj_scale_out, const cd *in,
                         cd *out, int64_t C, int64_t ngroups, int64_t in_step, int64_t in_stride,
                         int64_t out_step, int64_t out_stride, const cd *twl, const cd *twr,
                         int log2r, double scale, int64_t batch, int64_t mat_stride,
                         hipStream_t s, int64_t twn) {
  if (twiddle && conj_scale_out) return hipErrorInvalidValue;
  if (batch < 1 || batch > 65535) return hipErrorInvalidValue;
  switch (log2l) {
#define GDSP_CFC(L)                                                                           \
  case L:                                                                                     \
    return launch_colfft_t<L>(conj_in, twiddle, conj_scale_out, in, out, C, ngroups, in_step, \
                              in_stride, out_step, out_stride, twl, twr, log2r, scale, batch, \
                              mat_stride, twn, s);
    GDSP_CFC(4) GDSP_CFC(5) GDSP_CFC(6) GDSP_CFC(7) GDSP_CFC(8) GDSP_CFC(9)
    GDSP_CFC(10)  // (beyond kColMaxLog2: the two-pass four-step's 2^20 columns only)
#undef GDSP_CFC
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_transpose(const cd *in, cd *out, int64_t rows, int64_t cols, hipStream_t s,
                            int64_t batch, bool conj_scale, double scale, const cd *tw,
                            int64_t twn, bool tw_conj) {
  if (batch < 1 || batch > 65535) return hipErrorInvalidValue;
  if (tw && (rows - 1) * (cols - 1) >= twn) return hipErrorInvalidValue;  // r*c < twn
  // tile shape (rows x columns): 32 x 64 for large batches, 32 x 32 below
  // 2^22 elements, where twice the tiles spread better over the CUs (one
  // 2^20 transform: 8.3 against 10.3 us); 64 x 64 measured 1.156 against
  // 0.873 ms at 10^6
  const bool small = rows * cols * batch < ((int64_t)1 << 22);
  const int tr = 32, tc = small ? 32 : 64;
  const int64_t tiles = ((rows + tr - 1) / tr) * ((cols + tc - 1) / tc) * batch;
  const int64_t cap = 256 * 32;  // 32 tile-loop workgroups per CU
  const unsigned nb = (unsigned)(tiles < cap ? tiles : cap);
  if (small)
    hipLaunchKernelGGL((transpose_kernel<32, 32>), dim3(nb), dim3(256), 0, s, in, out, rows, cols,
                       batch, (int)conj_scale, scale, tw, twn, (int)tw_conj);
  else
    hipLaunchKernelGGL((transpose_kernel<32, 64>), dim3(nb), dim3(256), 0, s, in, out, rows, cols,
                       batch, (int)conj_scale, scale, tw, twn, (int)tw_conj);
  return hipGetLastError();
}

hipError_t launch_transpose_blu(const cd *in, cd *out, int64_t rows, int64_t cols, int64_t batch,
                                int mode, int64_t n, const cd *tab, bool inv, double scale,
                                hipStream_t s) {
  if (batch < 1 || batch > 65535 || (mode != 1 && mode != 2)) return hipErrorInvalidValue;
  if (mode == 2 && n > rows * cols) return hipErrorInvalidValue;
  const int64_t cap = 256 * 32;
#define GDSP_TBLU(TR, TC)                                                                    \
  do {                                                                                       \
    const int64_t tiles = ((rows + TR - 1) / TR) * ((cols + TC - 1) / TC) * batch;          \
    const unsigned nb = (unsigned)(tiles < cap ? tiles : cap);                               \
    hipLaunchKernelGGL((transpose_blu_kernel<TR, TC>), dim3(nb), dim3(256), 0, s, in, out,   \
                       rows, cols, batch, mode, n, tab, (int)inv, scale);                    \
  } while (0)
  if (rows <= 8) GDSP_TBLU(8, 256);
  else if (rows <= 16) GDSP_TBLU(16, 128);
  else GDSP_TBLU(32, 64);
#undef GDSP_TBLU
  return hipGetLastError();
}

hipError_t launch_real_to_complex(const double *in, cd *out, int64_t count, hipStream_t s) {
  hipLaunchKernelGGL(real_to_complex_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, s, in,
                     out, count);
  return hipGetLastError();
}

hipError_t launch_chirp_premul(const cd *in, cd *a, int64_t n, int64_t m, int64_t batch,
                               const cd *chirp, bool conj_in, hipStream_t s) {
  hipLaunchKernelGGL(chirp_premul_kernel, dim3(blocks_for(batch * m, 256)), dim3(256), 0, s, in,
                     a, n, m, batch, chirp, (int)conj_in);
  return hipGetLastError();
}

hipError_t launch_bhat_mul_conj(cd *a, int64_t m, int64_t batch, const cd *bhat, hipStream_t s) {
  hipLaunchKernelGGL(bhat_mul_conj_kernel, dim3(blocks_for(batch * m, 256)), dim3(256), 0, s, a, m,
                     batch, bhat);
  return hipGetLastError();
}

hipError_t launch_chirp_postmul(const cd *a, cd *out, int64_t n, int64_t m, int64_t batch,
                                const cd *chirp, bool inv, double scale, hipStream_t s) {
  hipLaunchKernelGGL(chirp_postmul_kernel, dim3(blocks_for(batch * n, 256)), dim3(256), 0, s, a,
                     out, n, m, batch, chirp, (int)inv, scale);
  return hipGetLastError();
}

hipError_t launch_pointwise_mul(const cd *a, const cd *b, cd *out, int64_t count, hipStream_t s) {
  hipLaunchKernelGGL(pointwise_mul_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, s, a, b,
                     out, count);
  return hipGetLastError();
}

hipError_t launch_scale(cd *a, int64_t count, double sc, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(count, 256)), dim3(256), 0, s, a, count, sc);
  return hipGetLastError();
}

hipError_t launch_fill_uniform(double *out, int64_t count, uint64_t seed, uint64_t offset,
                               hipStream_t s) {
  int64_t nb = (count + 255) / 256;
  if (nb > 8192) nb = 8192;
  if (nb < 1) nb = 1;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3((unsigned)nb), dim3(256), 0, s, out, count, seed,
                     offset);
  return hipGetLastError();
}

}  // namespace gdsp
