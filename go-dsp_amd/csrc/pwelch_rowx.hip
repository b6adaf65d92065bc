// pwelch_rowx.hip — experimental variants of pwelch_row_kernel<12> (the
// BASELINE Pwelch: NFFT 4096, Noverlap 2048, Hann) for occupancy: the window
// recomputed in registers instead of an LDS table, with or without the next
// pair's samples prefetched into registers, at 2 or 3 waves per SIMD.
#include "fft_device.hpp"
#include "launch.hpp"

namespace gdsp {

// The symmetric Hann window of window.go:62-76, w_n = 0.5 (1 - cos(2 pi n /
// (L - 1))), at a thread's elements n = t + k T (k = 0 .. E-1) by the
// three-term recurrence c_(k+1) = 2 cos(T theta) c_k - c_(k-1) from c_0, c_1
// (per-thread constants computed once per kernel): no table, one FMA per
// element plus the 0.5 - 0.5 c.
struct HannRec {
  double c0, c1, k2;  // cos(theta t), cos(theta (t + T)), 2 cos(theta T)
  template <int E>
  __device__ __forceinline__ void weights(double (&w)[E]) const {
    double cm = c0, c = c1;
    w[0] = fma(-0.5, cm, 0.5);
    if constexpr (E > 1) w[1] = fma(-0.5, c, 0.5);
#pragma unroll
    for (int k = 2; k < E; ++k) {
      const double cn = fma(k2, c, -cm);
      cm = c;
      c = cn;
      w[k] = fma(-0.5, c, 0.5);
    }
  }
};

// WIN 0: LDS table (as pwelch_row_kernel); 1: Hann in registers (HannRec)
// PREF: the next pair's samples loaded into registers during this pair
// NOCARRY: no samples kept across pairs: each pair loads its 3 rows-blocks
// (the first one an L2 hit: the previous pair's last block) at its start
// SPLIT: real and imaginary parts through one N-double buffer in turn (four
// barriers per exchange); false: two buffers, two barriers per exchange
template <int LOG2F, int WIN, bool PREF, int WPE, bool NOCARRY = false, bool SPLIT = true>
__global__ __launch_bounds__((Geo<LOG2F, 4>::WG)) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void pwelch_rowx_kernel(const double *__restrict__ x, int64_t seg_begin, int64_t seg_end,
                        int64_t pairs_per_worker, const double *__restrict__ win,
                        const cd *__restrict__ tw, double *__restrict__ partial) {
  using G = Geo<LOG2F, 4>;
  static_assert(G::TPW == 1, "one worker per workgroup");
  constexpr int E = G::E, H = E / 2, T = G::T;
  constexpr int64_t STRIDE = G::N / 2;
  constexpr int XD = SPLIT ? G::LDS_DOUBLES : 2 * G::LDS_DOUBLES;
  __shared__ double lds[XD + (WIN == 0 ? G::N : 0)];
  double *const lx = lds;
  double *const ly = SPLIT ? lds : lds + G::LDS_DOUBLES;
  double *const wl = lds + XD;
  const int t = threadIdx.x;
  const uint32_t lane = (uint32_t)t;
  HannRec hr{};
  if constexpr (WIN == 0) {
    for (int i = t; i < G::N; i += G::WG) wl[i] = win[i];
  } else {
    const double th = 2.0 * M_PI / (double)(G::N - 1);
    hr.c0 = cos(th * (double)t);
    hr.c1 = cos(th * (double)(t + T));
    hr.k2 = 2.0 * cos(th * (double)T);
  }
  using RT = RegTw<G::NPASS>;
  RT rtw;
#pragma unroll
  for (int p = 0; p < G::NPASS; ++p) rtw.base[p] = {1.0, 0.0};
  if constexpr (G::NPASS > 1) rtw.base[1] = pass_base<G::N, G::EMAX, G::ns(1)>(tw, t);
  if constexpr (G::NPASS > 2) rtw.base[2] = pass_base<G::N, G::EMAX, G::ns(2)>(tw, t);
  if constexpr (G::NPASS > 3) rtw.base[3] = pass_base<G::N, G::EMAX, G::ns(3)>(tw, t);
  if constexpr (WIN == 0) __syncthreads();
  const int64_t npairs = (seg_end - seg_begin + 1) / 2;
  const int64_t nfull = (seg_end - seg_begin) / 2;
  const int64_t p0 = (int64_t)blockIdx.x * pairs_per_worker;
  const int64_t pend = p0 + pairs_per_worker < npairs ? p0 + pairs_per_worker : npairs;
  const int64_t fend = pend < nfull ? pend : nfull;
  if (p0 >= pend) return;
  auto row = [&](int64_t p, int r) -> const double * {
    return opaque_ptr(x + (seg_begin + 2 * p) * STRIDE + (int64_t)r * T);
  };
  double carry[H], a2[H], c2[H];
  if constexpr (!NOCARRY) {
#pragma unroll
    for (int k = 0; k < H; ++k) carry[k] = row(p0, k)[lane];
  }
  auto issue = [&](int64_t p) {
    const int cr = p < nfull ? E : H;
#pragma unroll
    for (int k = 0; k < H; ++k) {
      a2[k] = row(p, H + k)[lane];
      c2[k] = row(p, cr + k)[lane];
    }
  };
  if constexpr (PREF) issue(p0);
  double acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.0;
  auto pair = [&](int64_t p, bool first, bool partner) {
    const int tt = opaque_int(t);
    if constexpr (NOCARRY) {
#pragma unroll
      for (int k = 0; k < H; ++k) carry[k] = row(p, k)[lane];
    }
    if constexpr (!PREF) issue(p);
    cd v[E];
    double wv[E];
    if constexpr (WIN == 0) {
#pragma unroll
      for (int k = 0; k < E; ++k) wv[k] = wl[tt + k * T];
    }
#pragma unroll
    for (int k = 0; k < H; ++k) {
      v[k] = {carry[k], partner ? a2[k] : 0.0};
      v[H + k] = {a2[k], partner ? c2[k] : 0.0};
    }
    if constexpr (!NOCARRY) {
#pragma unroll
      for (int k = 0; k < H; ++k) carry[k] = c2[k];
    }
    if constexpr (PREF)
      if (p + 1 < pend) issue(p + 1);
    RT rl = rtw;
#pragma unroll
    for (int q = 1; q < G::NPASS; ++q) rl.base[q] = opaque_cd(rl.base[q]);
    if constexpr (WIN == 1) {
      // laundered per pair: the weights are recomputed inside the loop, not
      // hoisted into 32 registers for the kernel's lifetime
      HannRec h = hr;
      const cd c01 = opaque_cd({h.c0, h.c1});
      h.c0 = c01.x;
      h.c1 = c01.y;
      h.weights<E>(wv);
    }
#pragma unroll
    for (int k = 0; k < E; ++k) v[k] = {v[k].x * wv[k], v[k].y * wv[k]};
    fft_regs<LOG2F, SPLIT, 2, 4, 0, 0, RT, 2, false, NoEpi, 0, 16>(v, tt, rl, lx, ly, first);
#pragma unroll
    for (int k = 0; k < E; ++k) acc[k] = fma(v[k].y, v[k].y, fma(v[k].x, v[k].x, acc[k]));
  };
  int64_t p = p0;
  for (; p < fend; ++p) pair(p, p == p0, true);
  if (p < pend) pair(p, p == p0, false);
  double *dst = partial + blockIdx.x * (int64_t)G::N;
#pragma unroll
  for (int k = 0; k < E; ++k) dst[t + k * T] = acc[k];
}

template <int WIN, bool PREF, int WPE, bool NOCARRY = false, bool SPLIT = true>
hipError_t launch_rowx(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                       int64_t nworkers, const double *win, const cd *tw, double *partial,
                       hipStream_t s) {
  hipLaunchKernelGGL((pwelch_rowx_kernel<12, WIN, PREF, WPE, NOCARRY, SPLIT>), dim3((unsigned)nworkers),
                     dim3(Geo<12>::WG), 0, s, x, seg_begin, seg_end, ppw, win, tw, partial);
  return hipGetLastError();
}

// variant: 1 = Hann in registers + prefetch, 2 waves; 2 = Hann in registers,
// no prefetch, 3 waves; 3 = LDS window, no prefetch, 2 waves; 4 = Hann in
// registers + prefetch, 3 waves; 5 / 6 = Hann in registers, no carry, no
// prefetch, 3 / 2 waves; 7 = LDS window, no carry, no prefetch, 2 waves;
// 8 = Hann in registers + prefetch, two exchange buffers, 2 waves
hipError_t launch_pwelch_rowx4096(int variant, const double *x, int64_t seg_begin,
                                  int64_t seg_end, int64_t ppw, int64_t nworkers,
                                  const double *win, const cd *tw, double *partial,
                                  hipStream_t s) {
  switch (variant) {
    case 1: return launch_rowx<1, true, 2>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 2: return launch_rowx<1, false, 3>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 3: return launch_rowx<0, false, 2>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 4: return launch_rowx<1, true, 3>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 5: return launch_rowx<1, false, 3, true>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 6: return launch_rowx<1, false, 2, true>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 7: return launch_rowx<0, false, 2, true>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
    case 8: return launch_rowx<1, true, 2, false, false>(x, seg_begin, seg_end, ppw, nworkers, win, tw, partial, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace gdsp
