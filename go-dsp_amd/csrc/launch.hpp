// launch.hpp — host launchers of the gfx950 kernels (fft_kernels.hip), used by
// the C ABI layer (gdsp_api.hip). Internal to libgdspfft.
#pragma once
#ifndef __HIPCC_RTC__  // the device-side parts are also compiled by hipRTC (mixed_jit.cpp)
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

namespace gdsp {

struct cd;

enum { LOAD_COMPLEX = 0, LOAD_REAL = 1 };

// largest power-of-2 length handled by the one-kernel LDS transform / the
// fused Bluestein kernel (M) / the fused Pwelch kernel
constexpr int kMaxLdsLog2 = 14;

// Mixed-radix one-kernel transform (fft_mixed.hip): n = prod of the radices
// in `codes` (5 bits per pass, radices 2,3,4,5,7,8,11,13,16 in the runtime-radix
// kernels, also 6,9,10,12,15,20,25 in the compiled specialisations), n <= kMixedMax
// (kMixedSpecMax for a specialisation).
struct MixedDesc {
  uint64_t codes;
  int n, npass, t1, tpw;
};
constexpr int kMixedMax = 4096;
// compiled specialisations (fft_specs*.hip) reach this far (re/im exchange)
constexpr int kMixedSpecMax = 8192;

#ifndef __HIPCC_RTC__

// ---- configuration (gdsp_api.hip) ------------------------------------------
// Deployment knobs: the only process environment the library reads.
enum Knob {
  KNOB_DEVICES,          // GDSP_DEVICES: initial multi-device set ("0,1,2" / "all")
  KNOB_MULTI_MIN_BYTES,  // GDSP_MULTI_MIN_BYTES: split threshold of host calls
  KNOB_JIT,              // GDSP_JIT=0: no runtime-compiled specialisations
  KNOB_JIT_INCLUDE,      // GDSP_JIT_INCLUDE: header directory for hipRTC
  KNOB_JIT_CACHE,        // GDSP_JIT_CACHE: code-object cache directory
  KNOB_JIT_VERBOSE,      // GDSP_JIT_VERBOSE: log runtime compilations
  KNOB_XDG_CACHE_HOME,   // default cache location
  KNOB_HOME,
};
const char *knob(Knob k);
// Algorithm selection flags (gdsp_set_algorithm, include/gdsp_fft.h) in
// force when a plan is built.
unsigned algo_flags();

hipError_t launch_fft_lds(int log2n, bool inv, int load, bool split, const void *in, cd *out,
                          int64_t batch, const cd *tw, double scale, hipStream_t s);
// the N = 4096 case of launch_fft_lds (fft_lds12.hip)
hipError_t launch_fft_lds12(bool inv, int load, bool split, const void *in, cd *out, int64_t batch,
                            const cd *tw, double scale, hipStream_t s);
// fused Pwelch over a mixed-radix segment length d.n = max(pad, nfft) with
// d.npass >= 2 (fft_mixed.hip); same partial layout as launch_pwelch
hipError_t launch_pwelch_mixed(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,
                               int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                               const double *win, const cd *tw, double *partial, hipStream_t s);
// fused Pwelch with wave-resident transforms (pwelch_wave.hip), 64 <= F <= 1024:
// the launch geometry (groups of pairs per wave, workgroups, partial rows)
bool pwelch_wave_applies(int log2f);
void pwelch_wave_geometry(int log2f, bool half, int64_t nsegs, int64_t *gpw, int64_t *nblk,
                          int64_t *nrows);
hipError_t launch_pwelch_wave(int log2f, bool half, const double *x, int64_t nfft, int64_t stride,
                              int64_t seg_begin, int64_t seg_end, int64_t gpw, int64_t nblk,
                              const double *win, const cd *tw, double *partial, hipStream_t s);
// fused Pwelch on a compiled specialisation (d = the plan's specialisation
// descriptor, d.n = max(pad, nfft)); workers per block, 0 if d is none or
// its kernel cannot stage a pair of span = stride + nfft samples
int pwelch_fixed_workers_per_block(const MixedDesc &d, int64_t span);
hipError_t launch_pwelch_fixed(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,
                               int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                               const double *win, const cd *tw, double *partial, hipStream_t s);
// runtime-compiled specialisations (mixed_jit.hip, hipRTC): a radix list for
// a smooth n <= kMixedSpecMax without a compiled one, and its kernels
struct JitSpec;
bool jit_enabled();
bool jit_radices(int n, int *rad, int *npass);
JitSpec *jit_spec_build(int dev, const int *rad, int np, int n);  // nullptr: not built
// colfixed_kernel (mixed_fixed.hpp) for the column length prod(rad)
struct JitCol;
JitCol *jit_col_build(int dev, const int *rad, int np);  // nullptr: not built
// rowt_fixed_kernel (mixed_fixed.hpp) for the row length prod(rad): rows of
// a two-pass mixed four-step with the transpose in their store
struct JitRowT;
JitRowT *jit_rowt_build(int dev, const int *rad, int np);  // nullptr: not built
hipError_t jit_launch_rowt(const JitRowT *j, bool conj_scale_out, const cd *in, cd *out,
                           int64_t rows, int64_t L, const cd *tw, double scale, hipStream_t s);
hipError_t jit_launch_col(const JitCol *j, bool conj_in, const cd *in, cd *out, int64_t C,
                          int64_t n, int64_t batch, const cd *tw, const cd *twn, hipStream_t s);
hipError_t jit_launch_fft(const JitSpec *j, bool inv, int load, const void *in, cd *out,
                          int64_t batch, const cd *tw, double scale, hipStream_t s);
int jit_pw_tpw(const JitSpec *j, int64_t span);  // as pwelch_fixed_workers_per_block
// rader_fixed_kernel (mixed_fixed.hpp): a prime P = prod(rad) + 1 by Rader's
// algorithm on the inlined mixed-radix chain of its N = P - 1
struct JitRader;
JitRader *jit_rader_build(int dev, const int *rad, int np);  // nullptr: not built
hipError_t jit_launch_rader(const JitRader *j, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, const cd *bhat, const int *gpow,
                            const int *ginv, double scale, hipStream_t s);
// rader_pfa_kernel (mixed_fixed.hpp): n = m * P (gcd 1), P = prod(rad) + 1
// prime, by the prime-factor map and m Rader sub-transforms in one kernel;
// launched by jit_launch_rader with the prime P's tables. nullptr: m has no
// in-register DFT, the geometry does not fit, or the kernel did not build.
bool pfa_cofactor_supported(int m);
// bluestein_fixed_kernel (mixed_fixed.hpp): the fused chirp-z on a smooth
// convolution length L = prod(rad) >= 2n - 1. blufix_length: L (and its list)
// where the lane-cost model puts it below 0.85 of the current fused kernel
// on m_now with list rad_now, else 0.
int blufix_length(int64_t n, int64_t m_now, const int *rad_now, int np_now, int *rad, int *np);
struct JitBlu;
JitBlu *jit_blu_build(int dev, int64_t n, const int *rad, int np);  // nullptr: not built
hipError_t jit_launch_blu(const JitBlu *j, bool inv, int load, const void *in, cd *out,
                          int64_t batch, const cd *tw, const cd *chirp, const cd *bhat,
                          double scale, hipStream_t s);
JitRader *jit_rader_pfa_build(int dev, int m, const int *rad, int np);
hipError_t jit_launch_pwelch(const JitSpec *j, const double *x, int64_t nfft, int64_t stride,
                             int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                             const double *win, const cd *tw, double *partial, hipStream_t s);
// radix list of a compiled specialisation for n (false: use the generic list)
bool mixed_fixed_radices(int n, int *rad, int *npass);
// the fused Pwelch's own list for n where it differs from the FFT's (fft_mixed.hip)
bool pwelch_fixed_radices(int n, int *rad, int *npass);
hipError_t launch_fft_mixed(const MixedDesc &d, bool inv, int load, const void *in, cd *out,
                            int64_t batch, const cd *tw, double scale, hipStream_t s);
hipError_t launch_bluestein(int log2m, bool inv, const cd *in, cd *out, int64_t n,
                            int64_t batch, const cd *twm, const cd *chirp, const cd *bhat,
                            double scale, hipStream_t s);
// fused chirp-z on M = 16 * RB * 16 (chirpz6k.hip): the smallest such M >=
// 2n - 1 of the kept pass-B radices RB, n >= 129, where it is not above the
// power of 2 (chirpz6k_m; 0 otherwise). tw = W_{16 RB}^k (k < 16) then W_M^k (k < M/16), bhat = FFT_M(b)/M; load LOAD_REAL: float64
// rows (forward only)
int chirpz6k_m(int64_t n);
// the pass radices of the fused chirp-z on m: {16, RB, 16} or {16, R1, R2, 16}
// (chirpz4_kernel); returns their count (0: not a chirpz6k length)
int chirpz6k_radices(int64_t m, int *rad);
hipError_t launch_chirpz6k(int64_t m, bool inv, int load, const void *in, cd *out, int64_t n,
                           int64_t batch, const cd *tw, const cd *chirp, const cd *bhat,
                           double scale, hipStream_t s);
// output-split chirp-z on M = 2^log2m (13 or 14): parts * kpart >= n outputs,
// n + kpart - 1 <= M, bhat = parts tables of M, twm = T_M
hipError_t launch_bluestein_parts(int log2m, bool inv, const cd *in, cd *out, int64_t n,
                                  int64_t batch, int parts, int64_t kpart, const cd *twm,
                                  const cd *chirp, const cd *bhat, double scale, hipStream_t s);
hipError_t launch_global_pass(int radix, bool conj_in, int load, bool conj_scale_out,
                              const void *in, cd *out, const cd *tw, int log2n, int log2ns,
                              int64_t batch, double scale, hipStream_t s);
int pwelch_workers_per_block(int log2f);
hipError_t launch_pwelch(int log2f, const double *x, int64_t nfft, int64_t stride,
                         int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,
                         const double *win, const cd *tw, double *partial, hipStream_t s);
// Noverlap = NFFT/2, Pad = NFFT, 5 <= log2f <= 14 (E even and T | F/2)
hipError_t launch_pwelch_half(int log2f, const double *x, int64_t seg_begin, int64_t seg_end,
                              int64_t ppw, int64_t nworkers, const double *win, const cd *tw,
                              double *partial, hipStream_t s);
// the row kernel (pwelch_row.hip) behind launch_pwelch_half(12, ...)
// any other overlap at F = 4096, Pad = NFFT (pwelch_rowg_kernel)
hipError_t launch_pwelch_rowg4096(const double *x, int64_t stride, int64_t seg_begin,
                                  int64_t seg_end, int64_t ppw, int64_t nworkers,
                                  const double *win, const cd *tw, double *partial,
                                  hipStream_t s);
hipError_t launch_pwelch_row4096(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                 int64_t nworkers, const double *win, const cd *tw,
                                 double *partial, hipStream_t s);
hipError_t launch_reduce_partials(const double *partial, int64_t nworkers, int64_t F, double *acc,
                                  double *scratch, hipStream_t s);
int64_t reduce_scratch_doubles(int64_t nworkers, int64_t F);
// materialised Pwelch: packed segment pairs (nrows rows of flen), then
// per-bin partial power sums over parts of rpp rows (<= 65535 parts)
hipError_t launch_segments_to_complex(const double *x, int64_t nfft, int64_t flen, int64_t stride,
                                      int64_t seg0, int64_t seg_end, int64_t nrows,
                                      const double *win, cd *buf, hipStream_t s);
hipError_t launch_power_partials(const cd *buf, int64_t nrows, int64_t flen, int64_t rpp,
                                 double *partial, hipStream_t s);
// Column pass of the mixed four-step for a single-radix column length L
// (fft_mixed.hip): DFT_L down each of the C columns of batch L x C matrices
// (matrix stride n = L*C), times W_n^(col*k), in place allowed
bool colradix_supported(int L);
hipError_t launch_colradix(int L, bool conj_in, const cd *in, cd *out, int64_t C, int64_t n,
                           int64_t batch, const cd *tw, hipStream_t s);
// FFT2 column pass on row-segment tiles; 4 <= log2l <= 9 (see fft_kernels.hip)
constexpr int kColMinLog2 = 4, kColMaxLog2 = 9;
// twiddle: 0 none, 1 W_R^(group*j), 2 W_R^(col*j); table index mod 2^log2r, or mod
// twn when twn > 0 (a non-power-of-2 N)
// the composed chirp-z's first column pass (DFT_R, R = 2^log2l, 7 ... 10, of
// the R x C view, times W_M^(col j)) on a = x * chirp zero-padded to M = R C,
// the premultiply folded into its loads: x rows of n, out rows of M
hipError_t launch_colfft_chirp(int log2l, bool conj_in, const cd *x, cd *out, int64_t C,
                               int64_t n, const cd *chirp, const cd *twl, const cd *twr,
                               int64_t batch, hipStream_t s);
// row DFT_C (C = 2^log2c, 4 ... 10) of `rows` rows (batch * R, any R) with
// the four-step transpose fused into the store: out[b N + k2 R + k1] =
// DFT_C(in row b R + k1)[k2] (fft_kernels.hip). mode 0 as is, 1 conj and
// scale (inverse), 2 conj(X tab) (the composed chirp-z's b-hat step), 3
// conj(X) tab for k < n into rows of n (its output step; inv: conj and scale)
hipError_t launch_rowfft_t(int log2c, int mode, const cd *in, cd *out, int64_t rows, int64_t R,
                           const cd *tw, double scale, hipStream_t s, const cd *tab = nullptr,
                           int64_t n = 0, bool inv = false);
hipError_t launch_colfft(int log2l, bool conj_in, int twiddle, bool conj_scale_out, const cd *in,
                         cd *out, int64_t C, int64_t ngroups, int64_t in_step, int64_t in_stride,
                         int64_t out_step, int64_t out_stride, const cd *twl, const cd *twr,
                         int log2r, double scale, int64_t batch, int64_t mat_stride,
                         hipStream_t s, int64_t twn = 0);
// batch <= 65535 matrices of rows x cols, consecutive; optional conj+scale
// out, and twiddle tw[r*c] (source row r, column c; needs r*c < twn)
hipError_t launch_transpose(const cd *in, cd *out, int64_t rows, int64_t cols, hipStream_t s,
                            int64_t batch = 1, bool conj_scale = false, double scale = 1.0,
                            const cd *tw = nullptr, int64_t twn = 0, bool tw_conj = false);
// the final transpose of a composed chirp-z FFT_M with the next chirp-z step
// folded in (fft_kernels.hip transpose_blu_kernel): mode 1 conj(v * bhat),
// mode 2 the result rows of n
hipError_t launch_transpose_blu(const cd *in, cd *out, int64_t rows, int64_t cols, int64_t batch,
                                int mode, int64_t n, const cd *tab, bool inv, double scale,
                                hipStream_t s);
hipError_t launch_real_to_complex(const double *in, cd *out, int64_t count, hipStream_t s);
hipError_t launch_chirp_premul(const cd *in, cd *a, int64_t n, int64_t m, int64_t batch,
                               const cd *chirp, bool conj_in, hipStream_t s);
hipError_t launch_bhat_mul_conj(cd *a, int64_t m, int64_t batch, const cd *bhat, hipStream_t s);
hipError_t launch_chirp_postmul(const cd *a, cd *out, int64_t n, int64_t m, int64_t batch,
                                const cd *chirp, bool inv, double scale, hipStream_t s);
hipError_t launch_pointwise_mul(const cd *a, const cd *b, cd *out, int64_t count, hipStream_t s);
hipError_t launch_scale(cd *a, int64_t count, double sc, hipStream_t s);
// wav.ReadFloats conversion (wav.hip): audio_format 1 (bits 8 / 16) or 3
hipError_t launch_wav_decode(const void *in, int64_t count, int audio_format, int bits,
                             void *out, bool f64, hipStream_t s);
hipError_t launch_fill_uniform(double *out, int64_t count, uint64_t seed, uint64_t offset,
                               hipStream_t s);

#endif  // __HIPCC_RTC__

}  // namespace gdsp
