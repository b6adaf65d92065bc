// dev.hpp — launchers of the measured-and-rejected kernels of the development
// build (make DEV=1 -> go-dsp_amd/lib_dev; DESIGN.md §3 "Wavefront shuffles").
// The product library has none of these, and no product source refers to
// them: dev_api.hip drives them through include/gdsp_fft_dev.h.
#pragma once
#include "../fft_device.hpp"
#include "../launch.hpp"

namespace gdsp {

// wave-resident chirp-z (fft_wave.hip): waves per transform Q = M / 2048 for
// 512 < n <= 1024 Q, 2n - 1 <= M (0: not this kernel's case)
int bluestein_wave_q(int64_t n, int64_t m);
// wbase[q 65 + j] = W_M^(q j) (j <= 64), bhatw[q 2048 + k] = bhat[Q k + q]
hipError_t launch_bluestein_wave(int q, bool inv, const cd *in, cd *out, int64_t n, int64_t batch,
                                 const cd *t2048, const cd *wbase, const cd *bhatw, const cd *chirp,
                                 double scale, hipStream_t s);
// M = 8192 chirp-z with in-wave exchanges (bluestein_shfl.hip), 2049 <= n <=
// 4096: bhatp[r 256 + t] = bhat[bluestein_shfl_bin(t, r)], twm = T_8192
int bluestein_shfl_bin(int t, int r);
hipError_t launch_bluestein_shfl(bool inv, const cd *in, cd *out, int64_t n, int64_t batch,
                                 const cd *twm, const cd *chirp, const cd *bhatp, double scale,
                                 hipStream_t s);
// NFFT = 4096 half overlap with the in-wave second exchange (pwelch_shfl.hip);
// same arguments and partial layout as launch_pwelch_half(12, ...)
hipError_t launch_pwelch4096_shfl(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                  int64_t nworkers, const double *win, const cd *tw,
                                  double *partial, hipStream_t s);

// the row kernel reshaped for three workgroups per CU (pwelch_row3.hip):
// LDS-DMA stage, half-size exchange; same arguments as launch_pwelch_half(12)
hipError_t launch_pwelch4096_row3(const double *x, int64_t seg_begin, int64_t seg_end, int64_t ppw,
                                  int64_t nworkers, const double *win, const cd *tw,
                                  double *partial, hipStream_t s);

}  // namespace gdsp
