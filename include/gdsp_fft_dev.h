/* gdsp_fft_dev.h — entry points of the DEVELOPMENT build of libgdspfft only
 * (make -C go-dsp_amd/csrc DEV=1 -> go-dsp_amd/lib_dev/libgdspfft.so).
 *
 * They run the measured-and-rejected kernels that only the development build
 * contains (go-dsp_amd/csrc/dev/, DESIGN.md §3 "Wavefront shuffles"; §7a),
 * so their tests can compare them with the oracle. The product library
 * (go-dsp_amd/lib) does not export them, no product code path reaches these
 * kernels, and a drop-in caller of include/gdsp_fft.h never needs them.
 * Device pointers, stream-ordered on `stream` (NULL: the null stream).
 */
#ifndef GDSP_FFT_DEV_H
#define GDSP_FFT_DEV_H

#include "gdsp_fft.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Waves per transform of the wave-resident chirp-z kernel (fft_wave.hip: one
 * 64-lane wavefront per 2048-point sub-transform, M = NextPowerOf2(2n-1) =
 * 2048 * waves) for 512 < n <= 4096, else 0. */
int gdsp_dev_chirpz_wave_q(int64_t n);
/* fft.FFT / IFFT of batch rows of n complex128 by Bluestein's algorithm
 * (fft/bluestein.go:68-94, the reference's M) on the wave-resident kernel
 * (n with gdsp_dev_chirpz_wave_q(n) > 0), or on the M = 8192 kernel whose FFTs
 * keep one exchange inside the wave (bluestein_shfl.hip, 2049 <= n <= 4096).
 * Synchronous on the first call for n (its tables). */
int gdsp_dev_fft_batch_chirpz_wave(int64_t n, const void *d_in, void *d_out, int64_t batch,
                                   int inverse, void *stream);
int gdsp_dev_fft_batch_chirpz_shfl(int64_t n, const void *d_in, void *d_out, int64_t batch,
                                   int inverse, void *stream);
/* gdsp_pwelch_accumulate_device for NFFT = Pad = 4096, Noverlap = 2048 on the
 * kernel with the in-wave second exchange (pwelch_shfl.hip): adds the packed
 * pairs' |Z_k|^2 of segments [seg_begin, seg_end) of d_x (n samples) to
 * d_acc (4096 doubles); d_win: the 4096-point window. Synchronous. */
int gdsp_dev_pwelch4096_shfl_accumulate(const double *d_x, int64_t n, int64_t seg_begin,
                                        int64_t seg_end, const double *d_win, double *d_acc,
                                        void *stream);
/* The same on the row kernel reshaped for three workgroups per CU
 * (pwelch_row3.hip: the next pair by LDS-DMA, a half-size exchange buffer,
 * 168 VGPRs of which 42 spill). */
int gdsp_dev_pwelch4096_row3_accumulate(const double *d_x, int64_t n, int64_t seg_begin,
                                        int64_t seg_end, const double *d_win, double *d_acc,
                                        void *stream);

#ifdef __cplusplus
}
#endif

#endif /* GDSP_FFT_DEV_H */
