/* gdsp_fft_dev.h — queries of the DEVELOPMENT build of libgdspfft only
 * (make -C go-dsp_amd/csrc DEV=1 -> go-dsp_amd/lib_dev/libgdspfft.so).
 *
 * They describe the measured-and-rejected kernels that only the development
 * build contains (DESIGN.md §3 "Wavefront shuffles"; §7a). The product
 * library (go-dsp_amd/lib) does not export them, and a drop-in caller of
 * include/gdsp_fft.h never needs them: the tests that exercise those kernels
 * load the development build and include this header's declarations.
 */
#ifndef GDSP_FFT_DEV_H
#define GDSP_FFT_DEV_H

#include "gdsp_fft.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Waves per transform of the wave-resident chirp-z kernel (fft_wave.hip:
 * one 64-lane wavefront per 2048-point sub-transform, M = 2048 * waves) that a
 * kind-3 plan with 512 < n <= 4096 runs (GDSP_BLU_WAVE=1), or 0 for any other
 * kernel. */
int gdsp_plan_wave_q(const gdsp_plan *plan);
/* 1 when a kind-3 plan (M = 8192, 2049 <= n <= 4096) runs the chirp-z kernel
 * whose FFTs keep one of their two exchanges inside the wavefront
 * (bluestein_shfl.hip, GDSP_BLU_SHFL=1), else 0. */
int gdsp_plan_shfl(const gdsp_plan *plan);

#ifdef __cplusplus
}
#endif

#endif /* GDSP_FFT_DEV_H */
