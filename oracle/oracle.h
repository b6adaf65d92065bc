/*
 * oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the go-dsp reference
 * algorithms (maddyblue/go-dsp @ /root/reference) used as the parity checker.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library. The product path (go-dsp_amd/, libgdspfft.so) never links or
 * calls it.
 *
 * Parity pinning: every function is checked against the reference's own golden
 * vectors (fft/fft_test.go:38-162,189-195, spectral/pwelch_test.go:31-46,
 * spectral/spectral_test.go:31-56, window/window_test.go:34-59) by
 * tests/test_oracle.py. The reference itself (Go) cannot be built here: no Go
 * toolchain in the image.
 *
 * Complex data are interleaved (re, im) float64 pairs — the memory layout of Go
 * complex128.
 */
#ifndef GDSP_ORACLE_H
#define GDSP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OR_OK = 0,
  OR_ERR_INVALID = 1,  /* bad argument (negative length, ...) */
  OR_ERR_UNEQUAL = 2,  /* "arrays not of equal size"  fft/fft.go:57 */
  OR_ERR_EMPTY = 3,    /* "empty input array"         fft/fft.go:126 / IFFT len 0 fft/fft.go:40 */
  OR_ERR_NOMEM = 4,
};

enum {
  OR_WIN_HANN = 0,        /* window/window.go:62-76 */
  OR_WIN_HAMMING = 1,     /* window/window.go:44-58 */
  OR_WIN_RECTANGULAR = 2, /* window/window.go:32-40 */
  OR_WIN_BARTLETT = 3,    /* window/window.go:80-98 */
  OR_WIN_FLATTOP = 4,     /* window/window.go:102-135 */
  OR_WIN_BLACKMAN = 5,    /* window/window.go:138-152 */
};

/* dsputils helpers, dsputils/dsputils.go:34-45 */
int or_is_pow2(int64_t x);
int64_t or_next_pow2(int64_t x);

/* radix2.go:184-199 / :172-180 */
uint64_t or_reverse_bits(uint64_t v, uint64_t s);
uint64_t or_log2(uint64_t v);

/* radix2.go:39-69: fills out[0..n) with the cached table T_n (n power of 2, n >= 4). */
int or_radix2_factors(int64_t n, double *out);

/* fft.go:72-87 (dispatch), radix2.go:80-154, bluestein.go:68-94 */
int or_fft(const double *x, double *out, int64_t n);
/* fft.go:35-52 */
int or_ifft(const double *x, double *out, int64_t n);
/* fft.go:25-27, :30-32 */
int or_fft_real(const double *x, double *out, int64_t n);
int or_ifft_real(const double *x, double *out, int64_t n);
/* fft.go:55-69 */
int or_convolve(const double *x, const double *y, double *out, int64_t n);
/* fft.go:104-154: x is rows*cols complex, row-major (x[j][i] at j*cols+i). */
int or_fft2(const double *x, double *out, int64_t rows, int64_t cols, int inverse);

/* fft.go:157-192 (FFTN / IFFTN over a row-major Matrix of dims[0..ndims)). */
int or_fftn(const double *x, double *out, const int64_t *dims, int ndims, int inverse);

/* Reference-threaded radix-2 (radix2.go:89-151 structure: nworkers workers,
 * contiguous butterfly ranges of >= n/nworkers, one barrier per stage). Used
 * only as bench.py's cpu_baseline. Same arithmetic as or_fft. */
int or_fft_threaded(const double *x, double *out, int64_t n, int nworkers);
/* Loop over rows as a user of fft.FFT would (one call per row). */
int or_fft_rows_threaded(const double *x, double *out, int64_t n, int64_t rows,
                         int nworkers);

/* window/window.go */
int or_window(int kind, int64_t L, double *out);

/* spectral/spectral.go:22-47 — number of segments (negative on error). */
int64_t or_segment_count(int64_t lx, int64_t size, int64_t noverlap);

/* spectral/pwelch.go:74-145. nfft/pad 0 => defaults (256, nfft). Outputs
 * pxx/freqs have lp = pad/2+1 entries (*lp_out). Empty x => *lp_out = 0. */
int or_pwelch(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
              int64_t noverlap, int window_kind, int scale_off, double *pxx,
              double *freqs, int64_t *lp_out);

/* or_pwelch with the reference's worker pool inside every FFTReal (the CPU
 * baseline of bench.py). */
int or_pwelch_threaded(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                       int64_t noverlap, int window_kind, int scale_off, double *pxx,
                       double *freqs, int64_t *lp_out, int nworkers);

/* Counter-based synthetic input generator shared with the device generator
 * (splitmix64; see DESIGN.md §Synthetic data): uniform [-1, 1). */
void or_fill_uniform(double *out, int64_t count, uint64_t seed, uint64_t offset);

/* wav.(*Wav).ReadFloats's conversion, wav/wav.go:135-161, of `count`
 * little-endian samples in `in` (ReadSamples, wav.go:110-131): PCM 8-bit
 * v/MaxUint8, PCM 16-bit (v - MinInt16)/(MaxInt16 - MinInt16), both in
 * float32 arithmetic; IEEE float32 copied. Returns -1 for a format the
 * reference rejects ("unknown bits per sample" / "unknown audio format"). */
int or_wav_floats(const void *in, int64_t count, int audio_format, int bits_per_sample,
                  float *out);

#ifdef __cplusplus
}
#endif
#endif
