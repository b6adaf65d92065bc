/*
 * gdsp_fft.h — C ABI of libgdspfft, the MI355X (gfx950) batched-FFT engine for
 * the go-dsp hot path (maddyblue/go-dsp: fft/, spectral/Pwelch, window/Hann).
 *
 * This is the drop-in boundary: each entry point names the reference Go
 * function it replaces (file:line under maddyblue/go-dsp). A Go maintainer
 * binds these through cgo; tests bind them via ctypes.
 *
 * Conventions (mirroring the reference):
 *  - complex data are interleaved (re, im) IEEE float64 pairs, i.e. the memory
 *    layout of Go []complex128 and of C99 double _Complex;
 *  - inputs are never modified; outputs are caller-owned buffers that the
 *    library fills (Go allocates the result slice, C fills it);
 *  - the library never retains a caller pointer after returning (cgo rule);
 *  - every compute runs on the GPU. There is no CPU fallback: without a usable
 *    HIP device the calls return GDSP_ERR_NO_DEVICE;
 *  - the reference's panics become status codes; the Go shim re-panics with
 *    the reference's message (gdsp_status_string);
 *  - host-pointer entry points are synchronous and thread-safe; device-pointer
 *    entry points ("_device") are stream-ordered on the given hipStream_t
 *    (passed as void*; NULL = the null/default stream, as in HIP) and run on
 *    the calling thread's current HIP device.
 */
#ifndef GDSP_FFT_H
#define GDSP_FFT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------- */
typedef enum {
  GDSP_OK = 0,
  GDSP_ERR_INVALID = 1,        /* bad argument (negative size, NULL pointer, ...) */
  GDSP_ERR_UNEQUAL = 2,        /* "arrays not of equal size"   fft/fft.go:57 */
  GDSP_ERR_EMPTY = 3,          /* "empty input array"          fft/fft.go:126;
                                  IFFT of len 0 (index out of range, fft/fft.go:40) */
  GDSP_ERR_RAGGED = 4,         /* "ragged input array"         fft/fft.go:133 */
  GDSP_ERR_DIVIDE_BY_ZERO = 5, /* Segment stride 0 (integer divide, spectral.go:31) */
  GDSP_ERR_NO_DEVICE = 6,      /* no HIP device / runtime error at init */
  GDSP_ERR_HIP = 7,            /* HIP runtime error during a call */
  GDSP_ERR_NOMEM = 8,          /* device or host allocation failed */
  GDSP_ERR_UNSUPPORTED = 9     /* size beyond what this build implements */
} gdsp_status;

/* Reference panic message (or a description) for a status code. */
const char *gdsp_status_string(int status);
/* Detail of the last error raised on the calling thread ("" if none). */
const char *gdsp_last_error(void);
/* Library version string. */
const char *gdsp_version(void);
/* Runtime compiler (hipRTC specialisations of smooth lengths) since process
 * start: modules compiled, modules loaded from the on-disk code-object cache
 * (GDSP_JIT_CACHE), and compilations that failed — each failure leaves its
 * plan on the slower path it would have replaced, with the same results. The
 * last failure's description is copied into last_failure (cap bytes, NUL-
 * terminated; may be NULL). */
int gdsp_jit_stats(int64_t *built, int64_t *cached, int64_t *failed, char *last_failure,
                   int64_t cap);
/* Number of visible HIP devices (0 without a GPU; never initialises a context
 * beyond hipGetDeviceCount). */
int gdsp_device_count(void);

/* Algorithm selection (no reference equivalent; additive). Every selection
 * computes the same DFT (the reference's results within the 1e-9 bound)
 * by another of the engine's paths; the default (0) takes the measured
 * fastest. Flags apply to plans built after the call (plans are cached per
 * length and flag set) and to Pwelch calls made after it; process-wide. */
enum {
  GDSP_ALGO_DEFAULT = 0,
  /* smooth non-power-of-2 lengths (transforms and fused Pwelch) on the
   * runtime-radix mixed kernels, without the compiled or runtime-compiled
   * (hipRTC) specialisations */
  GDSP_ALGO_GENERIC_MIXED = 1,
  /* primes in (8192, 14563] on the composed chirp-z instead of the
   * output-split fused kernel */
  GDSP_ALGO_NO_CHIRPZ_PARTS = 2,
  /* chirp-z on the reference's M = NextPowerOf2(2n-1) (fft/bluestein.go:70)
   * instead of a smaller smooth M: the composed chirp-z, and the fused one
   * for 129 <= n <= 3200 and 4097 <= n <= 6144 (by default M = 16 * RB * 16
   * or 16 * R1 * R2 * 16, the smallest kept one >= 2n - 1 where not above
   * the power of 2) */
  GDSP_ALGO_CHIRPZ_POW2 = 4,
  /* the composed chirp-z without its fused transposes */
  GDSP_ALGO_CHIRPZ_UNFUSED = 8,
  /* primes n <= 8193 whose n - 1 has a radix list, and the composites of
   * plan kind 8, on the chirp-z kernels instead of Rader's algorithm (plan
   * kinds 7 and 8) */
  GDSP_ALGO_NO_RADER = 16,
  /* no plan-time measurement: where the default races two kernels on
   * synthetic rows when a plan is built (plan kind 8 against the chirp-z
   * plan it would replace; the fused chirp-z on a smooth convolution length
   * against the one on a power of 2) and keeps the faster, take the
   * cost model's candidate instead */
  GDSP_ALGO_NO_RACE = 32
};
/* Unknown bits → GDSP_ERR_INVALID (the selection is left unchanged). */
int gdsp_set_algorithm(unsigned flags);
unsigned gdsp_get_algorithm(void);

/* ---- fft package: host pointers, synchronous ----------------------------- */

/* fft.FFT — fft/fft.go:72-87. n <= 1 copies; power of 2 → Stockham radix-16
 * kernels (reference: radix2FFT, fft/radix2.go:80-154); other n whose prime
 * factors are all <= 13 → a mixed-radix Stockham kernel (n <= 4096) or, above
 * 8192, a four-step over two such factors, computing the same DFT directly;
 * otherwise Bluestein (fft/bluestein.go:68-94).
 * x, out: n complex128. */
int gdsp_fft(const double *x, double *out, int64_t n);

/* fft.IFFT — fft/fft.go:35-52. n == 0 → GDSP_ERR_EMPTY (reference panics). */
int gdsp_ifft(const double *x, double *out, int64_t n);

/* fft.FFTReal — fft/fft.go:25-27. x: n float64; out: n complex128 (full
 * spectrum, as the reference returns). */
int gdsp_fft_real(const double *x, double *out, int64_t n);

/* fft.IFFTReal — fft/fft.go:30-32. */
int gdsp_ifft_real(const double *x, double *out, int64_t n);

/* fft.Convolve — fft/fft.go:55-69 (IFFT(FFT(x)·FFT(y))). The reference's
 * length check ("arrays not of equal size") is the caller's: both are n. */
int gdsp_convolve(const double *x, const double *y, double *out, int64_t n);

/* Additive batched entry point (no reference equivalent): the
 * same transform as fft.FFT / fft.IFFT applied to `batch` contiguous rows of n
 * complex128. inverse != 0 → IFFT semantics. */
int gdsp_fft_batch(const double *x, double *out, int64_t n, int64_t batch, int inverse);

/* Real-input batch (FFTReal per row): x is batch*n float64. */
int gdsp_fft_real_batch(const double *x, double *out, int64_t n, int64_t batch);

/* fft.FFT2 / fft.IFFT2 — fft/fft.go:109-121 → computeFFT2 :123-154. x is a
 * row-major rows×cols complex128 matrix (the Go shim flattens [][]complex128
 * after checking raggedness). rows == 0 → GDSP_ERR_EMPTY. */
int gdsp_fft2(const double *x, double *out, int64_t rows, int64_t cols, int inverse);

/* fft.FFT2Real / fft.IFFT2Real — fft/fft.go:104-107, :114-117. x: rows×cols
 * float64. */
int gdsp_fft2_real(const double *x, double *out, int64_t rows, int64_t cols, int inverse);

/* fft.FFTN / fft.IFFTN — fft/fft.go:157-192 (computeFFTN): the N-D DFT of a
 * row-major dsputils.Matrix (dsputils/matrix.go:21-57) with dims[0..ndims),
 * each >= 1 ("invalid dimensions" otherwise, GDSP_ERR_INVALID). x, out:
 * prod(dims) complex128. */
int gdsp_fftn(const double *x, double *out, const int64_t *dims, int ndims, int inverse);

/* fft.EnsureRadix2Factors — fft/radix2.go:35-37: pre-build (and cache) the
 * device plan for length n on the current device. Works for any n >= 2. */
int gdsp_ensure_plan(int64_t n);

/* fft.SetWorkerPoolSize — fft/fft.go:95-101. The GPU path has no worker
 * pool; the value is recorded (n < 0 → 0) and reported by
 * gdsp_worker_pool_size for API parity. */
void gdsp_set_worker_pool_size(int n);
int gdsp_worker_pool_size(void);

/* ---- spectral package ------------------------------------------------------ */

/* spectral.Segment — spectral/spectral.go:22-33: number of segments of length
 * `size` with `noverlap` overlap in a signal of length lx. Writes *count. */
int gdsp_segment_count(int64_t lx, int64_t size, int64_t noverlap, int64_t *count);

/* spectral.Pwelch — spectral/pwelch.go:74-145.
 * x: n float64 samples. nfft/pad/noverlap as PwelchOptions (0 = defaults:
 * nfft 256, pad nfft). Go's PwelchOptions.Window is a Go func, so the shim
 * passes its tables: win_seg = wf(max(pad, nfft)) — the window the reference
 * applies to each zero-padded segment (pwelch.go:108-109, window.go:25-29) —
 * and win_nfft = wf(nfft) for the normalisation (pwelch.go:124). NULL for
 * either selects window.Hann (the default, pwelch.go:89-91).
 * pxx, freqs: caller buffers of pad/2+1 float64; *lp_out receives the count
 * (0 for empty x, as the reference returns empty slices). */
int gdsp_pwelch(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                int64_t noverlap, const double *win_seg, const double *win_nfft,
                int scale_off, double *pxx, double *freqs, int64_t *lp_out);

/* window.Hann — window/window.go:62-76, as a host table generator used by the
 * shim for the default window (L float64 written to out). */
int gdsp_window_hann(int64_t L, double *out);

/* ---- wav package (the wav -> Pwelch feeder) -------------------------------- */

/* wav.(*Wav).ReadFloats — wav/wav.go:135-161 — on the GPU: converts `count`
 * little-endian samples of a WAV data chunk (what ReadSamples reads,
 * wav.go:110-131) with the reference's float32 formulas. audio_format 1 with
 * bits_per_sample 8 or 16 (PCM) or 3 (IEEE float32); anything else →
 * GDSP_ERR_UNSUPPORTED ("wav: unknown bits per sample" / "unknown audio
 * format" in the reference). out_f64 = 0 writes float32 (the reference's
 * []float32), 1 writes float64 (the float32 values widened: a Pwelch input).
 * Host-pointer form: in/out on the host, synchronous. */
int gdsp_wav_read_floats(const void *in, int64_t count, int audio_format, int bits_per_sample,
                         void *out, int out_f64);

/* ---- multi-device (one node's GPUs inside one call) ------------------------- */
/* The reference keeps its parallelism inside the call (radix2FFT's goroutine
 * pool, fft/radix2.go:89-151; Pwelch's one accumulation loop,
 * spectral/pwelch.go:107-122). These keep that across GPUs: a batched FFT
 * splits its rows into contiguous shards, one per device, with no
 * collective; Pwelch splits its segments (each device reads its samples plus
 * the nfft - stride halo) and combines the per-device accumulators with one
 * in-process RCCL reduce (sum, float64) before the host finalises Pxx. Each
 * multi-device call runs whole (accumulate, reduce, copy back) before the
 * next one from any host thread starts. */

/* Library-wide device set. When it has been configured (here, or by
 * GDSP_DEVICES="0,1,2,3" / "all" at first use) with more than one entry,
 * gdsp_fft_batch, gdsp_fft_real_batch and gdsp_pwelch split calls whose input
 * is at least GDSP_MULTI_MIN_BYTES (64 MiB by default) and has at least 2
 * rows / segments over it. Unconfigured (the default, or ndev = 0 here) the
 * set is the calling thread's current device, so no call leaves it. A device
 * may be listed more than once: its shards run side by side on separate
 * streams (a Pwelch over such a set, or without a loadable librccl, sums the
 * per-device accumulators on the host instead of by RCCL). Devices must be
 * visible. */
int gdsp_set_devices(const int *devices, int ndev);
/* The current device set: writes up to cap ids, returns the set's size (0
 * without a GPU). */
int gdsp_get_devices(int *devices, int cap);
/* Multi-device calls since process start (diagnostics and tests): batched
 * FFT calls and Pwelch calls split over a device set, and how the Pwelch
 * accumulators were combined (RCCL reduce / host sum). Any pointer may be
 * NULL. */
int gdsp_multi_stats(int64_t *batch_calls, int64_t *pwelch_calls, int64_t *rccl_reduces,
                     int64_t *host_reduces);

/* fft.FFT / fft.IFFT over `batch` rows of n complex128 (as gdsp_fft_batch),
 * always split over `devices` (NULL or ndev = 0: the library's device set);
 * at most `batch` devices take part. Host pointers, synchronous. */
int gdsp_fft_batch_multi(const double *x, double *out, int64_t n, int64_t batch, int inverse,
                         const int *devices, int ndev);

/* spectral.Pwelch (as gdsp_pwelch), always split over `devices` (NULL or
 * ndev = 0: the library's device set) with the RCCL reduce of the per-bin
 * accumulators — also for a single device (host sum for a set that repeats
 * a device). Thread-safe: the accumulators are owned by the call. */
int gdsp_pwelch_multi(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                      int64_t noverlap, const double *win_seg, const double *win_nfft,
                      int scale_off, double *pxx, double *freqs, int64_t *lp_out,
                      const int *devices, int ndev);

/* Shard i of ndev, as the calls above split the work: rows [*lo, *hi) of a
 * batch; and for Pwelch, segments [*seg_lo, *seg_hi) of nsegs and the
 * samples [*x_lo, *x_hi) they read (empty when the shard has no segment).
 * Host arithmetic only (no GPU needed). */
int gdsp_batch_shard(int64_t batch, int ndev, int i, int64_t *lo, int64_t *hi);
int gdsp_pwelch_shard(int64_t nsegs, int64_t nfft, int64_t noverlap, int ndev, int i,
                      int64_t *seg_lo, int64_t *seg_hi, int64_t *x_lo, int64_t *x_hi);

/* ---- device-pointer API (stream-ordered; multi-GPU building blocks) ---------- */

typedef struct gdsp_plan gdsp_plan;

/* Create / fetch the cached plan for transform length n on the current
 * device. Plans are owned by the library cache; destroy is a no-op for cached
 * plans and exists for API symmetry. */
int gdsp_plan_create(int64_t n, gdsp_plan **plan);
int gdsp_plan_destroy(gdsp_plan *plan);
/* The same transform as fft.FFT for non-power-of-2 n, always computed with
 * Bluestein's chirp-z (fft/bluestein.go:68-94) — the reference's algorithm —
 * even where the default plan uses the mixed-radix kernel. n >= 2. Cached
 * separately from gdsp_plan_create's plans. */
int gdsp_plan_create_chirpz(int64_t n, gdsp_plan **plan);
/* Which algorithm a plan runs: 0 trivial (n<=1), 1 one-kernel LDS Stockham,
 * 2 multi-pass global Stockham (large power of 2), 3 fused Bluestein,
 * 4 composed Bluestein (M > 16384), 5 one-kernel mixed radix (non-power-of-2
 * n <= 4096 whose prime factors are all <= 13), 6 mixed four-step (such n
 * above 8192 = n1*n2 with one-kernel factors: transposes + row kernels),
 * 7 Rader (a prime 17 <= n <= 8193 whose n - 1 has a list of radices <= 25
 * within 640 threads per transform: the DFT as
 * a cyclic convolution of length n - 1, two FFTs of n - 1 points in one
 * runtime-compiled kernel; GDSP_ALGO_NO_RADER keeps such primes on kind 3),
 * 8 prime-factor Rader (a composite n <= 8192 = n1 * n2, n2 > 31 its largest
 * prime factor with a kind-7 plan, gcd(n1, n2) = 1, n1 with an in-register
 * DFT: the Good-Thomas map, DFT_n1 per column and n1 Rader transforms of n2
 * points, one runtime-compiled kernel; GDSP_ALGO_NO_RADER keeps kind 3). */
int gdsp_plan_kind(const gdsp_plan *plan);
/* Geometry of a plan (any pointer may be NULL): its length n; the chirp-z
 * convolution length m (kinds 3 and 4; the reference's NextPowerOf2(2n-1),
 * bluestein.go:70, or a smooth m >= 2n-1 that the composed chirp-z may
 * choose; kind 7: Rader's cyclic convolution length n - 1; kind 8: n2 - 1);
 * the four-step split n = n1*n2 (kinds 2 and 6) or the prime-factor split
 * (kind 8: cofactor n1, prime n2); and whether a
 * runtime-compiled specialisation backs it (1) or not (0). 0 where n/a. */
int gdsp_plan_info(const gdsp_plan *plan, int64_t *n, int64_t *m, int64_t *n1, int64_t *n2,
                   int *runtime_compiled);
/* The radix list of a plan's mixed-radix passes: kind 5 its transform's,
 * kind 7 the cyclic convolution's (n - 1), kind 8 the prime factor's
 * convolution (n2 - 1). Writes min(count, cap) radices and returns the
 * count; 0 for the other kinds. */
int gdsp_plan_radices(const gdsp_plan *plan, int *rad, int cap);
/* Output parts of a kind-3 plan: 1 for the one-convolution chirp-z of
 * bluestein.go:68-94; P > 1 when n in (8192, 14563] (NextPowerOf2(2n-1) =
 * 32768, beyond one kernel) runs as P fused convolutions of M = 16384, each
 * giving ceil(n/P) of the outputs (GDSP_ALGO_NO_CHIRPZ_PARTS: the composed
 * chirp-z instead). */
int gdsp_plan_parts(const gdsp_plan *plan);

/* Batched C2C on device buffers: d_in/d_out hold batch*n complex128 (may
 * alias only if equal). inverse != 0 → IFFT semantics (1/n scaling). */
int gdsp_fft_batch_device(const gdsp_plan *plan, const void *d_in, void *d_out,
                          int64_t batch, int inverse, void *stream);

/* fft.FFTReal / fft.IFFTReal — fft/fft.go:25-32 — over `batch` device rows:
 * d_in holds batch*n float64 (read as they are: no ToComplex copy), d_out
 * batch*n complex128 and must not overlap d_in. inverse != 0 → IFFTReal
 * semantics (an empty plan is then GDSP_ERR_EMPTY, like IFFT). */
int gdsp_fft_real_batch_device(const gdsp_plan *plan, const double *d_in, void *d_out,
                               int64_t batch, int inverse, void *stream);

/* FFT2/IFFT2 on a device rows×cols complex128 matrix. d_work: scratch of
 * rows*cols complex128 (may be NULL: the library allocates stream-ordered). */
int gdsp_fft2_device(const void *d_in, void *d_out, int64_t rows, int64_t cols,
                     int inverse, void *d_work, void *stream);

/* FFTN/IFFTN on a device array (dims on the host). */
int gdsp_fftn_device(const void *d_in, void *d_out, const int64_t *dims, int ndims, int inverse,
                     void *stream);

/* One axis of FFTN: the 1-D FFT/IFFT along dimension `axis` of a device
 * row-major array (the per-dimension loop of computeFFTN, fft/fft.go:172-185;
 * axis 0 of a rows x cols matrix is computeFFT2's column pass, :138-147).
 * The building block of the multi-GPU FFT2 (row FFTs, all-to-all, column
 * FFTs on a column block). */
int gdsp_fft_axis_device(const void *d_in, void *d_out, const int64_t *dims, int ndims,
                         int axis, int inverse, void *stream);

/* Pwelch partial accumulation over segments [seg_begin, seg_end) of a device
 * signal d_x (n float64, sample 0 = sample 0 of segment 0). Adds into
 * d_acc[0..flen) (flen = max(pad, nfft)) the per-bin sums S_k of |Z_k|² over
 * the packed segment pairs; gdsp_pwelch_finalize turns the summed
 * accumulators (over every shard / rank) into Pxx. d_win_seg: flen float64
 * window table on the device. d_acc must be zeroed by the caller before the
 * first call. */
int gdsp_pwelch_accumulate_device(const double *d_x, int64_t n, int64_t nfft, int64_t pad,
                                  int64_t noverlap, int64_t seg_begin, int64_t seg_end,
                                  const double *d_win_seg, double *d_acc, void *stream);

/* Host finalisation (spectral/pwelch.go:113-142): from the summed
 * accumulators acc[0..flen) over all nsegs segments produce
 * pxx[j] = c_j * (acc[j] + acc[(flen-j)%flen]) / 2 / nsegs / norm and
 * freqs[j] = j*fs/pad for j < pad/2+1. */
int gdsp_pwelch_finalize(const double *acc, int64_t flen, int64_t nsegs, int64_t nfft,
                         int64_t pad, const double *win_nfft, double fs, int scale_off,
                         double *pxx, double *freqs);

/* gdsp_wav_read_floats on device buffers (d_in: the raw data-chunk bytes at
 * any alignment; d_out: count float32 or float64), stream-ordered: decode a
 * WAV stream straight into the HBM-resident Pwelch input. */
int gdsp_wav_read_floats_device(const void *d_in, int64_t count, int audio_format,
                                int bits_per_sample, void *d_out, int out_f64, void *stream);

/* Device synthetic input: d_out[i] = uniform[-1,1) from splitmix64(seed,
 * offset + i), i < count (float64). Identical to the host generator the tests
 * use; lets the bench generate inputs in HBM without a PCIe copy. */
int gdsp_fill_uniform_device(double *d_out, int64_t count, uint64_t seed, uint64_t offset,
                             void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GDSP_FFT_H */
