/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h). A plain-C restatement of
 * the go-dsp reference algorithms, written from their documented behaviour
 *  and checked against the reference's golden vectors.
 *
 * Compiled with -ffp-contract=off so that no multiply-add is fused: the Go
 * amd64 compiler does not fuse float64 operations, and the reference's
 * complex128 arithmetic is plain (ac-bd, ad+bc).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  double re, im;
} cplx;

static inline cplx cmul(cplx a, cplx b) {
  /* Go complex128 product: (ac - bd) + (ad + bc)i */
  cplx r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
  return r;
}
static inline cplx cadd(cplx a, cplx b) {
  cplx r = {a.re + b.re, a.im + b.im};
  return r;
}
static inline cplx csub(cplx a, cplx b) {
  cplx r = {a.re - b.re, a.im - b.im};
  return r;
}

/* ---- dsputils/dsputils.go:34-45 ------------------------------------------ */
int or_is_pow2(int64_t x) { return (x & (x - 1)) == 0; }

int64_t or_next_pow2(int64_t x) {
  if (or_is_pow2(x)) return x;
  /* int(math.Pow(2, math.Ceil(math.Log2(float64(x))))) */
  return (int64_t)pow(2.0, ceil(log2((double)x)));
}

/* ---- radix2.go:172-199 ---------------------------------------------------- */
uint64_t or_log2(uint64_t v) {
  uint64_t r = 0;
  for (v >>= 1; v != 0; v >>= 1) r++;
  return r;
}

uint64_t or_reverse_bits(uint64_t v, uint64_t s) {
  /* only the low s bits are reversed; the first bit is taken before the loop */
  uint64_t r = v & 1;
  s--;
  for (v >>= 1; v != 0; v >>= 1) {
    r <<= 1;
    r |= v & 1;
    s--;
  }
  return r << s;
}

/* ---- radix2.go:24-69: twiddle cache --------------------------------------
 * T_4 = {1, -i, -1, i} exactly; T_i built by doubling: even entries copied
 * from T_{i/2}, odd entries Sincos(-2*Pi/float64(i)*float64(n)). */
#define OR_MAX_LOG2 40
static cplx *g_fac[OR_MAX_LOG2 + 1];
static pthread_mutex_t g_fac_lock = PTHREAD_MUTEX_INITIALIZER;

static const cplx *radix2_factors(int64_t n) {
  if (n < 4) return NULL; /* radix2Factors[2] is nil in the reference */
  int lg = (int)or_log2((uint64_t)n);
  pthread_mutex_lock(&g_fac_lock);
  if (!g_fac[2]) {
    g_fac[2] = (cplx *)malloc(4 * sizeof(cplx));
    g_fac[2][0] = (cplx){1, 0};
    g_fac[2][1] = (cplx){0, -1};
    g_fac[2][2] = (cplx){-1, 0};
    g_fac[2][3] = (cplx){0, 1};
  }
  for (int k = 3; k <= lg; k++) {
    if (g_fac[k]) continue;
    int64_t i = (int64_t)1 << k;
    cplx *t = (cplx *)malloc((size_t)i * sizeof(cplx));
    const cplx *p = g_fac[k - 1];
    for (int64_t m = 0, j = 0; m < i; m += 2, j++) t[m] = p[j];
    for (int64_t m = 1; m < i; m += 2) {
      double ang = -2 * M_PI / (double)i * (double)m;
      double s, c;
      sincos(ang, &s, &c);
      t[m].re = c;
      t[m].im = s;
    }
    g_fac[k] = t;
  }
  const cplx *r = g_fac[lg];
  pthread_mutex_unlock(&g_fac_lock);
  return r;
}

int or_radix2_factors(int64_t n, double *out) {
  if (n < 4 || !or_is_pow2(n)) return OR_ERR_INVALID;
  const cplx *f = radix2_factors(n);
  memcpy(out, f, (size_t)n * sizeof(cplx));
  return OR_OK;
}

/* ---- radix2.go:157-168 ---------------------------------------------------- */
static void reorder(const cplx *x, cplx *r, int64_t n) {
  uint64_t s = or_log2((uint64_t)n);
  for (uint64_t i = 0; i < (uint64_t)n; i++) r[or_reverse_bits(i, s)] = x[i];
}

/* One butterfly range of one stage (radix2.go:101-123). */
static void stage_range(const cplx *r, cplx *t, const cplx *factors, int64_t stage,
                        int64_t blocks, int64_t start, int64_t end) {
  int64_t s_2 = stage / 2;
  for (int64_t nb = start; nb < end; nb += stage) {
    if (stage != 2) {
      for (int64_t j = 0; j < s_2; j++) {
        int64_t idx = j + nb;
        int64_t idx2 = idx + s_2;
        cplx ridx = r[idx];
        cplx w_n = cmul(r[idx2], factors[blocks * j]);
        t[idx] = cadd(ridx, w_n);
        t[idx2] = csub(ridx, w_n);
      }
    } else {
      int64_t n1 = nb + 1;
      cplx rn = r[nb], rn1 = r[n1];
      t[nb] = cadd(rn, rn1);
      t[n1] = csub(rn, rn1);
    }
  }
}

/* radix2.go:80-154, single-threaded (arithmetic identical to any worker split:
 * every butterfly is independent within a stage). Result left in *res. */
static int radix2(const cplx *x, cplx *out, int64_t n) {
  const cplx *factors = radix2_factors(n);
  cplx *r = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *t = (cplx *)malloc((size_t)n * sizeof(cplx));
  if (!r || !t) {
    free(r);
    free(t);
    return OR_ERR_NOMEM;
  }
  reorder(x, r, n);
  for (int64_t stage = 2; stage <= n; stage <<= 1) {
    stage_range(r, t, factors, stage, n / stage, 0, n);
    cplx *tmp = r;
    r = t;
    t = tmp;
  }
  memcpy(out, r, (size_t)n * sizeof(cplx));
  free(r);
  free(t);
  return OR_OK;
}

static int fft_c(const cplx *x, cplx *out, int64_t n);

/* ---- fft.go:35-52 -------------------------------------------------------- */
static int ifft_c(const cplx *x, cplx *out, int64_t n) {
  if (n <= 0) return OR_ERR_EMPTY; /* reference: index out of range panic */
  cplx *r = (cplx *)malloc((size_t)n * sizeof(cplx));
  if (!r) return OR_ERR_NOMEM;
  r[0] = x[0];
  for (int64_t i = 1; i < n; i++) r[i] = x[n - i];
  int st = fft_c(r, out, n);
  free(r);
  if (st) return st;
  double N = (double)n;
  for (int64_t i = 0; i < n; i++) {
    out[i].re /= N;
    out[i].im /= N;
  }
  return OR_OK;
}

/* ---- fft.go:55-69 -------------------------------------------------------- */
static int convolve_c(const cplx *x, const cplx *y, cplx *out, int64_t n) {
  cplx *fx = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *fy = (cplx *)malloc((size_t)n * sizeof(cplx));
  int st = OR_ERR_NOMEM;
  if (fx && fy) {
    st = fft_c(x, fx, n);
    if (!st) st = fft_c(y, fy, n);
    if (!st) {
      for (int64_t i = 0; i < n; i++) fx[i] = cmul(fx[i], fy[i]);
      st = ifft_c(fx, out, n);
    }
  }
  free(fx);
  free(fy);
  return st;
}

/* ---- bluestein.go:32-61 (chirp cache, angle Pi/N*k*k, k=0 exact) ---------
 * and bluestein.go:68-94 (a = x*conj(w) zero-padded to M, b symmetric, r =
 * Convolve(a, b), X = r*conj(w), first N). */
static int bluestein(const cplx *x, cplx *out, int64_t n) {
  int64_t m = or_next_pow2(n * 2 - 1);
  cplx *w = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *wi = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *a = (cplx *)calloc((size_t)m, sizeof(cplx));
  cplx *b = (cplx *)calloc((size_t)m, sizeof(cplx));
  cplx *r = (cplx *)malloc((size_t)m * sizeof(cplx));
  int st = OR_ERR_NOMEM;
  if (w && wi && a && b && r) {
    for (int64_t i = 0; i < n; i++) {
      double s, c;
      if (i == 0) {
        s = 0;
        c = 1;
      } else {
        sincos(M_PI / (double)n * (double)(i * i), &s, &c);
      }
      w[i] = (cplx){c, s};
      wi[i] = (cplx){c, -s};
    }
    for (int64_t i = 0; i < n; i++) a[i] = cmul(x[i], wi[i]);
    for (int64_t i = 0; i < n; i++) {
      b[i] = w[i];
      if (i != 0) b[m - i] = w[i];
    }
    st = convolve_c(a, b, r, m);
    if (!st)
      for (int64_t i = 0; i < n; i++) out[i] = cmul(r[i], wi[i]);
  }
  free(w);
  free(wi);
  free(a);
  free(b);
  free(r);
  return st;
}

/* ---- fft.go:72-87 -------------------------------------------------------- */
static int fft_c(const cplx *x, cplx *out, int64_t n) {
  if (n < 0) return OR_ERR_INVALID;
  if (n <= 1) {
    if (n == 1) out[0] = x[0];
    return OR_OK;
  }
  if (or_is_pow2(n)) return radix2(x, out, n);
  return bluestein(x, out, n);
}

int or_fft(const double *x, double *out, int64_t n) {
  return fft_c((const cplx *)x, (cplx *)out, n);
}
int or_ifft(const double *x, double *out, int64_t n) {
  return ifft_c((const cplx *)x, (cplx *)out, n);
}
int or_convolve(const double *x, const double *y, double *out, int64_t n) {
  return convolve_c((const cplx *)x, (const cplx *)y, (cplx *)out, n);
}

/* fft.go:25-32 via dsputils.ToComplex (dsputils.go:25-31) */
static cplx *to_complex(const double *x, int64_t n) {
  cplx *c = (cplx *)malloc((size_t)(n > 0 ? n : 1) * sizeof(cplx));
  if (!c) return NULL;
  for (int64_t i = 0; i < n; i++) c[i] = (cplx){x[i], 0};
  return c;
}
int or_fft_real(const double *x, double *out, int64_t n) {
  cplx *c = to_complex(x, n);
  if (!c) return OR_ERR_NOMEM;
  int st = fft_c(c, (cplx *)out, n);
  free(c);
  return st;
}
int or_ifft_real(const double *x, double *out, int64_t n) {
  cplx *c = to_complex(x, n);
  if (!c) return OR_ERR_NOMEM;
  int st = ifft_c(c, (cplx *)out, n);
  free(c);
  return st;
}

/* ---- fft.go:123-154: column pass (gather, FFT, scatter) then row pass ---- */
int or_fft2(const double *xd, double *outd, int64_t rows, int64_t cols, int inverse) {
  const cplx *x = (const cplx *)xd;
  cplx *r = (cplx *)outd;
  if (rows <= 0) return OR_ERR_EMPTY;
  int (*f)(const cplx *, cplx *, int64_t) = inverse ? ifft_c : fft_c;
  cplx *t = (cplx *)malloc((size_t)rows * sizeof(cplx));
  cplx *ft = (cplx *)malloc((size_t)rows * sizeof(cplx));
  cplx *row = (cplx *)malloc((size_t)(cols > 0 ? cols : 1) * sizeof(cplx));
  int st = OR_ERR_NOMEM;
  if (t && ft && row) {
    st = OR_OK;
    for (int64_t i = 0; i < cols && !st; i++) {
      for (int64_t j = 0; j < rows; j++) t[j] = x[j * cols + i];
      st = f(t, ft, rows);
      for (int64_t nn = 0; nn < rows && !st; nn++) r[nn * cols + i] = ft[nn];
    }
    for (int64_t nn = 0; nn < rows && !st && cols > 0; nn++) {
      memcpy(row, r + nn * cols, (size_t)cols * sizeof(cplx));
      st = f(row, r + nn * cols, cols);
    }
  }
  free(t);
  free(ft);
  free(row);
  return st;
}

/* ---- fft.go:157-192 computeFFTN: fftFunc along every line of dimension 0,
 * then 1, ... (Matrix.Dim/SetDim, dsputils/matrix.go:110-177). The decrDim
 * enumeration order (fft.go:197-224) does not change any value. */
int or_fftn(const double *xd, double *outd, const int64_t *dims, int ndims, int inverse) {
  int64_t total = 1;
  for (int i = 0; i < ndims; i++) {
    if (dims[i] < 1) return OR_ERR_INVALID; /* "invalid dimensions" matrix.go:43 */
    total *= dims[i];
  }
  cplx *cur = (cplx *)outd;
  memcpy(cur, xd, (size_t)total * sizeof(cplx));
  int (*f)(const cplx *, cplx *, int64_t) = inverse ? ifft_c : fft_c;
  for (int d = 0; d < ndims; d++) {
    int64_t L = dims[d], inner = 1;
    for (int e = d + 1; e < ndims; e++) inner *= dims[e];
    int64_t outer = total / (L * inner);
    cplx *line = (cplx *)malloc((size_t)L * sizeof(cplx));
    cplx *res = (cplx *)malloc((size_t)L * sizeof(cplx));
    if (!line || !res) {
      free(line);
      free(res);
      return OR_ERR_NOMEM;
    }
    for (int64_t o = 0; o < outer; o++)
      for (int64_t i = 0; i < inner; i++) {
        cplx *base = cur + o * L * inner + i;
        for (int64_t j = 0; j < L; j++) line[j] = base[j * inner];
        int st = f(line, res, L);
        if (st) {
          free(line);
          free(res);
          return st;
        }
        for (int64_t j = 0; j < L; j++) base[j * inner] = res[j];
      }
    free(line);
    free(res);
  }
  return OR_OK;
}

/* ---- Reference-threaded radix-2 (radix2.go:89-151) ------------------------
 * A persistent pool of spinning workers stands in for the goroutines the
 * reference spawns per call (a goroutine hand-off costs well under a
 * microsecond; pthread creation or condition-variable wake-ups cost tens of
 * microseconds, which would make the restatement unfairly slow). Per stage
 * the caller chops [0, n) into contiguous ranges that are multiples of
 * `stage` and at least idx_diff = n/nworkers long (radix2.go:97-100,135-148),
 * the workers run the butterflies and the caller waits for all of them (the
 * WaitGroup, radix2.go:149). */
#include <sched.h>
#include <stdatomic.h>

typedef struct {
  int nthreads;
  pthread_t *th;
  int64_t starts[1024], ends[1024];
  int njobs;
  const cplx *r;
  cplx *t;
  const cplx *factors;
  int64_t stage, blocks;
  atomic_int gen, next_job, done, quit;
} pool_t;

static pool_t *g_pool;
static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;

static void *pool_worker(void *arg) {
  pool_t *p = (pool_t *)arg;
  int seen = 0;
  for (;;) {
    int spins = 0;
    while (atomic_load(&p->gen) == seen && !atomic_load(&p->quit)) {
      if (++spins > 4096) sched_yield();
    }
    if (atomic_load(&p->quit)) break;
    seen = atomic_load(&p->gen);
    for (;;) {
      int j = atomic_fetch_add(&p->next_job, 1);
      if (j >= p->njobs) break;
      stage_range(p->r, p->t, p->factors, p->stage, p->blocks, p->starts[j], p->ends[j]);
      atomic_fetch_add(&p->done, 1);
    }
  }
  return NULL;
}

static void pool_stop(pool_t *p) {
  atomic_store(&p->quit, 1);
  for (int i = 0; i < p->nthreads; i++) pthread_join(p->th[i], NULL);
  free(p->th);
  free(p);
}

static pool_t *get_pool(int nworkers) {
  pthread_mutex_lock(&g_pool_lock);
  if (g_pool && g_pool->nthreads != nworkers) {
    pool_stop(g_pool);
    g_pool = NULL;
  }
  if (!g_pool) {
    pool_t *p = (pool_t *)calloc(1, sizeof(pool_t));
    p->nthreads = nworkers;
    p->th = (pthread_t *)calloc((size_t)nworkers, sizeof(pthread_t));
    for (int i = 0; i < nworkers; i++) pthread_create(&p->th[i], NULL, pool_worker, p);
    g_pool = p;
  }
  pool_t *p = g_pool;
  pthread_mutex_unlock(&g_pool_lock);
  return p;
}

static int radix2_threaded(const cplx *x, cplx *out, int64_t n, int nworkers, pool_t *p) {
  const cplx *factors = radix2_factors(n);
  cplx *r = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *t = (cplx *)malloc((size_t)n * sizeof(cplx));
  if (!r || !t) {
    free(r);
    free(t);
    return OR_ERR_NOMEM;
  }
  reorder(x, r, n);
  int64_t idx_diff = n / nworkers;
  if (idx_diff < 2) idx_diff = 2;
  for (int64_t stage = 2; stage <= n; stage <<= 1) {
    p->r = r;
    p->t = t;
    p->factors = factors;
    p->stage = stage;
    p->blocks = n / stage;
    p->njobs = 0;
    for (int64_t start = 0, end = stage;;) {
      if (end - start >= idx_diff || end == n) {
        if (p->njobs < 1024) {
          p->starts[p->njobs] = start;
          p->ends[p->njobs] = end;
          p->njobs++;
        } else { /* fold into the last job: same arithmetic */
          p->ends[p->njobs - 1] = end;
        }
        if (end == n) break;
        start = end;
      }
      end += stage;
    }
    atomic_store(&p->done, 0);
    atomic_store(&p->next_job, 0);
    atomic_fetch_add(&p->gen, 1); /* publish the stage */
    int spins = 0;
    while (atomic_load(&p->done) < p->njobs) {
      if (++spins > 4096) sched_yield();
    }
    cplx *tmp = r;
    r = t;
    t = tmp;
  }
  memcpy(out, r, (size_t)n * sizeof(cplx));
  free(r);
  free(t);
  return OR_OK;
}

/* fft.FFT with the reference's worker pool for every radix-2 transform,
 * including the three inside Bluestein's Convolve (bluestein.go:87 ->
 * fft.go:60-68 -> radix2.go:80). Same arithmetic as or_fft. */
static int fft_t(const cplx *x, cplx *out, int64_t n, int nworkers);

static int ifft_t(const cplx *x, cplx *out, int64_t n, int nworkers) {
  if (n <= 0) return OR_ERR_EMPTY;
  cplx *r = (cplx *)malloc((size_t)n * sizeof(cplx));
  if (!r) return OR_ERR_NOMEM;
  r[0] = x[0];
  for (int64_t i = 1; i < n; i++) r[i] = x[n - i];
  int st = fft_t(r, out, n, nworkers);
  free(r);
  if (st) return st;
  for (int64_t i = 0; i < n; i++) {
    out[i].re /= (double)n;
    out[i].im /= (double)n;
  }
  return OR_OK;
}

static int bluestein_t(const cplx *x, cplx *out, int64_t n, int nworkers) {
  int64_t m = or_next_pow2(n * 2 - 1);
  cplx *wi = (cplx *)malloc((size_t)n * sizeof(cplx));
  cplx *a = (cplx *)calloc((size_t)m, sizeof(cplx));
  cplx *b = (cplx *)calloc((size_t)m, sizeof(cplx));
  cplx *fa = (cplx *)malloc((size_t)m * sizeof(cplx));
  cplx *fb = (cplx *)malloc((size_t)m * sizeof(cplx));
  cplx *r = (cplx *)malloc((size_t)m * sizeof(cplx));
  int st = OR_ERR_NOMEM;
  if (wi && a && b && fa && fb && r) {
    for (int64_t i = 0; i < n; i++) {
      double sn = 0, cs = 1;
      if (i != 0) sincos(M_PI / (double)n * (double)(i * i), &sn, &cs);
      wi[i] = (cplx){cs, -sn};
      b[i] = (cplx){cs, sn};
      if (i != 0) b[m - i] = b[i];
    }
    for (int64_t i = 0; i < n; i++) a[i] = cmul(x[i], wi[i]);
    st = fft_t(a, fa, m, nworkers);
    if (!st) st = fft_t(b, fb, m, nworkers);
    if (!st) {
      for (int64_t i = 0; i < m; i++) fa[i] = cmul(fa[i], fb[i]);
      st = ifft_t(fa, r, m, nworkers);
    }
    if (!st)
      for (int64_t i = 0; i < n; i++) out[i] = cmul(r[i], wi[i]);
  }
  free(wi);
  free(a);
  free(b);
  free(fa);
  free(fb);
  free(r);
  return st;
}

static int fft_t(const cplx *x, cplx *out, int64_t n, int nworkers) {
  if (n <= 1) {
    if (n == 1) out[0] = x[0];
    return OR_OK;
  }
  if (or_is_pow2(n)) return radix2_threaded(x, out, n, nworkers, get_pool(nworkers));
  return bluestein_t(x, out, n, nworkers);
}

int or_fft_threaded(const double *x, double *out, int64_t n, int nworkers) {
  if (nworkers <= 0) nworkers = 1;
  return fft_t((const cplx *)x, (cplx *)out, n, nworkers);
}

int or_fft_rows_threaded(const double *x, double *out, int64_t n, int64_t rows,
                         int nworkers) {
  for (int64_t i = 0; i < rows; i++) {
    int st = or_fft_threaded(x + 2 * n * i, out + 2 * n * i, n, nworkers);
    if (st) return st;
  }
  return OR_OK;
}

/* ---- window/window.go ------------------------------------------------------ */
int or_window(int kind, int64_t L, double *r) {
  if (L <= 0) return L == 0 ? OR_OK : OR_ERR_INVALID;
  if (kind == OR_WIN_RECTANGULAR) { /* :32-40 */
    for (int64_t i = 0; i < L; i++) r[i] = 1;
    return OR_OK;
  }
  if (L == 1) {
    r[0] = 1;
    return OR_OK;
  }
  int64_t N = L - 1;
  switch (kind) {
    case OR_WIN_HANN: { /* :62-76 */
      double coef = 2 * M_PI / (double)N;
      for (int64_t n = 0; n <= N; n++) r[n] = 0.5 * (1 - cos(coef * (double)n));
      return OR_OK;
    }
    case OR_WIN_HAMMING: { /* :44-58 */
      double coef = M_PI * 2 / (double)N;
      for (int64_t n = 0; n <= N; n++) r[n] = 0.54 - 0.46 * cos(coef * (double)n);
      return OR_OK;
    }
    case OR_WIN_BARTLETT: { /* :80-98 */
      double coef = 2 / (double)N;
      int64_t n = 0;
      for (; n <= N / 2; n++) r[n] = coef * (double)n;
      for (; n <= N; n++) r[n] = 2 - coef * (double)n;
      return OR_OK;
    }
    case OR_WIN_FLATTOP: { /* :102-135 */
      const double a0 = 0.21557895, a1 = 0.41663158, a2 = 0.277263158, a3 = 0.083578947,
                   a4 = 0.006947368;
      double coef = 2 * M_PI / (double)N;
      for (int64_t n = 0; n <= N; n++) {
        double f = (double)n * coef;
        double t0 = a0, t1 = a1 * cos(f), t2 = a2 * cos(2 * f), t3 = a3 * cos(3 * f),
               t4 = a4 * cos(4 * f);
        r[n] = t0 - t1 + t2 - t3 + t4;
      }
      return OR_OK;
    }
    case OR_WIN_BLACKMAN: { /* :138-152 */
      for (int64_t n = 0; n <= N; n++) {
        double t1 = -0.5 * cos(2 * M_PI * (double)n / (double)N);
        double t2 = 0.08 * cos(4 * M_PI * (double)n / (double)N);
        r[n] = 0.42 + t1 + t2;
      }
      return OR_OK;
    }
  }
  return OR_ERR_INVALID;
}

/* ---- spectral/spectral.go:22-47 (count only; segments are index ranges) -- */
int64_t or_segment_count(int64_t lx, int64_t size, int64_t noverlap) {
  int64_t stride = size - noverlap;
  if (lx == size) return 1;
  if (lx > size) {
    if (stride <= 0) return -1; /* Go: integer divide by zero panic */
    return (lx - size) / stride + 1;
  }
  return 0;
}

/* ---- spectral/pwelch.go:74-145 ------------------------------------------- */
static int pwelch_impl(const double *x_in, int64_t n, double fs, int64_t nfft, int64_t pad,
                       int64_t noverlap, int window_kind, int scale_off, double *pxx,
                       double *freqs, int64_t *lp_out, int nworkers);

int or_pwelch(const double *x_in, int64_t n, double fs, int64_t nfft, int64_t pad,
              int64_t noverlap, int window_kind, int scale_off, double *pxx,
              double *freqs, int64_t *lp_out) {
  return pwelch_impl(x_in, n, fs, nfft, pad, noverlap, window_kind, scale_off, pxx, freqs,
                     lp_out, 0);
}

int or_pwelch_threaded(const double *x_in, int64_t n, double fs, int64_t nfft, int64_t pad,
                       int64_t noverlap, int window_kind, int scale_off, double *pxx,
                       double *freqs, int64_t *lp_out, int nworkers) {
  return pwelch_impl(x_in, n, fs, nfft, pad, noverlap, window_kind, scale_off, pxx, freqs,
                     lp_out, nworkers < 1 ? 1 : nworkers);
}

static int pwelch_impl(const double *x_in, int64_t n, double fs, int64_t nfft, int64_t pad,
                       int64_t noverlap, int window_kind, int scale_off, double *pxx,
                       double *freqs, int64_t *lp_out, int nworkers) {
  if (n == 0) {
    *lp_out = 0;
    return OR_OK;
  }
  if (nfft == 0) nfft = 256;
  if (pad == 0) pad = nfft;
  const double *x = x_in;
  double *xpad = NULL;
  int64_t lx = n;
  if (n < nfft) { /* dsputils.ZeroPadF(x, nfft) */
    xpad = (double *)calloc((size_t)nfft, sizeof(double));
    if (!xpad) return OR_ERR_NOMEM;
    memcpy(xpad, x_in, (size_t)n * sizeof(double));
    x = xpad;
    lx = nfft;
  }
  int64_t lp = pad / 2 + 1;
  int64_t nsegs = or_segment_count(lx, nfft, noverlap);
  if (nsegs < 0) {
    free(xpad);
    return OR_ERR_INVALID;
  }
  int64_t stride = nfft - noverlap;
  /* ZeroPadF(seg, pad) keeps the segment if pad <= nfft: FFT length is the max */
  int64_t flen = pad > nfft ? pad : nfft;
  double *seg = (double *)malloc((size_t)flen * sizeof(double));
  double *win = (double *)malloc((size_t)flen * sizeof(double));
  double *pg = (double *)malloc((size_t)flen * 2 * sizeof(double));
  double *cbuf = (double *)malloc((size_t)flen * 2 * sizeof(double));
  if (!seg || !win || !pg || !cbuf) {
    free(seg);
    free(win);
    free(pg);
    free(cbuf);
    free(xpad);
    return OR_ERR_NOMEM;
  }
  /* window.Apply(x, wf) computes wf(len(x)) = wf(flen) (window.go:25-29) */
  or_window(window_kind, flen, win);
  for (int64_t j = 0; j < lp; j++) pxx[j] = 0;
  for (int64_t s = 0; s < nsegs; s++) {
    memcpy(seg, x + s * stride, (size_t)nfft * sizeof(double));
    for (int64_t i = nfft; i < flen; i++) seg[i] = 0;
    for (int64_t i = 0; i < flen; i++) seg[i] *= win[i];
    if (nworkers > 0) { /* FFTReal (ToComplex + FFT) with the reference's worker pool */
      for (int64_t i = 0; i < flen; i++) {
        cbuf[2 * i] = seg[i];
        cbuf[2 * i + 1] = 0;
      }
      or_fft_threaded(cbuf, pg, flen, nworkers);
    } else {
      or_fft_real(seg, pg, flen);
    }
    for (int64_t j = 0; j < lp; j++) {
      double a = pg[2 * j], b = pg[2 * j + 1];
      /* real(conj(z)*z) = a*a - (-b)*b */
      double d = (a * a - (-b) * b) / (double)nsegs;
      if (j > 0 && j < lp - 1) d *= 2;
      pxx[j] += d;
    }
  }
  /* norm = sum(wf(nfft)^2), times Fs unless Scale_off (:124-136) */
  double *wn = (double *)malloc((size_t)nfft * sizeof(double));
  or_window(window_kind, nfft, wn);
  double norm = 0;
  for (int64_t i = 0; i < nfft; i++) norm += wn[i] * wn[i];
  if (!scale_off) norm *= fs;
  for (int64_t j = 0; j < lp; j++) pxx[j] /= norm;
  double coef = fs / (double)pad;
  for (int64_t j = 0; j < lp; j++) freqs[j] = (double)j * coef;
  *lp_out = lp;
  free(wn);
  free(seg);
  free(win);
  free(pg);
  free(cbuf);
  free(xpad);
  return OR_OK;
}

/* ---- synthetic data (DESIGN.md §Synthetic data) ---------------------------- */
static inline uint64_t splitmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

void or_fill_uniform(double *out, int64_t count, uint64_t seed, uint64_t offset) {
  for (int64_t i = 0; i < count; i++) {
    uint64_t z = splitmix64(seed + (offset + (uint64_t)i + 1) * 0x9E3779B97F4A7C15ULL);
    out[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

/* wav/wav.go:135-161 (ReadFloats) over the bytes ReadSamples (:110-131) reads
 * with binary.LittleEndian. Go evaluates float32(v) - math.MinInt16 and the
 * division in float32 (the untyped constants convert to float32). */
int or_wav_floats(const void *in, int64_t count, int audio_format, int bits_per_sample,
                  float *out) {
  const unsigned char *b = (const unsigned char *)in;
  if (audio_format == 1) {
    if (bits_per_sample == 8) {
      for (int64_t i = 0; i < count; i++) {
        volatile float v = (float)b[i];
        out[i] = v / 255.0f;
      }
      return 0;
    }
    if (bits_per_sample == 16) {
      for (int64_t i = 0; i < count; i++) {
        const int16_t s = (int16_t)((uint16_t)b[2 * i] | ((uint16_t)b[2 * i + 1] << 8));
        volatile float num = (float)s - (-32768.0f);
        out[i] = num / 65535.0f;
      }
      return 0;
    }
    return -1;
  }
  if (audio_format == 3) {
    for (int64_t i = 0; i < count; i++) {
      uint32_t u = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) |
                   ((uint32_t)b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
      float f;
      memcpy(&f, &u, 4);
      out[i] = f;
    }
    return 0;
  }
  return -1;
}
