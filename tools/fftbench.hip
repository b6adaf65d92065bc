// fftbench.hip — kernel-variant A/B harness for the N=4096 batched transform
// (development tool; not part of the product library). Builds the same
// device building blocks as libgdspfft with different load/store policies,
// occupancy bounds and exchange layouts, times them in interleaved rounds in
// one process (cdna_hip_programming.md §5.4 rule 24), and checks every
// variant against variant 0 bit-for-bit-ish (max |diff|).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../go-dsp_amd/csrc fftbench.hip -o fftbench
//   ./fftbench [batch] [rounds]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "fft_kernels.hip"

using namespace gdsp;
cd *g_chirp, *g_bhat, *g_tw8192;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <bool NT>
__device__ __forceinline__ cd ld(const cd *p) {
  if constexpr (NT) {
    return {__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y)};
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st(cd *p, cd v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
  } else {
    *p = v;
  }
}

// Variant kernel: LOG2N = 12 (T = 256, one transform per workgroup).
template <bool SPLIT, bool NTL, bool NTS, int MINW, bool XCD = false>
__global__ __launch_bounds__(256, MINW) void fft4096_v(const cd *__restrict__ in,
                                                        cd *__restrict__ out, int64_t batch,
                                                        const cd *__restrict__ tw) {
  using G = Geo<12>;
  __shared__ double lds[(SPLIT ? 1 : 2) * G::LDS_DOUBLES];
  const int t = threadIdx.x;
  int64_t g = blockIdx.x;
  if constexpr (XCD) {
    const int64_t nb = gridDim.x, full = nb & ~(int64_t)7;
    if (g < full) g = (g & 7) * (full >> 3) + (g >> 3);
  }
  double *lre = lds;
  double *lim = SPLIT ? lds : lds + G::LDS_DOUBLES;
  cd v[16];
  const cd *src = in + g * 4096;
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = ld<NTL>(src + t + k * 256);
  fft_regs<12, SPLIT>(v, t, tw, lre, lim);
  cd *dst = out + g * 4096;
#pragma unroll
  for (int k = 0; k < 16; ++k) st<NTS>(dst + t + k * 256, v[k]);
}

// No HBM traffic: registers seeded from the thread id, store only on an
// impossible condition (keeps the FFT live): the compute + LDS time alone.
template <int MINW>
__global__ __launch_bounds__(256, MINW) void fft4096_compute(const cd *__restrict__ in,
                                                             cd *__restrict__ out, int64_t batch,
                                                             const cd *__restrict__ tw) {
  using G = Geo<12>;
  __shared__ double lds[G::LDS_DOUBLES];
  const int t = threadIdx.x;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = {(double)(t + k + blockIdx.x), (double)(t - k)};
  fft_regs<12, true>(v, t, tw, lds, lds);
  double s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += v[k].x + v[k].y;
  if (s == 1.2345e300) out[t] = {s, s};
}

// Bluestein N=3000 / M=8192 variants (512 threads, 16 elements each)
template <int MINW, bool SB = false>
__global__ __launch_bounds__(512, MINW) void blu_v(const cd *__restrict__ in, cd *__restrict__ out,
                                                   int64_t batch, const cd *__restrict__ twm,
                                                   const cd *__restrict__ chirp,
                                                   const cd *__restrict__ bhat) {
  using G = Geo<13>;
  __shared__ double lds[G::LDS_DOUBLES];
  const int t = threadIdx.x;
  const int64_t g = blockIdx.x;
  const int n = 3000;
  cd v[16];
  const cd *src = in + g * n;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int idx = t + k * 512;
    v[k] = {0.0, 0.0};
    if (idx < n) v[k] = cmul(src[idx], chirp[idx]);
  }
  fft_regs<13, true>(v, t, twm, lds, lds, true);
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = conjg(cmul(v[k], bhat[t + k * 512]));
  int t2 = t;
  if constexpr (SB) asm volatile("" : "+s"(twm), "+v"(t2));
  fft_regs<13, true>(v, t2, twm, lds, lds, false);
  if constexpr (SB) asm volatile("" : "+s"(chirp), "+v"(t2));
  cd *dst = out + g * n;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int idx = t2 + k * 512;
    if (idx < n) dst[idx] = cmul(conjg(v[k]), chirp[idx]);
  }
}

// compute-only FFT-8192 (512 threads) and Bluestein-shaped double FFT
template <int NFFT, int LOG2E = 4>
__global__ __launch_bounds__((Geo<13, LOG2E>::WG)) void fft8192_compute(const cd *__restrict__ in,
                                                       cd *__restrict__ out, int64_t batch,
                                                       const cd *__restrict__ tw) {
  using G = Geo<13, LOG2E>;
  __shared__ double lds[G::LDS_DOUBLES];
  const int t = threadIdx.x;
  cd v[G::E];
#pragma unroll
  for (int k = 0; k < G::E; ++k) v[k] = {(double)(t + k + blockIdx.x), (double)(t - k)};
  fft_regs<13, true, true, LOG2E>(v, t, tw, lds, lds);
  if constexpr (NFFT == 2) fft_regs<13, true, true, LOG2E>(v, t, tw, lds, lds, false);
  double s = 0;
#pragma unroll
  for (int k = 0; k < G::E; ++k) s += v[k].x + v[k].y;
  if (s == 1.2345e300) out[t] = {s, s};
}

// Same memory pattern, no arithmetic: the ceiling of this access shape.
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy4096(const cd *__restrict__ in, cd *__restrict__ out,
                                                int64_t batch) {
  const int t = threadIdx.x;
  const int64_t g = blockIdx.x;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = ld<NTL>(in + g * 4096 + t + k * 256);
#pragma unroll
  for (int k = 0; k < 16; ++k) st<NTS>(out + g * 4096 + t + k * 256, v[k]);
}


// streaming-shape probes (ceilings for 16-B-per-lane read+write streams)
__global__ __launch_bounds__(256) void copy_one(const cd *__restrict__ in, cd *__restrict__ out,
                                                int64_t cnt) {
  const int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (i < cnt) out[i] = in[i];
}
template <int U>
__global__ __launch_bounds__(256) void copy_unroll(const cd *__restrict__ in,
                                                   cd *__restrict__ out, int64_t cnt) {
  const int64_t base = blockIdx.x * (int64_t)(256 * U) + threadIdx.x;
  cd v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < U; ++k) out[base + k * 256] = v[k];
}
template <int U>
__global__ __launch_bounds__(256) void copy_gs(const cd *__restrict__ in, cd *__restrict__ out,
                                               int64_t cnt) {
  for (int64_t base = blockIdx.x * (int64_t)(256 * U) + threadIdx.x; base < cnt;
       base += (int64_t)gridDim.x * 256 * U) {
    cd v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = in[base + k * 256];
#pragma unroll
    for (int k = 0; k < U; ++k) out[base + k * 256] = v[k];
  }
}
// 64 KiB per workgroup, each wave owning a contiguous 16 KiB quarter
__global__ __launch_bounds__(256) void copy_wave_contig(const cd *__restrict__ in,
                                                        cd *__restrict__ out, int64_t cnt) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t base = blockIdx.x * (int64_t)4096 + w * 1024 + l;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = in[base + k * 64];
#pragma unroll
  for (int k = 0; k < 16; ++k) out[base + k * 64] = v[k];
}
// our shape with an XCD-aware row map: the blocks one XCD runs (b % 8 equal)
// take consecutive rows
__global__ __launch_bounds__(256) void copy_xcd(const cd *__restrict__ in, cd *__restrict__ out,
                                                int64_t cnt) {
  const int64_t nb = gridDim.x;
  const int64_t row = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int64_t base = row * 4096 + threadIdx.x;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < 16; ++k) out[base + k * 256] = v[k];
}
// XCD map + each wave owning a contiguous 16 KiB quarter of the row
__global__ __launch_bounds__(256) void copy_xcd_wc(const cd *__restrict__ in, cd *__restrict__ out,
                                                   int64_t cnt) {
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t base = row * 4096 + w * 1024 + l;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = in[base + k * 64];
#pragma unroll
  for (int k = 0; k < 16; ++k) out[base + k * 64] = v[k];
}
// XCD map, loads in two halves (8 in flight, then 8)
__global__ __launch_bounds__(256) void copy_xcd_half(const cd *__restrict__ in,
                                                     cd *__restrict__ out, int64_t cnt) {
  const int64_t row = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t base = row * 4096 + threadIdx.x;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < 8; ++k) out[base + k * 256] = v[k];
#pragma unroll
  for (int k = 8; k < 16; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 8; k < 16; ++k) out[base + k * 256] = v[k];
}
// two rows per 512-thread workgroup, 16 loads per thread
__global__ __launch_bounds__(512) void copy_two(const cd *__restrict__ in, cd *__restrict__ out,
                                                int64_t cnt) {
  const int64_t base = (blockIdx.x * (int64_t)2 + (threadIdx.x >> 8)) * 4096 + (threadIdx.x & 255);
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < 16; ++k) out[base + k * 256] = v[k];
}
// our shape, stores in reverse k order (changes read/write interleaving)
__global__ __launch_bounds__(256) void copy_revst(const cd *__restrict__ in, cd *__restrict__ out,
                                                  int64_t cnt) {
  const int64_t base = blockIdx.x * (int64_t)4096 + threadIdx.x;
  cd v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 15; k >= 0; --k) out[base + k * 256] = v[k];
}
void l_cwc(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_wave_contig, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}
void l_cxcd(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_xcd, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}
void l_cxwc(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_xcd_wc, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}
void l_cxh(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_xcd_half, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}
void l_ctwo(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_two, dim3((unsigned)(b / 2)), dim3(512), 0, s, in, out, b * 4096);
}
void l_crev(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(copy_revst, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}

__global__ __launch_bounds__(256) void read_only(const cd *__restrict__ in, cd *__restrict__ out,
                                                 int64_t cnt) {
  const int64_t base = blockIdx.x * (int64_t)(256 * 16) + threadIdx.x;
  double s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    cd v = in[base + k * 256];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0].x = s;
}
__global__ __launch_bounds__(256) void write_only(const cd *__restrict__ in, cd *__restrict__ out,
                                                  int64_t cnt) {
  const int64_t base = blockIdx.x * (int64_t)(256 * 16) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 16; ++k) out[base + k * 256] = {1.0 * k, 2.0};
}

void l_copy_one(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  const int64_t cnt = b * 4096;
  hipLaunchKernelGGL(copy_one, dim3((unsigned)(cnt / 256)), dim3(256), 0, s, in, out, cnt);
}
template <int U>
void l_copy_unroll(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  const int64_t cnt = b * 4096;
  hipLaunchKernelGGL((copy_unroll<U>), dim3((unsigned)(cnt / 256 / U)), dim3(256), 0, s, in, out, cnt);
}
template <int U, int G>
void l_copy_gs(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  const int64_t cnt = b * 4096;
  hipLaunchKernelGGL((copy_gs<U>), dim3(G), dim3(256), 0, s, in, out, cnt);
}
void l_read(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(read_only, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}
void l_write(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  hipLaunchKernelGGL(write_only, dim3((unsigned)b), dim3(256), 0, s, in, out, b * 4096);
}

// production Pwelch / Bluestein kernels at different elements-per-thread
double *g_x1g, *g_win, *g_part;
template <int LOG2E>
void l_pwelch(const cd *in, cd *out, int64_t b, const cd *tw, hipStream_t s) {
  // 2^29 samples (the 4 GiB input buffer viewed as float64), NFFT 4096, 50 %
  using G = Geo<12, LOG2E>;
  const int64_t nsamp = (int64_t)1 << 29, nfft = 4096, stride = 2048;  // the 4 GiB input buffer
  const int64_t nseg = (nsamp - nfft) / stride + 1, npairs = (nseg + 1) / 2;
  const int64_t nworkers = 2048 * G::TPW;
  const int64_t ppw = (npairs + nworkers - 1) / nworkers;
  const int64_t nw = (npairs + ppw - 1) / ppw;
  hipLaunchKernelGGL((pwelch_kernel<12, true, LOG2E>), dim3((unsigned)((nw + G::TPW - 1) / G::TPW)),
                     dim3(G::WG), 0, s, (const double *)in, nfft, stride, (int64_t)0, nseg, ppw,
                     (const double *)g_win, tw, g_part);
}
template <int WM, int MINW = 1>
void l_pwelch_half(const cd *in, cd *out, int64_t b, const cd *tw, hipStream_t s) {
  const int64_t nsamp = (int64_t)1 << 29, nfft = 4096, stride = 2048;
  const int64_t nseg = (nsamp - nfft) / stride + 1, npairs = (nseg + 1) / 2;
  const int64_t nworkers = 2048;
  const int64_t ppw = (npairs + nworkers - 1) / nworkers;
  const int64_t nw = (npairs + ppw - 1) / ppw;
  launch_pwh_t<12, WM, MINW>((const double *)in, 0, nseg, ppw, nw, (const double *)g_win, tw, g_part, s);
}
template <int LOG2E>
void l_blu_prod(const cd *in, cd *out, int64_t b, const cd *, hipStream_t s) {
  using G = Geo<13, LOG2E>;
  hipLaunchKernelGGL((bluestein_kernel<13, false, true, LOG2E>), dim3((unsigned)((b + G::TPW - 1) / G::TPW)),
                     dim3(G::WG), 0, s, in, out, (int64_t)3000, b, g_tw8192, g_chirp, g_bhat, 1.0);
}

struct Variant {
  const char *name;
  void (*launch)(const cd *, cd *, int64_t, const cd *, hipStream_t);
  bool is_fft;
};

template <bool SPLIT, bool NTL, bool NTS, int MINW, bool XCD = false>
void launch_v(const cd *in, cd *out, int64_t batch, const cd *tw, hipStream_t s) {
  hipLaunchKernelGGL((fft4096_v<SPLIT, NTL, NTS, MINW, XCD>), dim3((unsigned)batch), dim3(256), 0, s,
                     in, out, batch, tw);
}
template <int NF, int LOG2E = 4>
void launch_comp8192(const cd *in, cd *out, int64_t batch, const cd *tw, hipStream_t s) {
  hipLaunchKernelGGL((fft8192_compute<NF, LOG2E>), dim3((unsigned)batch),
                     dim3(Geo<13, LOG2E>::WG), 0, s, in, out, batch, g_tw8192);
}
template <int MINW>
void launch_comp(const cd *in, cd *out, int64_t batch, const cd *tw, hipStream_t s) {
  hipLaunchKernelGGL((fft4096_compute<MINW>), dim3((unsigned)batch), dim3(256), 0, s, in, out,
                     batch, tw);
}
template <int MINW, bool SB = false>
void launch_blu(const cd *in, cd *out, int64_t batch, const cd *, hipStream_t s) {
  hipLaunchKernelGGL((blu_v<MINW, SB>), dim3((unsigned)batch), dim3(512), 0, s, in, out, batch,
                     g_tw8192, g_chirp, g_bhat);
}
template <bool NTL, bool NTS>
void launch_c(const cd *in, cd *out, int64_t batch, const cd *, hipStream_t s) {
  hipLaunchKernelGGL((copy4096<NTL, NTS>), dim3((unsigned)batch), dim3(256), 0, s, in, out, batch);
}

__global__ void fill(double *p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ULL + 0x5EED;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

int main(int argc, char **argv) {
  const int64_t batch = argc > 1 ? atoll(argv[1]) : 65536;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const int64_t n = 4096;
  const size_t bytes = (size_t)batch * n * sizeof(cd);
  cd *in, *out, *ref, *tw;
  CHECK(hipMalloc(&in, bytes));
  CHECK(hipMalloc(&out, bytes));
  CHECK(hipMalloc(&ref, bytes));
  CHECK(hipMalloc(&tw, n * sizeof(cd)));
  std::vector<cd> h(n);
  for (int k = 0; k < n; ++k) {
    long double a = -2.0L * 3.141592653589793238462643383279502884L * k / n;
    h[k] = {(double)cosl(a), (double)sinl(a)};
  }
  CHECK(hipMemcpy(tw, h.data(), n * sizeof(cd), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (double *)in, (int64_t)(2 * batch * n));
  CHECK(hipMalloc(&g_chirp, 8192 * sizeof(cd)));
  CHECK(hipMalloc(&g_bhat, 8192 * sizeof(cd)));
  CHECK(hipMalloc(&g_tw8192, 8192 * sizeof(cd)));
  {
    std::vector<cd> t8(8192);
    for (int k = 0; k < 8192; ++k) {
      long double a = -2.0L * 3.141592653589793238462643383279502884L * k / 8192;
      t8[k] = {(double)cosl(a), (double)sinl(a)};
    }
    CHECK(hipMemcpy(g_tw8192, t8.data(), 8192 * sizeof(cd), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(g_chirp, t8.data(), 8192 * sizeof(cd), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(g_bhat, t8.data(), 8192 * sizeof(cd), hipMemcpyHostToDevice));
    std::vector<double> w(4096);
    for (int i = 0; i < 4096; ++i) w[i] = 0.5 * (1 - cos(2 * M_PI * i / 4095.0));
    CHECK(hipMalloc(&g_win, 4096 * sizeof(double)));
    CHECK(hipMemcpy(g_win, w.data(), 4096 * sizeof(double), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&g_part, (size_t)2 * 2048 * 4096 * sizeof(double)));
  }
  CHECK(hipDeviceSynchronize());

  std::vector<Variant> vs = {
      {"split", launch_v<true, false, false, 1>, true},
      {"split_xcd", launch_v<true, false, false, 1, true>, true},
      {"twobuf_xcd", launch_v<false, false, false, 1, true>, true},
      {"split_w3_xcd", launch_v<true, false, false, 3, true>, true},
      {"split_ntl", launch_v<true, true, false, 1>, true},
      {"split_nts", launch_v<true, false, true, 1>, true},
      {"split_ntl_nts", launch_v<true, true, true, 1>, true},
      {"split_w4", launch_v<true, false, false, 4>, true},
      {"split_w3", launch_v<true, false, false, 3>, true},
      {"twobuf", launch_v<false, false, false, 1>, true},
      {"twobuf_w3", launch_v<false, false, false, 3>, true},
      {"compute_only", launch_comp<1>, false},
      {"compute_only_w4", launch_comp<4>, false},
      {"comp8192_x1", launch_comp8192<1>, false},
      {"comp8192_x2", launch_comp8192<2>, false},
      {"comp8192_x1_e32", launch_comp8192<1, 5>, false},
      {"comp8192_x2_e32", launch_comp8192<2, 5>, false},
      {"blu_prod_e32", l_blu_prod<5>, false},
      {"pwelch_e16", l_pwelch<4>, false},
      {"pwelch_e8", l_pwelch<3>, false},
      {"pwelch_half_wreg", l_pwelch_half<0>, false},
      {"pwelch_half_wglb", l_pwelch_half<1>, false},
      {"pwelch_half_wlds", l_pwelch_half<2>, false},
      {"pwelch_half_wlds_w3", l_pwelch_half<2, 3>, false},
      {"pwelch_half_wlds_w4", l_pwelch_half<2, 4>, false},
      {"blu_prod_e16", l_blu_prod<4>, false},
      {"blu_prod_e8", l_blu_prod<3>, false},
      {"blu3000", launch_blu<1>, false},
      {"blu3000_w4", launch_blu<4>, false},
      {"blu3000_w3", launch_blu<3>, false},
      {"blu3000_sb", launch_blu<1, true>, false},
      {"blu3000_sb_w4", launch_blu<4, true>, false},
      {"copy", launch_c<false, false>, false},
      {"copy_ntl_nts", launch_c<true, true>, false},
      {"copy_one", l_copy_one, false},
      {"copy_wave_contig", l_cwc, false},
      {"copy_xcd", l_cxcd, false},
      {"copy_xcd_wc", l_cxwc, false},
      {"copy_xcd_half", l_cxh, false},
      {"copy_two", l_ctwo, false},
      {"copy_revst", l_crev, false},
      {"copy_u2", l_copy_unroll<2>, false},
      {"copy_u4", l_copy_unroll<4>, false},
      {"copy_u8", l_copy_unroll<8>, false},
      {"copy_gs4_2048", l_copy_gs<4, 2048>, false},
      {"copy_gs4_4096", l_copy_gs<4, 4096>, false},
      {"copy_gs8_1024", l_copy_gs<8, 1024>, false},
      {"copy_gs1_8192", l_copy_gs<1, 8192>, false},
      {"read_only(x2)", l_read, false},
      {"write_only(x2)", l_write, false},
  };
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // reference output
  vs[0].launch(in, ref, batch, tw, s);
  CHECK(hipStreamSynchronize(s));
  std::vector<std::vector<float>> times(vs.size());
  const int reps = 5;
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      vs[i].launch(in, out, batch, tw, s);  // warm
      CHECK(hipEventRecord(e0, s));
      for (int k = 0; k < reps; ++k) vs[i].launch(in, out, batch, tw, s);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      times[i].push_back(ms / reps);
      CHECK(hipGetLastError());
    }
  }
  // correctness vs variant 0
  std::vector<cd> a(n * 64), b(n * 64);
  for (size_t i = 0; i < vs.size(); ++i) {
    vs[i].launch(in, out, batch, tw, s);
    CHECK(hipStreamSynchronize(s));
    double md = 0;
    if (vs[i].is_fft) {
      for (int64_t off : {(int64_t)0, batch / 2 * n, (batch - 64) * n}) {
        CHECK(hipMemcpy(a.data(), out + off, a.size() * sizeof(cd), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(b.data(), ref + off, b.size() * sizeof(cd), hipMemcpyDeviceToHost));
        for (size_t j = 0; j < a.size(); ++j)
          md = std::max(md, std::max(fabs(a[j].x - b[j].x), fabs(a[j].y - b[j].y)));
      }
    }
    std::vector<float> t = times[i];
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf("%-16s median %.4f ms  min %.4f ms  %7.1f GB/s  maxdiff %.3g\n", vs[i].name, med, t[0],
           2.0 * bytes / (med * 1e-3) / 1e9, md);
  }
  return 0;
}
