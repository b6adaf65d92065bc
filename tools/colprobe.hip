// colprobe.hip — memory-pattern probe for a one-pass FFT2 column kernel
// (development tool; not part of the product library). Question: can a
// workgroup that holds whole 8192-row columns, CW columns wide (16*CW bytes
// per row), stream a 8192 x 8192 complex128 matrix at near copy speed when
// the workgroups that share 128-B lines run at the same time on one XCD?
// Each variant loads its tile, does one LDS round trip per column (the
// exchange a real FFT needs), and stores the tile back to a second matrix.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 colprobe.hip -o colprobe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

struct __attribute__((aligned(16))) cd {
  double x, y;
};

constexpr int L = 8192;  // column length (rows)

// MAP 0: block b -> column block b; 1: XCD-aware (blocks b, b+8, b+16 ...
// share an XCD, so they get adjacent column blocks)
template <int CW, int WG, int MAP, bool NT>
__global__ __launch_bounds__(WG) void col_probe(const cd *__restrict__ in, cd *__restrict__ out,
                                                int64_t C) {
  constexpr int TPC = WG / CW;  // threads per column
  constexpr int E = L / TPC;    // elements per thread
  __shared__ double lds[L];     // one column's real (then imaginary) parts
  const int64_t nb = gridDim.x, b = blockIdx.x;
  int64_t cb = b;
  if (MAP == 1) cb = (b & 7) * (nb >> 3) + (b >> 3);
  const int lt = threadIdx.x;
  const int c = lt % CW, t = lt / CW;
  const int64_t col = cb * CW + c;
  cd v[E];
#pragma unroll
  for (int k = 0; k < E; ++k) {
    const cd *p = in + (int64_t)(t + k * TPC) * C + col;
    if (NT) v[k] = {__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y)};
    else v[k] = *p;
  }
  // per column: real parts through LDS in a permuted order, then imaginary
  for (int cc = 0; cc < CW; ++cc) {
    __syncthreads();
    if (c == cc) {
#pragma unroll
      for (int k = 0; k < E; ++k) lds[(t * E + k) ^ 1] = v[k].x;
    }
    __syncthreads();
    if (c == cc) {
#pragma unroll
      for (int k = 0; k < E; ++k) v[k].x = lds[(t * E + k) ^ 1];
    }
  }
#pragma unroll
  for (int k = 0; k < E; ++k) {
    cd *p = out + (int64_t)(t + k * TPC) * C + col;
    if (NT) {
      __builtin_nontemporal_store(v[k].x, &p->x);
      __builtin_nontemporal_store(v[k].y, &p->y);
    } else {
      *p = v[k];
    }
  }
}

__global__ void copy_kernel(const cd *__restrict__ in, cd *__restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    cd v = {__builtin_nontemporal_load(&in[i].x), __builtin_nontemporal_load(&in[i].y)};
    __builtin_nontemporal_store(v.x, &out[i].x);
    __builtin_nontemporal_store(v.y, &out[i].y);
  }
}

template <class F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int CW, int WG, int MAP, bool NT>
static void run(const cd *in, cd *out, int64_t C, int reps, const char *name) {
  const unsigned nb = (unsigned)(C / CW);
  float ms = time_ms(
      [&] { hipLaunchKernelGGL((col_probe<CW, WG, MAP, NT>), dim3(nb), dim3(WG), 0, 0, in, out, C); },
      reps);
  CHECK(hipGetLastError());
  const double bytes = 2.0 * (double)L * (double)C * sizeof(cd);
  printf("%-34s %8.3f ms  %6.2f TB/s\n", name, ms, bytes / ms / 1e9);
}

int main(int argc, char **argv) {
  const int64_t C = 8192;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const size_t n = (size_t)L * C;
  cd *in, *out;
  CHECK(hipMalloc(&in, n * sizeof(cd)));
  CHECK(hipMalloc(&out, n * sizeof(cd)));
  CHECK(hipMemset(in, 0, n * sizeof(cd)));
  float ms = time_ms([&] { hipLaunchKernelGGL(copy_kernel, dim3(8192), dim3(256), 0, 0, in, out, (int64_t)n); }, reps);
  printf("%-34s %8.3f ms  %6.2f TB/s\n", "contiguous copy (nt)", ms, 2.0 * n * sizeof(cd) / ms / 1e9);
  run<1, 512, 0, false>(in, out, C, reps, "CW=1 WG=512 plain");
  run<1, 512, 1, false>(in, out, C, reps, "CW=1 WG=512 xcd");
  run<1, 512, 1, true>(in, out, C, reps, "CW=1 WG=512 xcd nt");
  run<2, 1024, 0, false>(in, out, C, reps, "CW=2 WG=1024 plain");
  run<2, 1024, 1, false>(in, out, C, reps, "CW=2 WG=1024 xcd");
  run<2, 1024, 1, true>(in, out, C, reps, "CW=2 WG=1024 xcd nt");
  run<2, 512, 1, false>(in, out, C, reps, "CW=2 WG=512 xcd");
  CHECK(hipFree(in));
  CHECK(hipFree(out));
  return 0;
}
