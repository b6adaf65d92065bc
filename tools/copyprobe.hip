// copyprobe.hip — is the 6.29 TB/s float4 copy the ceiling for the row
// kernels' access shape? (development tool; not part of the product library)
// Each workgroup (256 threads) copies one 64 KiB row of a 65536-row matrix
// (the N = 4096 complex128 batch: 4 GiB in, 4 GiB out), rows XCD-remapped as
// in fft_lds_kernel:
//   0 registers: 16 global_load_dwordx4 (nt) per thread, then 16 nt stores
//   1 registers, loads with the default policy
//   2 LDS-DMA: 64 x 1 KiB buffer_load ... lds (nt) into LDS, ds_read_b128,
//     nt stores (MI355X_MICROARCH.md: LDS-DMA read streams 6.5-6.8 TB/s nt)
//   3 LDS-DMA with the default policy
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 copyprobe.hip -o copyprobe
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

using v4 = __attribute__((ext_vector_type(4))) unsigned;
constexpr int ROWB = 65536;  // bytes per row
constexpr int WG = 256;

__device__ __forceinline__ int64_t remap(int64_t b, int64_t nb) {
  const int64_t full = nb & ~(int64_t)7;
  return b < full ? (b & 7) * (full >> 3) + (b >> 3) : b;
}

template <int V>
__global__ __launch_bounds__(WG) void copy_row(const v4 *__restrict__ in, v4 *__restrict__ out,
                                               int64_t rows) {
  const int64_t g = remap(blockIdx.x, gridDim.x);
  const int t = threadIdx.x;
  const v4 *src = in + g * (ROWB / 16);
  v4 *dst = out + g * (ROWB / 16);
  constexpr int E = ROWB / 16 / WG;  // 16
  v4 x[E];
  if constexpr (V <= 1) {
#pragma unroll
    for (int k = 0; k < E; ++k) x[k] = V == 0 ? __builtin_nontemporal_load(&src[t + k * WG]) : src[t + k * WG];
  } else {
    __shared__ v4 lds[ROWB / 16];
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<v4 *>(src), (short)0, ROWB, 0x00020000);
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t lane16 = (uint32_t)(t & 63) * 16u;
#pragma unroll
    for (int i = 0; i < ROWB / 1024 / (WG / 64); ++i) {
      const int p = w + i * (WG / 64);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void *)((char *)lds + p * 1024), 16, lane16,
          __builtin_amdgcn_readfirstlane(p * 1024), 0, V == 2 ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E; ++k) x[k] = lds[t + k * WG];
  }
#pragma unroll
  for (int k = 0; k < E; ++k) __builtin_nontemporal_store(x[k], &dst[t + k * WG]);
}

int main(int argc, char **argv) {
  const int64_t rows = 65536;
  const size_t bytes = (size_t)rows * ROWB;
  v4 *a, *b;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMemset(a, 1, bytes));
  CHECK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](int v) {
    switch (v) {
      case 0: hipLaunchKernelGGL(copy_row<0>, dim3(rows), dim3(WG), 0, 0, a, b, rows); break;
      case 1: hipLaunchKernelGGL(copy_row<1>, dim3(rows), dim3(WG), 0, 0, a, b, rows); break;
      case 2: hipLaunchKernelGGL(copy_row<2>, dim3(rows), dim3(WG), 0, 0, a, b, rows); break;
      default: hipLaunchKernelGGL(copy_row<3>, dim3(rows), dim3(WG), 0, 0, a, b, rows); break;
    }
  };
  for (int v = 0; v < 4; ++v)
    for (int i = 0; i < 20; ++i) run(v);  // warm-up (clocks)
  CHECK(hipDeviceSynchronize());
  const char *name[4] = {"registers nt", "registers default", "LDS-DMA nt", "LDS-DMA default"};
  for (int round = 0; round < 3; ++round) {
    for (int v = 0; v < 4; ++v) {
      const int reps = 20;
      CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) run(v);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / reps;
      printf("%-18s %.4f ms  %.3f TB/s (read + write)\n", name[v], per, 2.0 * bytes / (per * 1e-3) / 1e12);
    }
  }
  CHECK(hipGetLastError());
  return 0;
}
