// Issue cost of the cross-lane moves the shuffle kernels use, against FP64
// adds (GPU): one wave (and then 2 waves per SIMD over the whole chip) runs
// ITER iterations of 16 independent operations of one kind; clock64() per
// wave gives cycles per operation.
//   hipcc --offload-arch=gfx950 -O3 tools/xlane_rate.hip -o tools/xlane_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITER = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void rate(unsigned *out, long long *cyc, unsigned seed) {
  unsigned r[32];
  double d[16];
#pragma unroll
  for (int i = 0; i < 32; ++i) r[i] = seed * (i + 1) + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; ++i) d[i] = (double)r[i];
  const long long t0 = clock64();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (KIND == 0) {
        d[i] = d[i] + d[(i + 1) & 15];  // v_add_f64
      } else if constexpr (KIND == 1) {
        r[i] = __builtin_amdgcn_update_dpp(r[i], r[i + 16], 0x118, 0xF, 0xC, false);  // v_mov_b32_dpp
      } else if constexpr (KIND == 2) {
        auto p = __builtin_amdgcn_permlane16_swap(r[i], r[i + 16], false, false);
        r[i] = p[0];
        r[i + 16] = p[1];
      } else {
        auto p = __builtin_amdgcn_permlane32_swap(r[i], r[i + 16], false, false);
        r[i] = p[0];
        r[i + 16] = p[1];
      }
    }
  }
  const long long t1 = clock64();
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) acc ^= r[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= (unsigned)(long long)d[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int KIND>
void run(const char *name, int blocks, int threads) {
  unsigned *o;
  long long *c;
  const int waves = blocks * threads / 64;
  hipMalloc(&o, (size_t)blocks * threads * 4);
  hipMalloc(&c, (size_t)waves * 8);
  hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(threads), 0, 0, o, c, 7u);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(threads), 0, 0, o, c, 11u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  long long *h = new long long[waves];
  hipMemcpy(h, c, (size_t)waves * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < waves; ++i) s += (double)h[i];
  const double ops = 16.0 * ITER;
  printf("%-16s waves=%6d  clock64/op/wave=%7.2f  wall ns/op/wave-slot=%.3f\n", name, waves,
         s / waves / ops, ms * 1e6 / ops / ((double)waves / 1024.0));
  delete[] h;
  hipFree(o);
  hipFree(c);
}

int main() {
  for (int cfg = 0; cfg < 2; ++cfg) {
    const int blocks = cfg ? 512 : 1, threads = cfg ? 256 : 64;  // 1 wave / 2 waves per SIMD
    run<0>("v_add_f64", blocks, threads);
    run<1>("v_mov_b32_dpp", blocks, threads);
    run<2>("permlane16_swap", blocks, threads);
    run<3>("permlane32_swap", blocks, threads);
  }
  return 0;
}
