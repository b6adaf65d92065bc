// fp64peak.hip — measured FP64 vector FMA rate of the box (the peak the
// bench's fp64 roofline is quoted against). 16 independent FMA chains per
// lane, 1024 threads per workgroup, 8 workgroups per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void fma_loop(double *out, int iters, double a, double b) {
  double x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 1e-9 + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = fma(x[k], a, b);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += x[k];
  if (s == 12345.678) out[threadIdx.x] = s;  // keep the loop alive
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  double *d;
  hipMalloc(&d, 4096 * sizeof(double));
  const int blocks = p.multiProcessorCount * 16, iters = 20000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  fma_loop<<<blocks, 256>>>(d, 100, 0.999999, 1e-7);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) fma_loop<<<blocks, 256>>>(d, iters, 0.999999, 1e-7);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 5.0 * blocks * 256.0 * iters * 16 * 2;
  printf("{\"cus\": %d, \"clock_mhz\": %d, \"fp64_fma_tflops\": %.2f}\n", p.multiProcessorCount,
         p.clockRate / 1000, flop / (ms * 1e-3) / 1e12);
  return 0;
}
