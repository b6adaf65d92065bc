// host_latency.cpp — where the time of one small synchronous host call goes
// (development tool; not part of the product library): an empty kernel
// launch + hipStreamSynchronize, the same with the stream polled by
// hipStreamQuery, a zero-copy kernel touching 24 KiB of mapped host memory,
// and gdsp_fft_real(n = 1024) through the C ABI (BASELINE configs[0]).
//
//   hipcc -O2 -std=c++17 -I include tools/host_latency.cpp -L go-dsp_amd/lib -lgdspfft \
//     -Wl,-rpath,'$ORIGIN/../../go-dsp_amd/lib' -o tools/bin/host_latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "gdsp_fft.h"

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void empty_kernel() {}
__global__ void touch_kernel(const double *in, double *out, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[2 * i] = out[2 * i + 1] = in[i];
}

using clk = std::chrono::steady_clock;
template <class F>
double avg_us(F f, int reps = 2000) {
  for (int i = 0; i < 100; ++i) f();
  const auto t0 = clk::now();
  for (int i = 0; i < reps; ++i) f();
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / reps;
}

int main() {
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 1024;
  double *h;
  void *d;
  CHECK(hipHostMalloc((void **)&h, 3 * n * sizeof(double), hipHostMallocMapped));
  CHECK(hipHostGetDevicePointer(&d, h, 0));
  std::vector<double> x(n), y(2 * n);
  for (int i = 0; i < n; ++i) x[i] = (double)(i % 17) - 8.0;
  for (int round = 0; round < 2; ++round) {
    printf("empty launch + hipStreamSynchronize   %7.2f us\n", avg_us([&] {
             hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
             (void)hipStreamSynchronize(s);
           }));
    printf("empty launch + hipStreamQuery spin    %7.2f us\n", avg_us([&] {
             hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
             while (hipStreamQuery(s) == hipErrorNotReady) {
             }
           }));
    printf("mapped 8+16 KiB kernel + sync         %7.2f us\n", avg_us([&] {
             memcpy(h, x.data(), n * sizeof(double));
             hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(256), 0, s, (const double *)d,
                                (double *)d + n, n);
             (void)hipStreamSynchronize(s);
             memcpy(y.data(), h + n, 2 * n * sizeof(double));
           }));
    printf("mapped 8+16 KiB kernel + spin         %7.2f us\n", avg_us([&] {
             memcpy(h, x.data(), n * sizeof(double));
             hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(256), 0, s, (const double *)d,
                                (double *)d + n, n);
             while (hipStreamQuery(s) == hipErrorNotReady) {
             }
             memcpy(y.data(), h + n, 2 * n * sizeof(double));
           }));
    printf("gdsp_fft_real(n = 1024)               %7.2f us\n", avg_us([&] {
             if (gdsp_fft_real(x.data(), y.data(), n) != GDSP_OK) {
               fprintf(stderr, "gdsp_fft_real: %s\n", gdsp_last_error());
               exit(1);
             }
           }));
  }
  return 0;
}
