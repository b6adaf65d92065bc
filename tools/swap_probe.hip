// Probe of the cross-lane primitives pwelch_shfl.hip relies on (GPU):
// value (reg r, lane l) = 100 r + l, after each single-bit swap the element
// from (reg c, lane bit b) must sit at (reg bit := b, lane bit := c).
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ unsigned upd(unsigned old, unsigned src, int which) {
  switch (which) {
    case 0: return __builtin_amdgcn_update_dpp(old, src, 0x114, 0xF, 0xA, false);  // row_shr:4 banks 1,3
    case 1: return __builtin_amdgcn_update_dpp(old, src, 0x104, 0xF, 0x5, false);  // row_shl:4 banks 0,2
    case 2: return __builtin_amdgcn_update_dpp(old, src, 0x118, 0xF, 0xC, false);  // row_shr:8 banks 2,3
    default: return __builtin_amdgcn_update_dpp(old, src, 0x108, 0xF, 0x3, false);  // row_shl:8 banks 0,1
  }
}

__global__ void probe(unsigned *out) {
  const int l = threadIdx.x;
  unsigned x = 100 * 0 + l, y = 100 * 1 + l;
  // bit 2 (S = 4)
  unsigned nx = upd(x, y, 0), ny = upd(y, x, 1);
  out[0 * 128 + l] = nx;
  out[0 * 128 + 64 + l] = ny;
  nx = upd(x, y, 2); ny = upd(y, x, 3);
  out[1 * 128 + l] = nx;
  out[1 * 128 + 64 + l] = ny;
  auto p16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[2 * 128 + l] = p16[0];
  out[2 * 128 + 64 + l] = p16[1];
  auto p32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[3 * 128 + l] = p32[0];
  out[3 * 128 + 64 + l] = p32[1];
}

int main() {
  unsigned *d, h[512];
  hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const int bits[4] = {2, 3, 4, 5};
  int bad = 0;
  for (int t = 0; t < 4; ++t) {
    const int b = bits[t];
    for (int rr = 0; rr < 2; ++rr)
      for (int l = 0; l < 64; ++l) {
        // new (reg rr, lane l) holds old (reg = lane bit b of l, lane = l with bit b := rr)
        const int oreg = (l >> b) & 1, olane = (l & ~(1 << b)) | (rr << b);
        const unsigned want = 100 * oreg + olane, got = h[t * 128 + rr * 64 + l];
        if (got != want) {
          if (bad < 20) printf("bit %d reg %d lane %d: got %u want %u\n", b, rr, l, got, want);
          ++bad;
        }
      }
  }
  printf("swap probe: %d mismatches\n", bad);
  return bad != 0;
}
