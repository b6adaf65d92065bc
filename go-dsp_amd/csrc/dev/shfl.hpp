// shfl.hpp — cross-lane register exchanges for gfx950 (no LDS): one lane
// bit swapped with one register bit of a register pair, element by element.
// The element at (register bit c, lane bit b) moves to (register bit b, lane
// bit c). Used by the FFT kernels whose last exchange stays inside the wave
// (pwelch_shfl.hip, bluestein_shfl.hip); tools/swap_probe.hip checks the
// primitives on the GPU.
#pragma once
#include "../fft_device.hpp"

namespace gdsp {

__device__ __forceinline__ unsigned lo32(double d) {
  return (unsigned)__builtin_bit_cast(unsigned long long, d);
}
__device__ __forceinline__ unsigned hi32(double d) {
  return (unsigned)(__builtin_bit_cast(unsigned long long, d) >> 32);
}
__device__ __forceinline__ double mk64(unsigned lo, unsigned hi) {
  return __builtin_bit_cast(double, (unsigned long long)lo | ((unsigned long long)hi << 32));
}

// Swap lane bit log2(S) (S = 4: bit 2, S = 8: bit 3) with a register bit:
// x holds the register-bit-0 element, y the register-bit-1 one. New x = y from
// lane l - S on the lanes with the bit set (row_shr, banks of those lanes
// only), new y = x from lane l + S on the others (row_shl); the lanes a bank
// mask leaves out keep their value, so no select is needed.
template <int S>
__device__ __forceinline__ void dpp_swap(double &x, double &y) {
  constexpr int SHR = 0x110 + S, SHL = 0x100 + S;
  constexpr int BSET = S == 4 ? 0xA : 0xC, BCLR = S == 4 ? 0x5 : 0x3;
  const unsigned xl = lo32(x), xh = hi32(x), yl = lo32(y), yh = hi32(y);
  const unsigned nxl = __builtin_amdgcn_update_dpp(xl, yl, SHR, 0xF, BSET, false);
  const unsigned nxh = __builtin_amdgcn_update_dpp(xh, yh, SHR, 0xF, BSET, false);
  const unsigned nyl = __builtin_amdgcn_update_dpp(yl, xl, SHL, 0xF, BCLR, false);
  const unsigned nyh = __builtin_amdgcn_update_dpp(yh, xh, SHL, 0xF, BCLR, false);
  x = mk64(nxl, nxh);
  y = mk64(nyl, nyh);
}

// lane bit 4 (ROW16) or 5 <-> register bit: v_permlane16_swap / 32_swap
template <bool ROW16>
__device__ __forceinline__ void perm_swap(double &x, double &y) {
  const unsigned xl = lo32(x), xh = hi32(x), yl = lo32(y), yh = hi32(y);
  if constexpr (ROW16) {
    const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    x = mk64(l[0], h[0]);
    y = mk64(l[1], h[1]);
  } else {
    const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    x = mk64(l[0], h[0]);
    y = mk64(l[1], h[1]);
  }
}

}  // namespace gdsp
