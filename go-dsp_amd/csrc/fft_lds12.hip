// fft_lds12.hip — fft_lds_kernel for N = 4096 (the BASELINE headline, a
// batched radix-2 FFT: fft/radix2.go:80-154) in its own translation unit, so
// it alone is compiled with the wave-priority pass (Makefile: each wave runs
// at raised priority until its row loads are issued): 1.3598 / 1.3414 against
// 1.3703 / 1.3515 ms per 65536 transforms; the same pass made the n = 3000
// mixed kernel 4 % and FFT2 1-2 % slower (scripts/gpu_r03_flags.sh).
#include "lds_kernel.hpp"

namespace gdsp {

hipError_t launch_fft_lds12(bool inv, int load, bool split, const void *in, cd *out, int64_t batch,
                            const cd *tw, double scale, hipStream_t s) {
#ifdef GDSP_DEV_BUILD
  // the row by LDS-DMA (lds_kernel.hpp DMA), forward complex, split exchange
  if (const char *e = dev_switch("GDSP_LDS12_DMA");
      e && (e[0] == '1' || e[0] == '2') && load == LOAD_COMPLEX && !inv && split) {
    if (e[0] == '1')
      hipLaunchKernelGGL((fft_lds_kernel<12, false, LOAD_COMPLEX, true, 4, 1>), dim3((unsigned)batch),
                         dim3(256), 0, s, in, out, batch, tw, scale);
    else
      hipLaunchKernelGGL((fft_lds_kernel<12, false, LOAD_COMPLEX, true, 4, 2>), dim3((unsigned)batch),
                         dim3(256), 0, s, in, out, batch, tw, scale);
    return hipGetLastError();
  }
#endif
  if (load == LOAD_COMPLEX)
    return inv ? launch_lds_s<12, true, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s)
               : launch_lds_s<12, false, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s);
  return launch_lds_s<12, false, LOAD_REAL>(in, out, batch, tw, scale, split, s);
}

}  // namespace gdsp
