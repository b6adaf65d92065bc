// fft_lds12.hip — fft_lds_kernel for N = 4096 (the BASELINE headline, a
// batched radix-2 FFT: fft/radix2.go:80-154) in its own translation unit, so
// it alone is compiled with the wave-priority pass (Makefile: each wave runs
// at raised priority until its row loads are issued): 1.3598 / 1.3414 against
// 1.3703 / 1.3515 ms per 65536 transforms; the same pass made the n = 3000
// mixed kernel 4 % and FFT2 1-2 % slower (scripts/archive/gpu_r03_flags.sh).
#include "lds_kernel.hpp"

namespace gdsp {

hipError_t launch_fft_lds12(bool inv, int load, bool split, const void *in, cd *out, int64_t batch,
                            const cd *tw, double scale, hipStream_t s) {
  // (round 4: the row by LDS-DMA instead of register loads measured 1.382 /
  // 1.471 against 1.379 ms, profiles/r04/lds12_dma_ab.txt: register loads stay)
  if (load == LOAD_COMPLEX)
    return inv ? launch_lds_s<12, true, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s)
               : launch_lds_s<12, false, LOAD_COMPLEX>(in, out, batch, tw, scale, split, s);
  return launch_lds_s<12, false, LOAD_REAL>(in, out, batch, tw, scale, split, s);
}

}  // namespace gdsp
