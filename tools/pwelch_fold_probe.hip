// pwelch_fold_probe.hip — compile-only probe (tools/resusage.py) of the
// NFFT 4096 / 50 % Pwelch kernels with the per-bin accumulators folded
// (acc[k] + acc[F - k]): the product row kernel
// (register prefetch, two waves per SIMD) and the development three-wave
// kernel (LDS-DMA stage, half exchange buffer), each with and without FOLD.
//   python3 tools/resusage.py tools/pwelch_fold_probe.hip pwelch_row
//   RESUSAGE_FLAGS="-mllvm -amdgpu-sched-strategy=max-ilp" ... (the product TU's flags)
// Not linked anywhere: the kernels and their launchers are the library's.
#include "../go-dsp_amd/csrc/pwelch_row.hip"
#include "../go-dsp_amd/csrc/dev/pwelch_row3.hip"

namespace gdsp {
template __global__ void pwelch_row_kernel<12, 4, true, 2, false>(
    const double *, int64_t, int64_t, int64_t, const double *, const cd *, double *);
template __global__ void pwelch_row_kernel<12, 4, true, 2, true>(
    const double *, int64_t, int64_t, int64_t, const double *, const cd *, double *);
template __global__ void pwelch_row3_kernel<true>(const double *, int64_t, int64_t, int64_t,
                                                  const double *, const cd *, double *);
}  // namespace gdsp
