// mixed_specs.hpp — the groups of compiled mixed-radix specialisations
// (fft_specs*.hip, GDSP_SPEC_GROUP in mixed_fixed.hpp) as seen by fft_mixed.hip.
#pragma once
#include "launch.hpp"

namespace gdsp {
struct cd;
#define GDSP_DECL_SPEC_GROUP(NAME)                                                            \
  bool NAME##_find(int n, int *rad, int *npass);                                              \
  bool NAME##_launch(const MixedDesc &d, bool inv, int load, const void *in, cd *out,         \
                     int64_t batch, const cd *tw, double scale, hipStream_t s);              \
  int NAME##_pw_tpw(const MixedDesc &d, int64_t span);                                    \
  bool NAME##_pw_launch(const MixedDesc &d, const double *x, int64_t nfft, int64_t stride,    \
                        int64_t seg_begin, int64_t seg_end, int64_t ppw, int64_t nworkers,   \
                        const double *win, const cd *tw, double *partial, hipStream_t s);
GDSP_DECL_SPEC_GROUP(specs0)
GDSP_DECL_SPEC_GROUP(specs1)
GDSP_DECL_SPEC_GROUP(specs2)
GDSP_DECL_SPEC_GROUP(specs3)
GDSP_DECL_SPEC_GROUP(specspw)  // fused-Pwelch-only lists (fft_specs0.hip)
#undef GDSP_DECL_SPEC_GROUP
}  // namespace gdsp
