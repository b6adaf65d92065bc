// chirpz6k_c.hip — the fused chirp-z kernel (chirpz6k.hpp) for pass-B radices
// 3 ... 6 (M = 256 RB, several transforms per workgroup; the table and
// dispatch: chirpz6k.hip)
#include "chirpz6k.hpp"

namespace gdsp {
GDSP_C6_LAUNCH(, 3)
GDSP_C6_LAUNCH(, 4)
GDSP_C6_LAUNCH(, 5)
GDSP_C6_LAUNCH(, 6)
}  // namespace gdsp
