// chirpz6k_a.hip — the fused chirp-z kernel (chirpz6k.hpp) for pass-B radices
// 9, 10, 13, 14, 15, 16 (M = 256 RB; the table and dispatch: chirpz6k.hip)
#include "chirpz6k.hpp"

namespace gdsp {
GDSP_C6_LAUNCH(, 9)
GDSP_C6_LAUNCH(, 10)
GDSP_C6_LAUNCH(, 13)
GDSP_C6_LAUNCH(, 14)
GDSP_C6_LAUNCH(, 15)
GDSP_C6_LAUNCH(, 16)
}  // namespace gdsp
