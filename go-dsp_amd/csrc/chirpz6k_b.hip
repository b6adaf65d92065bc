// chirpz6k_b.hip — the fused chirp-z kernel (chirpz6k.hpp) for pass-B radices
// 18, 20, 21, 25 (M = 256 RB; the table and dispatch: chirpz6k.hip)
#include "chirpz6k.hpp"

namespace gdsp {
GDSP_C6_LAUNCH(, 18)
GDSP_C6_LAUNCH(, 20)
GDSP_C6_LAUNCH(, 21)
GDSP_C6_LAUNCH(, 25)
}  // namespace gdsp
