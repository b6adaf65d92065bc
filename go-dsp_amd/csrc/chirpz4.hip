// chirpz4.hip — the four-pass fused chirp-z kernel (chirpz6k.hpp,
// chirpz4_kernel) for M = 16 * R1 * R2 * 16 (the table and dispatch:
// chirpz6k.hip)
#include "chirpz6k.hpp"

namespace gdsp {
GDSP_C4_LAUNCH(, 6, 6)
GDSP_C4_LAUNCH(, 8, 5)
GDSP_C4_LAUNCH(, 8, 6)
}  // namespace gdsp
