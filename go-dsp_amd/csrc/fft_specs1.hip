// fft_specs1.hip — compiled mixed-radix specialisations, group 1: short lengths (two passes where the radices allow).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last. Late in round 5 (scripts/archive/gpu_r05_specd.sh,
// profiles/r05/radix_lists_ab.txt) lists that keep more of a transform's
// threads busy in every pass replaced 100 (25 4), 300 (25 12), 360 (12 3 10),
// 400 (25 16), 600 (25 6 4), 640 (16 10 4) and 1470 (7 5 6 7): fused Pwelch
// per 2^28 samples -10 to -64 % (600: 2.98 -> 1.06 ms), batched FFT 0 to
// -11 %; Rader's 101 / 601 -17 / -9 %, 641 +8 %.
// Last (scripts/archive/gpu_r05_t12.sh, f2.sh), the three-pass lists the fused
// Pwelch took for 250 and 500 (1.62 -> 0.87 and 1.57 -> 0.86 ms per 2^28
// samples) as FFT lists too: 250 10 5 5 0.752 against 0.777-0.781 ms per
// 2^27 samples (Rader's 251 1.16 against 1.26), 500 10 5 10 0.760-0.762
// against 0.770-0.773.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs1,
                Spec<10, 10>,  // 100
                Spec<15, 8>,  // 120
                Spec<15, 10>,  // 150
                Spec<10, 16>,  // 160
                Spec<25, 8>,  // 200
                Spec<15, 16>,  // 240
                Spec<10, 5, 5>,  // 250 (25 10 until late round 5)
                Spec<15, 20>,  // 300
                Spec<20, 16>,  // 320
                Spec<15, 3, 8>,  // 360
                Spec<16, 25>,  // 400
                Spec<10, 5, 10>,  // 500 (25 20 until late round 5)
                Spec<15, 5, 8>,  // 600
                Spec<16, 8, 5>,  // 640
                Spec<25, 15>,  // 375 (four-step rows)
                Spec<25, 25>,  // 625 (four-step rows)
                Spec<7, 3, 6, 7>,  // 882 (four-step rows)
                Spec<15, 7, 2, 7>,  // 1470 (44.1 kHz audio frames)
                Spec<9, 5, 7, 7>)  // 2205 (44.1 kHz audio frames)
