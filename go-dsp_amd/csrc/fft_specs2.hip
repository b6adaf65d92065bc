// fft_specs2.hip — compiled mixed-radix specialisations, group 2: 720 .. 2500.
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last. Late in round 5 (scripts/archive/gpu_r05_specd.sh,
// profiles/r05/radix_lists_ab.txt) lists that keep more of a transform's
// threads busy in every pass replaced 720 (20 9 4), 750 (25 5 6), 1080
// (15 9 8), 1152 (16 9 8), 1280 (16 10 8), 2160 (15 9 16), 1125 (25 5 9) and
// 1875 (25 3 25): fused Pwelch per 2^28 samples -5 to -61 % (750: 3.13 ->
// 1.22 ms), batched FFT -8 to +2.5 % (2160); Rader's 751 / 1153 / 2161 -8 /
// -10 / -8 %.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs2,
                Spec<16, 15, 3>,  // 720
                Spec<15, 10, 5>,  // 750
                Spec<16, 6, 8>,  // 768
                Spec<25, 8, 4>,  // 800 (25 2 16 until round 5, fft_specs0.hip)
                Spec<15, 15, 4>,  // 900
                Spec<15, 6, 12>,  // 1080
                Spec<8, 12, 12>,  // 1152
                Spec<16, 5, 16>,  // 1280
                Spec<15, 6, 16>,  // 1440
                Spec<20, 5, 16>,  // 1600
                Spec<15, 15, 8>,  // 1800
                Spec<12, 12, 15>,  // 2160
                Spec<25, 10, 10>,  // 2500
                Spec<15, 15, 5>,  // 1125 (four-step rows)
                Spec<9, 7, 7, 4>,  // 1764 (four-step rows)
                Spec<25, 15, 5>,  // 1875 (four-step rows)
                Spec<9, 3, 9, 9>,  // 2187
                Spec<25, 6, 15>,  // 2250 (four-step rows)
                Spec<9, 6, 7, 7>,  // 2646 (44.1 kHz audio frames)
                Spec<12, 5, 7, 7>)  // 2940 (44.1 kHz audio frames)
