// fft_specs2.hip — compiled mixed-radix specialisations, group 2: 720 .. 2500.
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs2,
                Spec<20, 9, 4>,  // 720
                Spec<25, 5, 6>,  // 750
                Spec<16, 6, 8>,  // 768
                Spec<25, 8, 4>,  // 800 (25 2 16 until round 5, fft_specs0.hip)
                Spec<15, 15, 4>,  // 900
                Spec<15, 9, 8>,  // 1080
                Spec<16, 9, 8>,  // 1152
                Spec<16, 10, 8>,  // 1280
                Spec<15, 6, 16>,  // 1440
                Spec<20, 5, 16>,  // 1600
                Spec<15, 15, 8>,  // 1800
                Spec<15, 9, 16>,  // 2160
                Spec<25, 10, 10>,  // 2500
                Spec<25, 5, 9>,  // 1125 (four-step rows)
                Spec<9, 7, 7, 4>,  // 1764 (four-step rows)
                Spec<25, 3, 25>,  // 1875 (four-step rows)
                Spec<9, 3, 9, 9>,  // 2187
                Spec<25, 6, 15>,  // 2250 (four-step rows)
                Spec<9, 6, 7, 7>,  // 2646 (44.1 kHz audio frames)
                Spec<12, 5, 7, 7>)  // 2940 (44.1 kHz audio frames)
