// fft_specs1.hip — compiled mixed-radix specialisations, group 1: short lengths (two passes where the radices allow).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs1,
                Spec<25, 4>,  // 100
                Spec<15, 8>,  // 120
                Spec<15, 10>,  // 150
                Spec<10, 16>,  // 160
                Spec<25, 8>,  // 200
                Spec<15, 16>,  // 240
                Spec<25, 10>,  // 250
                Spec<25, 12>,  // 300
                Spec<20, 16>,  // 320
                Spec<12, 3, 10>,  // 360
                Spec<25, 16>,  // 400
                Spec<25, 20>,  // 500
                Spec<25, 6, 4>,  // 600
                Spec<16, 10, 4>,  // 640
                Spec<25, 15>,  // 375 (four-step rows)
                Spec<25, 25>,  // 625 (four-step rows)
                Spec<7, 3, 6, 7>,  // 882 (four-step rows)
                Spec<7, 5, 6, 7>,  // 1470 (44.1 kHz audio frames)
                Spec<9, 5, 7, 7>)  // 2205 (44.1 kHz audio frames)
