// fft_specs0.hip — compiled mixed-radix specialisations, group 0: the original set (BASELINE config 3 is n = 3000).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs0,
                Spec<25, 15, 8>,  // 3000
                Spec<10, 10, 10>,  // 1000
                Spec<25, 5, 16>,  // 2000
                Spec<15, 10, 10>,  // 1500
                Spec<25, 6, 16>,  // 2400
                Spec<25, 3, 16>,  // 1200
                Spec<15, 8, 8>,  // 960
                Spec<15, 16, 8>,  // 1920
                Spec<15, 8, 4>,  // 480
                Spec<12, 16, 8>,  // 1536
                Spec<12, 16, 16>,  // 3072
                Spec<9, 7, 7>,  // 441 (44.1 kHz audio frames)
                Spec<15, 7, 7>,  // 735 (44.1 kHz audio frames)
                Spec<9, 3, 7, 7>)  // 1323 (44.1 kHz audio frames)
