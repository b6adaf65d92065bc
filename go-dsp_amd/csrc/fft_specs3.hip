// fft_specs3.hip — compiled mixed-radix specialisations, group 3: 2560 .. 8000 (above 4096 the exchange goes through LDS as re/im halves).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last. Round 5 (scripts/archive/gpu_r05_spec6.sh, two
// alternating rounds, profiles/r05/radix_lists_ab.txt): lists whose passes
// keep more of the transform's threads busy (tools/spec_candidates.py) took
// 2880 from 20 9 16, 3200 from 20 10 16, 3840 from 20 12 16, 4500 from
// 25 9 20 and 6000 from 25 12 20: batched FFT -7 to -22 %, fused Pwelch
// (half overlap) -20 to -38 % (6000 equal); then (scripts/archive/gpu_r05_specd.sh)
// 8000 from 25 20 16 (-8 % / -20 %) and 5880 from 20 6 7 7 (-4 % / -12 %,
// Rader's 5881 -4 %). 2560, 4000 and the others keep their lists. Last
// (scripts/archive/gpu_r05_f1.sh), the four-pass lists the fused Pwelch got for
// itself (fft_specs0.hip, specspw) as FFT lists too: 5000 10 10 10 5 0.774
// against 0.942-0.945 ms per 2^27 samples, 7500 20 5 5 15 0.813-0.821
// against 0.876-0.879, 3750 15 5 5 10 0.938-0.946 against 0.986-0.992; 768,
// 1875, 2250, 2500, 3125 and 4000 were 2-13 % slower, 6000 and 6400 equal.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs3,
                Spec<16, 10, 16>,  // 2560
                Spec<16, 12, 15>,  // 2880
                Spec<25, 8, 16>,  // 3200
                Spec<15, 15, 16>,  // 3600
                Spec<15, 16, 16>,  // 3840
                Spec<25, 20, 8>,  // 4000
                Spec<15, 20, 15>,  // 4500
                Spec<20, 15, 16>,  // 4800
                Spec<10, 10, 10, 5>,  // 5000 (25 25 8 until late round 5)
                Spec<20, 16, 16>,  // 5120
                Spec<20, 20, 15>,  // 6000
                Spec<25, 16, 16>,  // 6400
                Spec<20, 5, 5, 15>,  // 7500 (25 15 20 until late round 5)
                Spec<16, 25, 20>,  // 8000
                Spec<25, 5, 25>,  // 3125 (four-step rows)
                Spec<12, 6, 7, 7>,  // 3528 (four-step rows)
                Spec<15, 5, 5, 10>,  // 3750 (four-step rows; 25 6 25 until late round 5)
                Spec<25, 5, 25, 2>,  // 6250 (four-step rows)
                Spec<15, 6, 7, 7>,  // 4410 (44.1 kHz audio frames)
                Spec<8, 7, 7, 15>)  // 5880 (44.1 kHz audio frames)
