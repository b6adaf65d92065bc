// fft_specs0.hip — compiled mixed-radix specialisations, group 0: the original set (BASELINE config 3 is n = 3000).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last — and, since round 5, no pass with far
// more butterflies than the others: the fused Pwelch is compute-bound, and a
// list whose middle radix is small (25 5 16: 400 threads per transform for
// the radix-5 pass, 80 of them busy in the radix-25 one) leaves most of its
// waves idle in the other passes. Per 2^28 samples, fused Pwelch / batched
// FFT (scripts/gpu_r05_specb.sh, profiles/r05/radix_lists_ab.txt): 2000
// 25 5 16 -> 25 20 4: 2.33 -> 1.36 ms (Noverlap 0: 1.22 -> 0.76) / 0.766 ->
// 0.745-0.751; 2400 25 6 16 -> 20 15 8: 1.90 -> 1.57 / 0.745 -> 0.748; 800
// 25 2 16 -> 25 8 4: 1.83 -> 1.30 / 0.824-0.839 -> 0.802-0.805. 1200: 25 12 4
// made the batched FFT 4 % faster but the Pwelch 20 % and Rader's 1201
// (which uses this list for 1200) 9 % slower; 15 5 16 (late in round 5,
// scripts/gpu_r05_specd.sh: tools/spec_candidates.py's ranking, two lists per
// length against the default, two alternating rounds) is faster for all
// three: 1.42 -> 1.16 ms, 0.781-0.797 -> 0.743, 1201 1.52-1.59 -> 1.34-1.44
// ms per 2^27 samples. 1000 25 20 2 and 1500 25 15 4 were slower for both
// (Pwelch 1.15 -> 1.50, 1.26 -> 1.49 ms; FFT 0.78 -> 0.87, 0.76 -> 0.81).
// The other lists changed that way: fft_specs1..3.hip and
// profiles/r05/radix_lists_ab.txt.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs0,
                Spec<25, 15, 8>,  // 3000
                Spec<10, 10, 10>,  // 1000
                Spec<25, 20, 4>,  // 2000 (25 5 16 until round 5, see above)
                Spec<15, 10, 10>,  // 1500
                Spec<20, 15, 8>,  // 2400 (25 6 16 until round 5)
                Spec<15, 5, 16>,  // 1200
                Spec<15, 8, 8>,  // 960
                Spec<15, 16, 8>,  // 1920
                Spec<15, 8, 4>,  // 480
                Spec<12, 16, 8>,  // 1536
                Spec<12, 16, 16>,  // 3072
                Spec<9, 7, 7>,  // 441 (44.1 kHz audio frames)
                Spec<15, 7, 7>,  // 735 (44.1 kHz audio frames)
                Spec<9, 3, 7, 7>)  // 1323 (44.1 kHz audio frames)
