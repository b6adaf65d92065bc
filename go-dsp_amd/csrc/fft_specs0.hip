// fft_specs0.hip — compiled mixed-radix specialisations, group 0: the original set (BASELINE config 3 is n = 3000).
// Each Spec is a radix list (first pass .. last pass); the batched transform
// and fused Pwelch kernels for it are instantiated here (mixed_fixed.hpp).
// Radix lists: as few passes as the radices <= 25 allow, full waves where
// possible, a power-of-2 radix last — and, since round 5, no pass with far
// more butterflies than the others: the fused Pwelch is compute-bound, and a
// list whose middle radix is small (25 5 16: 400 threads per transform for
// the radix-5 pass, 80 of them busy in the radix-25 one) leaves most of its
// waves idle in the other passes. Per 2^28 samples, fused Pwelch / batched
// FFT (scripts/archive/gpu_r05_specb.sh, profiles/r05/radix_lists_ab.txt): 2000
// 25 5 16 -> 25 20 4: 2.33 -> 1.36 ms (Noverlap 0: 1.22 -> 0.76) / 0.766 ->
// 0.745-0.751; 2400 25 6 16 -> 20 15 8: 1.90 -> 1.57 / 0.745 -> 0.748; 800
// 25 2 16 -> 25 8 4: 1.83 -> 1.30 / 0.824-0.839 -> 0.802-0.805. 1200: 25 12 4
// made the batched FFT 4 % faster but the Pwelch 20 % and Rader's 1201
// (which uses this list for 1200) 9 % slower; 15 5 16 (late in round 5,
// scripts/archive/gpu_r05_specd.sh: tools/spec_candidates.py's ranking, two lists per
// length against the default, two alternating rounds) is faster for all
// three: 1.42 -> 1.16 ms, 0.781-0.797 -> 0.743, 1201 1.52-1.59 -> 1.34-1.44
// ms per 2^27 samples. 1000 25 20 2 and 1500 25 15 4 were slower for both
// (Pwelch 1.15 -> 1.50, 1.26 -> 1.49 ms; FFT 0.78 -> 0.87, 0.76 -> 0.81).
// Then (scripts/archive/gpu_r05_specp.sh, six lists each) 2000 25 20 4 -> 10 10 20
// (Pwelch 1.37-1.38 -> 1.25 ms, FFT equal), 2400 20 15 8 -> 15 16 10 (1.51
// -> 1.26, FFT -1 %) and 1500 15 10 10 -> 15 20 5 (1.20-1.21 -> 1.08-1.09,
// FFT equal); 3000 keeps 25 15 8 for the FFT (every other list 5-15 % slower
// there) and gives the fused Pwelch its own list (specspw below).
// The other lists changed that way: fft_specs1..3.hip and
// profiles/r05/radix_lists_ab.txt.
#include "mixed_fixed.hpp"

GDSP_SPEC_GROUP(specs0,
                Spec<25, 15, 8>,  // 3000
                Spec<10, 10, 10>,  // 1000
                Spec<10, 10, 20>,  // 2000 (25 5 16, then 25 20 4 in round 5, see above)
                Spec<15, 20, 5>,  // 1500 (15 10 10 until late round 5)
                Spec<15, 16, 10>,  // 2400 (25 6 16, then 20 15 8 in round 5)
                Spec<15, 5, 16>,  // 1200
                Spec<15, 8, 8>,  // 960
                Spec<15, 16, 8>,  // 1920
                Spec<15, 8, 4>,  // 480
                Spec<12, 16, 8>,  // 1536
                Spec<12, 16, 16>,  // 3072
                Spec<9, 7, 7>,  // 441 (44.1 kHz audio frames)
                Spec<15, 7, 7>,  // 735 (44.1 kHz audio frames)
                Spec<9, 3, 7, 7>)  // 1323 (44.1 kHz audio frames)

// Fused-Pwelch-only lists (pwelch_fixed_radices, fft_mixed.hip): the batched
// FFT of these lengths keeps the list above, the fused Pwelch takes this one.
// 3000: 15 5 5 8 (four passes, 200 threads, every pass >= 94 % busy) runs the
// Pwelch at half overlap in 1.32-1.33 against 1.68 ms per 2^28 samples, but
// the batched FFT in 0.845 against 0.803-0.809 ms per 2^27 samples (HBM-bound
// there, where the extra exchange costs and the idle lanes do not)
// (scripts/archive/gpu_r05_specp.sh, profiles/r05/radix_lists_ab.txt).
// Four-pass lists for the others measured (scripts/archive/gpu_r05_specq.sh, three
// each, two alternating rounds): 6000 15 5 5 16 2.45 against 2.77-2.78 ms,
// 4000 10 10 10 4 1.53 against 1.74-1.75 ms; 4500, 800, 2880, 3200, 1536 and
// 2400 were slower or within 3 % and keep their FFT list.
// Then 16 more lengths, two four-pass lists each (scripts/archive/gpu_r05_s12.sh):
// nine faster, per 2^28 samples: 768 1.27-1.28 -> 0.99-1.01 ms, 1875 1.32
// -> 1.16, 2250 2.11-2.14 -> 1.45, 2500 1.71 -> 1.07, 3125 1.94 -> 1.65,
// 3750 2.45 -> 1.54, 5000 3.55 -> 1.44, 6400 2.89 -> 2.46-2.47, 7500 2.58 ->
// 2.45; 400, 441, 750, 1440, 2160, 2560 and 3072 keep their FFT list.
// (3750, 5000 and 7500 then took those lists for the FFT too: fft_specs3.hip.)
// 44.1 kHz frames (scripts/archive/gpu_r05_audio.sh, two lists each): 5880 15 7 7 8
// 2.44-2.45 against 2.69-2.70 ms; 4410, 2940 and 2646 keep their FFT list.
// Then 14 more (scripts/archive/gpu_r05_t12.sh): 500 10 5 10 0.85-0.87 against
// 1.57-1.58 ms, 250 10 5 5 0.87 against 1.62, 375 15 5 5 1.02-1.03 against
// 1.60, 200 10 2 10 0.88 against 1.19, 1152 12 2 4 12 1.02 against 1.32, 625
// 5 5 25 1.24 against 1.54, 320 16 20 0.93 against 0.99; 4800, 5120, 3600,
// 1600, 1800, 1920 and 960 keep their FFT list. (250 and 500 took theirs for the FFT
// too: fft_specs1.hip.)
// The short lengths last (scripts/archive/gpu_r05_c12.sh, 17 lengths): 735 7 7 15
// 1.28-1.29 against 1.35 ms, 900 15 4 15 1.17 against 1.19-1.21; the other 15
// (100 ... 1764) keep their FFT list.
GDSP_SPEC_GROUP(specspw,
                Spec<15, 5, 5, 8>,    // 3000 (fused Pwelch)
                Spec<10, 10, 10, 4>,  // 4000 (fused Pwelch)
                Spec<15, 5, 5, 16>,   // 6000 (fused Pwelch)
                Spec<12, 4, 4, 4>,    // 768 (fused Pwelch)
                Spec<15, 5, 5, 5>,    // 1875 (fused Pwelch)
                Spec<15, 2, 5, 15>,   // 2250 (fused Pwelch)
                Spec<10, 5, 5, 10>,   // 2500 (fused Pwelch)
                Spec<5, 5, 5, 25>,    // 3125 (fused Pwelch)
                Spec<5, 5, 16, 16>,   // 6400 (fused Pwelch)
                Spec<15, 7, 7, 8>,    // 5880 (fused Pwelch)
                Spec<5, 5, 25>,       // 625 (fused Pwelch)
                Spec<15, 5, 5>,       // 375 (fused Pwelch)
                Spec<10, 2, 10>,      // 200 (fused Pwelch)
                Spec<16, 20>,         // 320 (fused Pwelch)
                Spec<12, 2, 4, 12>,   // 1152 (fused Pwelch)
                Spec<7, 7, 15>,       // 735 (fused Pwelch)
                Spec<15, 4, 15>)      // 900 (fused Pwelch)
