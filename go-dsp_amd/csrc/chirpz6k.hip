// chirpz6k.hip — fused chirp-z (Bluestein, fft/bluestein.go:68-94) on the
// convolution length M = 16 * RB * 16: for 129 <= n <= 3200 the smallest
// such M >= 2n - 1 over the kept pass-B radices RB (kC6RB below). Round 3
// built RB = 24 (M = 6144, 2049 <= n <= 3072) and RB = 12 (3072); round 6
// measured every RB 2 ... 32 with an in-register DFT (pass B: dft3x for 24
// and 12 as measured, dft_m — native or coprime split — for the others;
// several transforms per workgroup below RB = 9, c6_fft_multi).
//
// bluestein.go:70 pads the circular convolution to NextPowerOf2(2n - 1)
// because its FFT is radix 2. Any M >= 2n - 1 gives the same linear
// convolution, hence the same DFT; where this kernel is taken its M is below
// the power of 2 (at most 1.5 (2n - 1), where the power of 2 is up to twice
// it). At M = 6144 the exchange buffer (48 KiB)
// and a 16-point-per-thread register set let two 384-thread workgroups share
// a CU at 128 VGPRs, where the M = 8192 kernel (bluestein_kernel<13>, 32
// points per thread, 256 VGPRs) runs two 256-thread ones.
//
// One workgroup per transform, T = max(M / 16, 256) threads (thread t):
//   premultiply  a[t + NA r] = x * conj(w), r < KN (n <= NA KN; rest zero),
//                NA = M / 16 (pass A and C butterflies)
//   FFT 1        pass A  R = 16, NS = 1:      DFT_16 of t + NA r (pruned input)
//                pass B  R = RB, NS = 16:     t < 256, inputs t + 256 r
//                pass C  R = 16, NS = 16 RB:  outputs t + NA r (natural order)
//   middle       v = conj(A * bhat) in registers: pass C's outputs are pass
//                A's inputs of FFT 2, so no exchange between the two FFTs
//   FFT 2        pass A, B, C again; the outputs r < KN are the wanted ones:
//                X = conj(v) * conj(w) (the rest of the last DFT is dead code)
// Stockham passes (fft_device.hpp): butterfly j of pass (R, NS) reads
// j + r M/R and writes (j / NS) NS R + j % NS + r NS, twiddle W_{NS R}^{(j %
// NS) r}. Exchanges go through one M-double LDS buffer, real then imaginary
// parts. Slots: after pass A (stride-16 writes) XOR-swizzled, i ^ ((i >> 4)
// & 15) — every 16-lane write group and 32-lane read group hits distinct
// banks; after pass B plain (16 contiguous writes, 32 contiguous reads).
#include "chirpz6k.hpp"

namespace gdsp {

GDSP_C6_LAUNCH(, 12)
GDSP_C6_LAUNCH(, 24)
GDSP_C6_LAUNCH(extern, 3)
GDSP_C6_LAUNCH(extern, 4)
GDSP_C6_LAUNCH(extern, 5)
GDSP_C6_LAUNCH(extern, 6)
GDSP_C6_LAUNCH(extern, 9)
GDSP_C6_LAUNCH(extern, 10)
GDSP_C6_LAUNCH(extern, 13)
GDSP_C6_LAUNCH(extern, 14)
GDSP_C6_LAUNCH(extern, 15)
GDSP_C6_LAUNCH(extern, 16)
GDSP_C6_LAUNCH(extern, 18)
GDSP_C6_LAUNCH(extern, 20)
GDSP_C6_LAUNCH(extern, 21)
GDSP_C6_LAUNCH(extern, 25)
GDSP_C4_LAUNCH(extern, 6, 6)
GDSP_C4_LAUNCH(extern, 8, 5)
GDSP_C4_LAUNCH(extern, 8, 6)

// The pass-B radices, ascending: a length takes the first M = 256 RB >=
// 2n - 1 (n >= 129) unless the power of 2 is smaller (0 = none: the
// power-of-2 chirp-z). Measured against the round-5 choice (M = 3072 / 6144 /
// the power of 2) on the first and last prime of each RB's range, forced
// chirp-z plans, 2^27 samples (profiles/r06/chirpz_rb_sweep.jsonl): RB 3-6,
// 9, 10, 13-16, 18, 20, 21, 25 are 1.04-1.25x faster; not kept: 2 (0.96-0.98x),
// 7 and 8 (0.94-0.96x; 0.89-0.98x at two waves per SIMD), 11 (0.99x), 22
// (0.77x; 0.97x at 128 VGPRs), 26-32 (0.78-0.82x: 144-168 VGPRs hold their
// 7-8-wave workgroups to one per CU; 26 at 128 VGPRs spills 40 and runs
// 0.90x), where M = 6144 or the power of 2 stays.
static const int kC6RB[] = {3, 4, 5, 6, 9, 10, 12, 13, 14, 15, 16, 18, 20, 21, 24, 25};
// four-pass entries (chirpz4_kernel): M = 256 R1 R2, ascending. Measured
// against the previous choice (the power of 2, or the smooth-L chirp-z where
// it won its race) on the first and last prime of each range, forced chirp-z
// plans, 2^27 samples (profiles/r06/chirpz_rb_sweep.jsonl, session r06s4):
// kept (6, 6) 1.09-1.10x (1.01x where the smooth-L chirp-z won its race on
// the same M), (8, 5) 1.13-1.14x, (8, 6) 1.07-1.12x over 5121 ... 6144
// (session r06t); not kept (9, 3), (7, 4), (6, 5), (8, 4) (0.63-0.96x
// against the M = 8192 kernel), (7, 6) 1.01-1.02x, (9, 5) 0.96x, (9, 6)
// 0.88x, (8, 7) 0.97x, (10, 6) 0.86x, (9, 7) 0.89x, (8, 8) 0.97-1.02x
// against the M = 16384 kernel: one 9-16-wave workgroup per CU and a third
// exchange cost about what the smaller M saves.
struct C4Entry {
  int r1, r2;
};
static const C4Entry kC4[] = {{6, 6}, {8, 5}, {8, 6}};

int chirpz6k_m(int64_t n) {
  if (n < 129) return 0;
  int64_t p2 = 1;
  while (p2 < 2 * n - 1) p2 <<= 1;
  int64_t m = 0;
  for (int rb : kC6RB)
    if (256 * (int64_t)rb >= 2 * n - 1) {
      m = 256 * rb;
      break;
    }
  for (const C4Entry &e : kC4) {
    const int64_t m4 = 256 * (int64_t)e.r1 * e.r2;
    if (m4 >= 2 * n - 1) {
      if (!m || m4 < m) m = m4;
      break;
    }
  }
  return m && m <= p2 ? (int)m : 0;
}

int chirpz6k_radices(int64_t m, int *rad) {
  for (int rb : kC6RB)
    if (256 * (int64_t)rb == m) {
      rad[0] = 16, rad[1] = rb, rad[2] = 16;
      return 3;
    }
  for (const C4Entry &e : kC4)
    if (256 * (int64_t)e.r1 * e.r2 == m) {
      rad[0] = 16, rad[1] = e.r1, rad[2] = e.r2, rad[3] = 16;
      return 4;
    }
  return 0;
}

hipError_t launch_chirpz6k(int64_t m, bool inv, int load, const void *in, cd *out, int64_t n,
                           int64_t batch, const cd *tw, const cd *chirp, const cd *bhat,
                           double scale, hipStream_t s) {
  if (chirpz6k_m(n) != m || batch < 0 || batch > 0x7fffffff || (inv && load == LOAD_REAL))
    return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  int rad[4];
  if (chirpz6k_radices(m, rad) == 4) {
    switch (rad[1] * 16 + rad[2]) {
#define C4_CASE(R1, R2) \
  case R1 * 16 + R2: return launch_c4<R1, R2>(inv, load, in, out, n, batch, tw, chirp, bhat, scale, s);
      C4_CASE(6, 6) C4_CASE(8, 5) C4_CASE(8, 6)
#undef C4_CASE
      default: return hipErrorInvalidValue;
    }
  }
  switch (m / 256) {
#define C6_CASE(RB) \
  case RB: return launch_c6<RB>(inv, load, in, out, n, batch, tw, chirp, bhat, scale, s);
    C6_CASE(3) C6_CASE(4) C6_CASE(5) C6_CASE(6)
    C6_CASE(9) C6_CASE(10) C6_CASE(12) C6_CASE(13) C6_CASE(14) C6_CASE(15) C6_CASE(16)
    C6_CASE(18) C6_CASE(20) C6_CASE(21) C6_CASE(24) C6_CASE(25)
#undef C6_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace gdsp
