// fft_wave.hip — wave-resident FFT-2048 and the chirp-z kernel built on it.
//
// One 64-lane wavefront holds a 2048-point transform, 32 complex128 per lane
// (element lane + 64 k in register k), and computes it in three Stockham
// passes (radix 32, 32, 2) whose exchanges never leave the wave:
//   - after pass 1, a 5-bit register <-> lane transpose through the wave's own
//     LDS region (LDS instructions of one wave execute in order, so the write
//     -> read hand-off needs no workgroup barrier);
//   - after pass 2, a swap of lane bit 5 with register bit 0: one
//     v_permlane32_swap per dword pair, no LDS at all (the wavefront shuffle of
//     the last, radix-2 stage).
// Nothing in the transform synchronises the workgroup, so the waves of a CU
// drift apart and one wave's exchange overlaps its neighbours' FP64 work
// (the block-wide kernels of fft_kernels.hip stop every wave of a workgroup
// at each exchange).
//
// bluestein_wave_kernel<Q>: chirp-z (fft/bluestein.go:68-94 with Convolve,
// fft/fft.go:55-69) for M = 2048 * Q (Q = 1, 2, 4: the reference's
// M = NextPowerOf2(2n-1); Q = 3: M = 6144, the same convolution on a smaller
// M >= 2n - 1). Q waves share one transform:
//   1. a = x conj(w) (the chirp premultiply), each element once, into LDS;
//      then the first radix-Q step of FFT_M (decimation in frequency): wave q
//      reads b_q[m] = (a[m] + W_Q^q a[m + 2048]) W_M^(q m), so A[Q k + q] =
//      FFT_2048(b_q)[k] (a is zero beyond n <= 4096);
//   2. C = A * bhat (bhat permuted per wave), IFFT_2048 per wave as
//      conj(FFT(conj C)): G_q;
//   3. last radix-Q step (decimation in time) across the Q waves:
//      r[n' + 2048 p] = sum_q W_Q^(-p q) (W_M^(-n' q) G_q[n']), through LDS
//      as real and imaginary halves (three workgroup barriers per transform);
//      only p with n' + 2048 p < n is computed;
//   4. X = r * conj(w) (the chirp), first n.
#include "dev.hpp"

namespace gdsp {

namespace {

constexpr int kWaveN = 2048;
#ifdef GDSP_WV_NOSCHED
constexpr bool kWvSched = false;
#else
constexpr bool kWvSched = true;
#endif
// doubles of one wave's exchange region: linear slots i + i/32 (i < 2048)
constexpr int kWaveLds = kWaveN + kWaveN / 32;

// compiler-only ordering of the wave's LDS accesses (the hardware executes a
// wave's LDS instructions in order)
__device__ __forceinline__ void wave_lds_order() {
#ifndef GDSP_WV_NOFENCE
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#endif
  __builtin_amdgcn_wave_barrier();
}

// v_permlane32_swap on a double pair: lanes 32-63 of a <-> lanes 0-31 of b
__device__ __forceinline__ void swap32(double &a, double &b) {
  const unsigned long long ua = __builtin_bit_cast(unsigned long long, a);
  const unsigned long long ub = __builtin_bit_cast(unsigned long long, b);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi =
      __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, (unsigned long long)lo[0] | ((unsigned long long)hi[0] << 32));
  b = __builtin_bit_cast(double, (unsigned long long)lo[1] | ((unsigned long long)hi[1] << 32));
}

// Forward FFT-2048 of the wave's registers: v[k] = element lane + 64 k, in and
// out (natural order). t2048[k] = exp(-2 pi i k / 2048). lw: this wave's LDS
// region (kWaveLds doubles).
#ifdef GDSP_WV_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
void wave_fft2048(cd (&v)[32], int lane, const cd *__restrict__ t2048, double *lw) {
#ifndef GDSP_WV_NOINLINE
  lane = opaque_int(lane);
  t2048 = opaque_ptr(t2048);
#endif
  // pass 1: radix 32, butterfly j = lane over elements lane + 64 r; output r
  // is element 32 lane + r
  pass_compute<kWaveN, 32, 64, 32, 1>(v, lane, t2048);
  // exchange 1 (wave-local LDS, real then imaginary half): slot(i) = i + i/32,
  // so the writes are 33 lane + r and the reads lane + lane/32 + 66 k, both a
  // per-lane base plus constants; conflict-free for ds_write_b64 (16-lane
  // groups: (lane + r) mod 16) and ds_read_b64 (32-lane groups: lane + 2k)
  double *wr = lw + 33 * lane;
  const double *rd = lw + lane + (lane >> 5);
  wave_lds_order();
#pragma unroll
  for (int r = 0; r < 32; ++r) wr[r] = v[r].x;
  wave_lds_order();
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k].x = rd[66 * k];
  wave_lds_order();
#pragma unroll
  for (int r = 0; r < 32; ++r) wr[r] = v[r].y;
  wave_lds_order();
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k].y = rd[66 * k];
  wave_lds_order();
  // pass 2: radix 32 with twiddles W_1024^((lane % 32) r); output r of
  // butterfly lane is element (lane / 32) 1024 + lane % 32 + 32 r
  pass_compute<kWaveN, 32, 64, 32, 32>(v, lane, t2048);
  // exchange 2: element (lane 32h + a, reg 2s + b) belongs at (lane a + 32b,
  // reg 16h + s): swap lane bit 5 with register bit 0 (v_permlane32_swap),
  // then rename registers
  cd u[32];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    cd a = v[2 * s], b = v[2 * s + 1];
    swap32(a.x, b.x);
    swap32(a.y, b.y);
    u[s] = a;
    u[16 + s] = b;
  }
  // pass 3: radix 2, butterfly j = lane + 64 b over elements j, j + 1024
  // (registers b, b + 16), twiddle W_2048^j = W_2048^lane W_32^b
  const cd base = t2048[lane];
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    const cd t = rot32(cmul(u[16 + b], base), b);
    v[b] = u[b] + t;
    v[16 + b] = u[b] - t;
  }
}

// W_Q^(-p q) = exp(+2 pi i p q / Q), real and imaginary part
template <int Q>
__device__ __forceinline__ constexpr double wq_re(int pq) {
  return Q == 1 ? 1.0
       : Q == 2 ? ((pq & 1) ? -1.0 : 1.0)
       : Q == 4 ? ((pq & 3) == 0 ? 1.0 : (pq & 3) == 2 ? -1.0 : 0.0)
                : ((pq % 3) == 0 ? 1.0 : -0.5);
}
template <int Q>
__device__ __forceinline__ constexpr double wq_im(int pq) {
  return Q == 1 || Q == 2 ? 0.0
       : Q == 4 ? ((pq & 3) == 1 ? 1.0 : (pq & 3) == 3 ? -1.0 : 0.0)
                : ((pq % 3) == 0 ? 0.0 : (pq % 3) == 1 ? 0.86602540378443864676
                                                       : -0.86602540378443864676);
}

}  // namespace

template <int Q>
struct WaveGeo {
  static constexpr int TPW = Q == 3 ? 1 : 4 / Q;  // transforms per workgroup
  static constexpr int WAVES = Q * TPW;
  static constexpr int WG = 64 * WAVES;
  // nonzero input / needed output range n <= 1024 Q: registers k < KMAX
  static constexpr int KMAX = Q == 1 ? 16 : 32;
  static constexpr int P = Q >= 3 ? 2 : 1;  // output blocks of 2048 (n <= 4096)
  static constexpr int CH = (32 + Q - 1) / Q;  // 64-element chunks a wave combines
};

template <int Q, bool INV>
__global__ __launch_bounds__(WaveGeo<Q>::WG, 2) void bluestein_wave_kernel(
    const cd *__restrict__ in, cd *__restrict__ out, int64_t n, int64_t batch,
    const cd *__restrict__ t2048, const cd *__restrict__ wbase, const cd *__restrict__ bhatw,
    const cd *__restrict__ chirp, double scale) {
  using G = WaveGeo<Q>;
  constexpr int NA = 1024 * Q;  // n <= NA: the input's (zero-padded) extent
  __shared__ double lds[G::WAVES * kWaveLds];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int slot = wave / Q, q = wave - slot * Q;
  const int64_t g = xcd_remap(blockIdx.x, gridDim.x) * G::TPW + slot;
  const bool valid = g < batch;
  double *lw = lds + wave * kWaveLds;          // this wave's exchange region
  double *lt = lds + slot * Q * kWaveLds;      // the transform's Q regions
  const cd *src = in + (valid ? g : 0) * n;
  cd v[32];
  if constexpr (Q == 1) {
    // a[m] = x[m] conj(w_m) straight into registers (n <= 1024: k < 16)
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int m = lane + 64 * k;
      v[k] = {0.0, 0.0};
      if (k < 16 && valid && m < n) {
        cd x = src[m];
        if constexpr (INV) x.y = -x.y;
        v[k] = cmul(x, chirp[m]);
      }
    }
  } else {
    // 1. a[i] = x[i] conj(w_i), i < NA (zero beyond n), computed once per
    //    element by the wave owning chunk i / 64 (= q mod Q), into LDS as real
    //    [0, NA) and imaginary [NA, 2 NA) halves of the transform's regions
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = lane + 64 * (q + Q * j);
      cd a = {0.0, 0.0};
      if (valid && i < n) {
        cd x = src[i];
        if constexpr (INV) x.y = -x.y;
        a = cmul(x, chirp[i]);
      }
      lt[i] = a.x;
      lt[NA + i] = a.y;
    }
    __syncthreads();
    // 2. first radix-Q step of FFT_M (decimation in frequency):
    //    b_q[m] = (a[m] + W_Q^q a[m + 2048]) W_M^(q m), m = lane + 64 k
    //    (a[m + 4096] = 0: n <= 4096); W_M^(q m) by recurrence from
    //    wbase[q][lane] = W_M^(q lane) with step wbase[q][64] = W_M^(64 q)
    const cd wq1 = {wq_re<Q>(q), -wq_im<Q>(q)};  // W_Q^q = conj(W_Q^(-q))
    cd w = wbase[q * 65 + lane];
    const cd step = wbase[q * 65 + 64];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (kWvSched && k % 8 == 0) __builtin_amdgcn_sched_barrier(0);
      const int m = lane + 64 * k;
      cd b = {lt[m], lt[NA + m]};
      if constexpr (Q >= 3) {
        if (64 * k + 63 + kWaveN < NA) b = b + cmul(cd{lt[m + kWaveN], lt[NA + m + kWaveN]}, wq1);
      }
      v[k] = b;
      if (q > 0) {
        v[k] = cmul(b, w);
        w = cmul(w, step);
      }
    }
    __syncthreads();  // every wave has read a[] before the regions become exchange buffers
  }
  wave_fft2048(v, lane, t2048, lw);  // A[Q k + q], k = lane + 64 k'
  {
    const cd *bh = opaque_ptr(bhatw) + q * kWaveN + lane;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (kWvSched && k % 16 == 0) __builtin_amdgcn_sched_barrier(0);
      v[k] = conjg(cmul(v[k], bh[64 * k]));  // conj(A bhat / M)
    }
  }
  wave_fft2048(v, lane, t2048, lw);  // conj(G_q)
  if constexpr (Q == 1) {
    if (valid) {
      cd *dst = out + g * n;
      const cd *ch = opaque_ptr(chirp);
      const int lo = opaque_int(lane);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int i = lo + 64 * k;
        if (i < n) {
          cd y = cmul(conjg(v[k]), ch[i]);
          if constexpr (INV) y = {y.x * scale, -y.y * scale};
          st_nt(&dst[i], y);
        }
      }
    }
  } else {
    // H_q = conj(v W_M^(n' q)) = G_q W_M^(-n' q), the same recurrence
    if (q > 0) {
      const cd *wb = opaque_ptr(wbase) + q * 65;
      cd w = wb[lane];
      const cd step = wb[64];
#pragma unroll
      for (int k = 0; k < 32; ++k) {
        v[k] = cmul(v[k], w);
        w = cmul(w, step);
      }
    }
    // 3. last radix-Q step (decimation in time) across the waves:
    //    r_p[n'] = sum_qq W_Q^(-p qq) H_qq[n'] for this wave's chunks n' / 64 =
    //    q + Q c; linear in (Re H, Im H), so the halves cross LDS in turn
    cd r[G::CH][G::P];
#pragma unroll
    for (int c = 0; c < G::CH; ++c)
#pragma unroll
      for (int p = 0; p < G::P; ++p) r[c][p] = {0.0, 0.0};
    const double *lr = lt + lane;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h) __syncthreads();  // every wave has read the real halves
#pragma unroll
      for (int k = 0; k < 32; ++k) lw[lane + 64 * k] = h ? -v[k].y : v[k].x;
      __syncthreads();
#pragma unroll
      for (int c = 0; c < G::CH; ++c) {
        const int chunk = q + Q * c;
        if (kWvSched && c % 4 == 0) __builtin_amdgcn_sched_barrier(0);
        if (chunk < 32) {
#pragma unroll
          for (int qq = 0; qq < Q; ++qq) {
            const double a = lr[qq * kWaveLds + 64 * chunk];
#pragma unroll
            for (int p = 0; p < G::P; ++p) {
              const double wr = wq_re<Q>(p * qq), wi = wq_im<Q>(p * qq);
              if (h == 0) {
                if (wr != 0.0) r[c][p].x += wr * a;
                if (wi != 0.0) r[c][p].y += wi * a;
              } else {
                if (wi != 0.0) r[c][p].x -= wi * a;
                if (wr != 0.0) r[c][p].y += wr * a;
              }
            }
          }
        }
      }
    }
    // 4. X = r conj(w), first n
    if (valid) {
      cd *dst = out + g * n;
#pragma unroll
      for (int c = 0; c < G::CH; ++c) {
        const int chunk = q + Q * c;
#pragma unroll
        for (int p = 0; p < G::P; ++p) {
          const int i = lane + 64 * chunk + kWaveN * p;
          if (chunk < 32 && i < n) {
            cd y = cmul(r[c][p], chirp[i]);
            if constexpr (INV) y = {y.x * scale, -y.y * scale};
            st_nt(&dst[i], y);
          }
        }
      }
    }
  }
}

int bluestein_wave_q(int64_t n, int64_t m) {
  if (n <= 512 || n > 4096 || m % kWaveN) return 0;
  const int64_t q = m / kWaveN;
  return (q >= 1 && q <= 4 && 2 * n - 1 <= m && n <= 1024 * q) ? (int)q : 0;
}

template <int Q, bool INV>
static hipError_t launch_bw_t(const cd *in, cd *out, int64_t n, int64_t batch, const cd *t2048,
                              const cd *wbase, const cd *bhatw, const cd *chirp, double scale,
                              hipStream_t s) {
  using G = WaveGeo<Q>;
  const int64_t nblk = (batch + G::TPW - 1) / G::TPW;
  hipLaunchKernelGGL((bluestein_wave_kernel<Q, INV>), dim3((unsigned)nblk), dim3(G::WG), 0, s, in,
                     out, n, batch, t2048, wbase, bhatw, chirp, scale);
  return hipGetLastError();
}

hipError_t launch_bluestein_wave(int q, bool inv, const cd *in, cd *out, int64_t n, int64_t batch,
                                 const cd *t2048, const cd *wbase, const cd *bhatw, const cd *chirp,
                                 double scale, hipStream_t s) {
  if (batch <= 0) return hipSuccess;
  if (n <= 512 || n > 1024 * (int64_t)q) return hipErrorInvalidValue;
#define GDSP_BW(QQ)                                                                            \
  case QQ:                                                                                     \
    return inv ? launch_bw_t<QQ, true>(in, out, n, batch, t2048, wbase, bhatw, chirp, scale, s) \
               : launch_bw_t<QQ, false>(in, out, n, batch, t2048, wbase, bhatw, chirp, scale, s);
  switch (q) {
    GDSP_BW(1)
    GDSP_BW(2)
    GDSP_BW(3)
    GDSP_BW(4)
    default: return hipErrorInvalidValue;
  }
#undef GDSP_BW
}

}  // namespace gdsp
