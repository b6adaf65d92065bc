// wav.hip — the wav -> Pwelch feeder on the GPU:
// wav.(*Wav).ReadFloats's sample conversion (wav/wav.go:135-161) over the
// little-endian data chunk that ReadSamples reads (wav.go:110-131), written
// as float32 (the reference's type) or as float64 (that float32 widened:
// what a caller hands to spectral.Pwelch), straight into HBM.
//
//   PCM  8-bit : float32(v) / MaxUint8
//   PCM 16-bit : (float32(v) - MinInt16) / (MaxInt16 - MinInt16)
//   IEEE float : the float32 as stored
// Go evaluates both PCM forms in float32 (the untyped constants convert to
// float32); __fdiv_rn keeps the division correctly rounded like Go's.
// The main kernel converts two samples per lane and step (contiguous 16-B
// float64-pair or 8-B float32-pair stores across the wave), nontemporal on
// both sides since the data is streamed once; a byte-load kernel takes the
// odd last sample and any data chunk that is not sample-pair aligned.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.hpp"

namespace gdsp {

template <int FMT>
__device__ __forceinline__ float wav_sample(uint32_t bits) {
  if constexpr (FMT == 8) {
    return __fdiv_rn((float)(bits & 0xff), 255.0f);
  } else if constexpr (FMT == 16) {
    return __fdiv_rn((float)(int16_t)(bits & 0xffff) - (-32768.0f), 65535.0f);
  } else {
    return __uint_as_float(bits);
  }
}

// Two samples per lane and step: the stores are 16 B (float64 pairs) or 8 B
// per lane and contiguous across the wave, the loads 2..8 B per lane.
template <int FMT, bool F64>
__global__ __launch_bounds__(256) void wav_decode_vec_kernel(const unsigned char *__restrict__ in,
                                                             int64_t npairs, void *__restrict__ out) {
  constexpr int B = FMT / 8;  // bytes per sample
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < npairs;
       j += (int64_t)gridDim.x * blockDim.x) {
    uint32_t lo, hi;
    if constexpr (B == 1) {
      const uint32_t w = __builtin_nontemporal_load(reinterpret_cast<const uint16_t *>(in) + j);
      lo = w;
      hi = w >> 8;
    } else if constexpr (B == 2) {
      const uint32_t w = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(in) + j);
      lo = w;
      hi = w >> 16;
    } else {
      const uint32_t *s = reinterpret_cast<const uint32_t *>(in) + 2 * j;
      lo = __builtin_nontemporal_load(s);
      hi = __builtin_nontemporal_load(s + 1);
    }
    const float f0 = wav_sample<FMT>(lo), f1 = wav_sample<FMT>(hi);
    if constexpr (F64) {
      double *d = reinterpret_cast<double *>(out) + 2 * j;
      __builtin_nontemporal_store((double)f0, d);
      __builtin_nontemporal_store((double)f1, d + 1);
    } else {
      float *d = reinterpret_cast<float *>(out) + 2 * j;
      __builtin_nontemporal_store(f0, d);
      __builtin_nontemporal_store(f1, d + 1);
    }
  }
}

template <int FMT, bool F64>
__global__ __launch_bounds__(256) void wav_decode_kernel(const unsigned char *__restrict__ in,
                                                         int64_t count, void *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * blockDim.x) {
    float f;
    if constexpr (FMT == 8) {
      f = __fdiv_rn((float)in[i], 255.0f);
    } else if constexpr (FMT == 16) {
      const int16_t s = (int16_t)((uint16_t)in[2 * i] | ((uint16_t)in[2 * i + 1] << 8));
      f = __fdiv_rn((float)s - (-32768.0f), 65535.0f);
    } else {
      const uint32_t u = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) |
                         ((uint32_t)in[4 * i + 2] << 16) | ((uint32_t)in[4 * i + 3] << 24);
      f = __uint_as_float(u);
    }
    if constexpr (F64)
      reinterpret_cast<double *>(out)[i] = (double)f;
    else
      reinterpret_cast<float *>(out)[i] = f;
  }
}

template <int FMT>
static hipError_t launch_fmt(const unsigned char *b, int64_t count, void *out, bool f64,
                             hipStream_t s) {
  constexpr int B = FMT / 8;
  const size_t osz = f64 ? sizeof(double) : sizeof(float);
  int64_t head = 0;  // samples taken by the sample-pair kernel
  if ((uintptr_t)b % (2 * B) == 0 && (uintptr_t)out % (2 * osz) == 0 && count >= 2) {
    const int64_t npairs = count / 2;
    int64_t nb = (npairs + 255) / 256;
    if (nb > 65536) nb = 65536;
    if (f64)
      hipLaunchKernelGGL((wav_decode_vec_kernel<FMT, true>), dim3((unsigned)nb), dim3(256), 0, s,
                         b, npairs, out);
    else
      hipLaunchKernelGGL((wav_decode_vec_kernel<FMT, false>), dim3((unsigned)nb), dim3(256), 0,
                         s, b, npairs, out);
    head = npairs * 2;
  }
  const int64_t rest = count - head;
  if (rest > 0) {
    int64_t nb = (rest + 255) / 256;
    if (nb > 16384) nb = 16384;
    const unsigned char *bt = b + head * B;
    void *ot = (char *)out + head * osz;
    if (f64)
      hipLaunchKernelGGL((wav_decode_kernel<FMT, true>), dim3((unsigned)nb), dim3(256), 0, s, bt,
                         rest, ot);
    else
      hipLaunchKernelGGL((wav_decode_kernel<FMT, false>), dim3((unsigned)nb), dim3(256), 0, s, bt,
                         rest, ot);
  }
  return hipGetLastError();
}

hipError_t launch_wav_decode(const void *in, int64_t count, int audio_format, int bits,
                             void *out, bool f64, hipStream_t s) {
  const unsigned char *b = (const unsigned char *)in;
  if (count <= 0) return hipSuccess;
  if (audio_format == 1 && bits == 8) return launch_fmt<8>(b, count, out, f64, s);
  if (audio_format == 1 && bits == 16) return launch_fmt<16>(b, count, out, f64, s);
  if (audio_format == 3) return launch_fmt<32>(b, count, out, f64, s);
  return hipErrorInvalidValue;
}

}  // namespace gdsp
