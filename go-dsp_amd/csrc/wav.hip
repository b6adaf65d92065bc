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
// Byte loads per lane stay coalesced (one 64..256-B segment per wave
// instruction) and work at any data-chunk alignment.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.hpp"

namespace gdsp {

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

hipError_t launch_wav_decode(const void *in, int64_t count, int audio_format, int bits,
                             void *out, bool f64, hipStream_t s) {
  int64_t nb = (count + 255) / 256;
  if (nb > 16384) nb = 16384;
  if (nb < 1) nb = 1;
  const unsigned char *b = (const unsigned char *)in;
  const dim3 g((unsigned)nb), blk(256);
#define GDSP_WAV(F)                                                                          \
  do {                                                                                       \
    if (f64)                                                                                 \
      hipLaunchKernelGGL((wav_decode_kernel<F, true>), g, blk, 0, s, b, count, out);        \
    else                                                                                     \
      hipLaunchKernelGGL((wav_decode_kernel<F, false>), g, blk, 0, s, b, count, out);       \
  } while (0)
  if (audio_format == 1 && bits == 8)
    GDSP_WAV(8);
  else if (audio_format == 1 && bits == 16)
    GDSP_WAV(16);
  else if (audio_format == 3)
    GDSP_WAV(32);
  else
    return hipErrorInvalidValue;
#undef GDSP_WAV
  return hipGetLastError();
}

}  // namespace gdsp
