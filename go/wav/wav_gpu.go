//go:build gdspgpu

// wav_gpu.go — the GPU build of (*Wav).ReadFloats (github.com/mjibson/go-dsp/
// wav, wav/wav.go:135-161): the sample conversion of a data chunk runs on
// the GPU (gdsp_wav_read_floats) with the reference's float32 formulas. The
// header parsing (New) and ReadSamples stay pure Go.
//
// Install (go/README.md): move wav.go's ReadFloats (wav.go:135-161) into a
// file tagged `//go:build !gdspgpu` and copy this file beside it.
// Replayed call for call by tests/cpp/shim_replay.cpp.
package wav

/*
#cgo LDFLAGS: -lgdspfft
#include "gdsp_fft.h"
*/
import "C"

import (
	"fmt"
	"io"
	"unsafe"
)

// ReadFloats is like ReadSamples, but it converts any underlying data to a
// float32 (wav.go:135-161): PCM8 v/255, PCM16 (v + 32768)/65535, float32 as
// stored. The n raw samples are read here, converted on the GPU.
func (w *Wav) ReadFloats(n int) ([]float32, error) {
	var size int
	switch w.AudioFormat {
	case wavFormatPCM:
		switch w.BitsPerSample {
		case 8, 16:
			size = int(w.BitsPerSample) / 8
		default:
			return nil, fmt.Errorf("wav: unknown bits per sample: %v", w.BitsPerSample)
		}
	case wavFormatIEEEFloat:
		size = 4
	default:
		return nil, fmt.Errorf("wav: unknown audio format")
	}
	raw := make([]byte, n*size)
	if _, err := io.ReadFull(w.r, raw); err != nil {
		return nil, err // io.EOF / io.ErrUnexpectedEOF, as binary.Read returns them
	}
	f := make([]float32, n)
	if n == 0 {
		return f, nil
	}
	st := C.gdsp_wav_read_floats(unsafe.Pointer(&raw[0]), C.int64_t(n), C.int(w.AudioFormat),
		C.int(w.BitsPerSample), unsafe.Pointer(&f[0]), 0)
	if st != C.GDSP_OK {
		panic("gdspfft: " + C.GoString(C.gdsp_status_string(st)) + ": " +
			C.GoString(C.gdsp_last_error()))
	}
	return f, nil
}
