//go:build gdspgpu

// pwelch_gpu.go — the GPU build of spectral.Pwelch (github.com/mjibson/go-dsp/
// spectral): the segment loop of spectral/pwelch.go:104-122 (window, FFTReal,
// |X|^2 accumulation over every segment) runs as one fused kernel per device
// (gdsp_pwelch, include/gdsp_fft.h); Segment (spectral.go) stays pure Go.
//
// Install (go/README.md): copy this file into the reference's spectral/
// directory and put `//go:build !gdspgpu` on top of spectral/pwelch.go (this
// file declares PwelchOptions with the reference's fields, pwelch.go:28-65).
// Replayed call for call by tests/cpp/shim_replay.cpp.
package spectral

/*
#cgo LDFLAGS: -lgdspfft
#include "gdsp_fft.h"
*/
import "C"

import (
	"unsafe"

	"github.com/mjibson/go-dsp/window"
)

// PwelchOptions is spectral/pwelch.go:28-65's options struct, field for
// field (see the reference for each field's documentation).
type PwelchOptions struct {
	NFFT      int                  // points per segment; default 256
	Window    func(int) []float64  // default window.Hann
	Pad       int                  // FFT length per segment; default NFFT
	Noverlap  int                  // points of overlap between segments; default 0
	Scale_off bool                 // true: no division by Fs
}

// Pwelch replaces spectral/pwelch.go:74-145. A nil o dereferences (panics)
// as in the reference. The Window option is a Go function that C cannot call,
// so the shim evaluates the two tables the reference uses and passes them:
// wf(max(NFFT, Pad)), applied to each zero-padded segment (pwelch.go:108-109 ->
// window.go:25-29: ZeroPadF leaves a segment longer than Pad as it is), and
// wf(NFFT) for the normalisation (pwelch.go:124). Large calls split over the
// device set inside the library (fft.SetDevices / GDSP_DEVICES).
func Pwelch(x []float64, Fs float64, o *PwelchOptions) (Pxx, freqs []float64) {
	if len(x) == 0 {
		return []float64{}, []float64{}
	}
	nfft, pad, wf := o.NFFT, o.Pad, o.Window
	if nfft == 0 {
		nfft = 256
	}
	if wf == nil {
		wf = window.Hann
	}
	if pad == 0 {
		pad = nfft
	}
	flen := nfft
	if pad > flen {
		flen = pad
	}
	wseg, wnfft := wf(flen), wf(nfft)
	lp := pad/2 + 1
	Pxx, freqs = make([]float64, lp), make([]float64, lp)
	scaleOff := C.int(0)
	if o.Scale_off {
		scaleOff = 1
	}
	var got C.int64_t
	st := C.gdsp_pwelch((*C.double)(unsafe.Pointer(&x[0])), C.int64_t(len(x)), C.double(Fs),
		C.int64_t(nfft), C.int64_t(pad), C.int64_t(o.Noverlap),
		(*C.double)(unsafe.Pointer(&wseg[0])), (*C.double)(unsafe.Pointer(&wnfft[0])),
		scaleOff, (*C.double)(unsafe.Pointer(&Pxx[0])), (*C.double)(unsafe.Pointer(&freqs[0])),
		&got)
	switch st {
	case C.GDSP_OK:
	case C.GDSP_ERR_DIVIDE_BY_ZERO:
		// Noverlap == NFFT: Segment's integer divide (spectral.go:31)
		panic(C.GoString(C.gdsp_status_string(st)))
	case C.GDSP_ERR_INVALID:
		// Noverlap > NFFT: Segment's negative count ("makeslice: len out of range")
		panic(C.GoString(C.gdsp_last_error()))
	default:
		panic("gdspfft: " + C.GoString(C.gdsp_status_string(st)) + ": " +
			C.GoString(C.gdsp_last_error()))
	}
	return Pxx[:got], freqs[:got]
}
