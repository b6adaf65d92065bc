//go:build gdspgpu

// fft_gpu.go — the GPU build of package fft (github.com/mjibson/go-dsp/fft):
// the exported functions of fft/fft.go with their bodies on libgdspfft
// (include/gdsp_fft.h, hand-written gfx950 kernels), same signatures, same
// results within 1e-9 normwise, same panics.
//
// Install (go/README.md): copy this file into the reference's fft/ directory
// and put `//go:build !gdspgpu` on top of fft/fft.go, fft/radix2.go and
// fft/bluestein.go. No reference FFT code is compiled into the GPU build:
// every call, at every n, runs on the library (EnsureRadix2Factors and the
// reverseBits helper fft_test.go uses are defined here).
// Build with `go build -tags gdspgpu` and the library on the cgo paths:
//
//	CGO_CFLAGS="-I<repo>/include"
//	CGO_LDFLAGS="-L<repo>/go-dsp_amd/lib -Wl,-rpath,<repo>/go-dsp_amd/lib"
//
// Each function below is replayed call for call, in C++, by
// tests/cpp/shim_replay.cpp (tests/test_cpp_mirror.py, on the GPU): the same
// C-ABI calls with the same arguments, the same flattening of [][]complex128,
// the same status -> panic mapping and the same small-n policy.
package fft

/*
#cgo LDFLAGS: -lgdspfft
#include "gdsp_fft.h"
*/
import "C"

import (
	"unsafe"

	"github.com/mjibson/go-dsp/dsputils"
)

// check maps a libgdspfft status to the reference's panic: the misuse
// statuses carry the reference's own messages (fft.go:57, :126, :133,
// spectral.go:31); GDSP_ERR_NO_DEVICE / GDSP_ERR_HIP have no reference
// equivalent and panic with the library's detail (there is no silent CPU
// fallback).
func check(st C.int) {
	switch st {
	case C.GDSP_OK:
		return
	case C.GDSP_ERR_UNEQUAL, C.GDSP_ERR_EMPTY, C.GDSP_ERR_RAGGED, C.GDSP_ERR_DIVIDE_BY_ZERO:
		panic(C.GoString(C.gdsp_status_string(st)))
	}
	panic("gdspfft: " + C.GoString(C.gdsp_status_string(st)) + ": " + C.GoString(C.gdsp_last_error()))
}

// cplx / real64 give the C ABI a slice's first element (nil when empty). A
// complex128 is the library's (re, im) float64 pair: no conversion.
func cplx(x []complex128) *C.double {
	if len(x) == 0 {
		return nil
	}
	return (*C.double)(unsafe.Pointer(&x[0]))
}

func real64(x []float64) *C.double {
	if len(x) == 0 {
		return nil
	}
	return (*C.double)(unsafe.Pointer(&x[0]))
}

// FFT replaces fft/fft.go:72-87: radix2FFT (radix2.go:80-154) for powers of
// 2, bluesteinFFT (bluestein.go:68-94) otherwise. x is not modified; the
// result is a fresh slice.
func FFT(x []complex128) []complex128 {
	r := make([]complex128, len(x))
	check(C.gdsp_fft(cplx(x), cplx(r), C.int64_t(len(x))))
	return r
}

// IFFT replaces fft/fft.go:35-52. An empty x panics with the runtime's index
// error, as the reference's x[0] does.
func IFFT(x []complex128) []complex128 {
	_ = x[0]
	n := len(x)
	r := make([]complex128, n)
	check(C.gdsp_ifft(cplx(x), cplx(r), C.int64_t(n)))
	return r
}

// FFTReal replaces fft/fft.go:25-27: the float64 samples go over as they are
// (the kernel reads real rows; no ToComplex copy).
func FFTReal(x []float64) []complex128 {
	r := make([]complex128, len(x))
	check(C.gdsp_fft_real(real64(x), cplx(r), C.int64_t(len(x))))
	return r
}

// IFFTReal replaces fft/fft.go:30-32 (panics on an empty x like IFFT).
func IFFTReal(x []float64) []complex128 {
	_ = x[0]
	r := make([]complex128, len(x))
	check(C.gdsp_ifft_real(real64(x), cplx(r), C.int64_t(len(x))))
	return r
}

// Convolve replaces fft/fft.go:55-69: IFFT(FFT(x) * FFT(y)).
func Convolve(x, y []complex128) []complex128 {
	if len(x) != len(y) {
		panic("arrays not of equal size")
	}
	r := make([]complex128, len(x))
	check(C.gdsp_convolve(cplx(x), cplx(y), cplx(r), C.int64_t(len(x))))
	return r
}

// rows2D checks and flattens a [][]T: the reference's panics for an empty
// or ragged input (fft.go:125-134), then one contiguous row-major buffer
// (a [][]T holds Go pointers, which cgo cannot pass).
func rows2D(nrows int, rowLen func(int) int) (rows, cols int) {
	if nrows == 0 {
		panic("empty input array")
	}
	cols = rowLen(0)
	for i := 1; i < nrows; i++ {
		if rowLen(i) != cols {
			panic("ragged input array")
		}
	}
	return nrows, cols
}

// split2D slices the flat result into rows that share its backing array
// (each with its own capacity, so an append to one row cannot run into the
// next).
func split2D(flat []complex128, rows, cols int) [][]complex128 {
	r := make([][]complex128, rows)
	for i := range r {
		r[i] = flat[i*cols : (i+1)*cols : (i+1)*cols]
	}
	return r
}

func fft2(x [][]complex128, inverse C.int) [][]complex128 {
	rows, cols := rows2D(len(x), func(i int) int { return len(x[i]) })
	flat := make([]complex128, rows*cols)
	for i, row := range x {
		copy(flat[i*cols:], row)
	}
	out := make([]complex128, rows*cols)
	check(C.gdsp_fft2(cplx(flat), cplx(out), C.int64_t(rows), C.int64_t(cols), inverse))
	return split2D(out, rows, cols)
}

func fft2Real(x [][]float64, inverse C.int) [][]complex128 {
	rows, cols := rows2D(len(x), func(i int) int { return len(x[i]) })
	flat := make([]float64, rows*cols)
	for i, row := range x {
		copy(flat[i*cols:], row)
	}
	out := make([]complex128, rows*cols)
	check(C.gdsp_fft2_real(real64(flat), cplx(out), C.int64_t(rows), C.int64_t(cols), inverse))
	return split2D(out, rows, cols)
}

// FFT2 / IFFT2 replace fft/fft.go:109 / :119 (computeFFT2, fft.go:123-154).
func FFT2(x [][]complex128) [][]complex128  { return fft2(x, 0) }
func IFFT2(x [][]complex128) [][]complex128 { return fft2(x, 1) }

// FFT2Real / IFFT2Real replace fft/fft.go:104 / :114: the real rows go over as
// float64 (half the bytes of ToComplex2's complex rows).
func FFT2Real(x [][]float64) [][]complex128  { return fft2Real(x, 0) }
func IFFT2Real(x [][]float64) [][]complex128 { return fft2Real(x, 1) }

func fftn(m *dsputils.Matrix, inverse C.int) *dsputils.Matrix {
	dims := m.Dimensions()
	cdims := make([]C.int64_t, len(dims))
	n := 1
	for i, d := range dims {
		cdims[i] = C.int64_t(d)
		n *= d
	}
	// flatten in row-major order through the public accessor (Matrix keeps
	// its list private, dsputils/matrix.go:21-24)
	flat := make([]complex128, n)
	idx := make([]int, len(dims))
	for i := 0; i < n; i++ {
		flat[i] = m.Value(idx)
		for d := len(dims) - 1; d >= 0; d-- {
			if idx[d]++; idx[d] < dims[d] {
				break
			}
			idx[d] = 0
		}
	}
	out := make([]complex128, n)
	check(C.gdsp_fftn(cplx(flat), cplx(out), &cdims[0], C.int(len(dims)), inverse))
	return dsputils.MakeMatrix(out, dims)
}

// FFTN / IFFTN replace fft/fft.go:157 / :162 (computeFFTN, fft.go:166-192).
func FFTN(m *dsputils.Matrix) *dsputils.Matrix  { return fftn(m, 0) }
func IFFTN(m *dsputils.Matrix) *dsputils.Matrix { return fftn(m, 1) }

// SetWorkerPoolSize replaces fft/fft.go:95-101. The library records it
// (gdsp_worker_pool_size); the GPU's parallelism does not depend on it.
func SetWorkerPoolSize(n int) {
	if n < 0 {
		n = 0
	}
	C.gdsp_set_worker_pool_size(C.int(n))
}

// EnsureRadix2Factors replaces fft/radix2.go:35-37: the reference builds its
// host twiddle table for input_len ahead of the first call; this builds the
// device plan (twiddle, chirp or Rader tables) for it.
func EnsureRadix2Factors(input_len int) {
	EnsurePlan(input_len)
}

// EnsurePlan builds the GPU plan for input_len ahead of the first call.
func EnsurePlan(input_len int) {
	check(C.gdsp_ensure_plan(C.int64_t(input_len)))
}

// reverseBits returns the first s bits of v in reverse order, the helper
// fft_test.go:242-247 tests (radix2.go:182-199 in the pure-Go build). The
// Stockham kernels need no bit reversal; it is kept so the reference's own
// test file compiles under the gdspgpu tag.
func reverseBits(v, s uint) uint {
	var r uint
	for i := uint(0); i < s; i++ {
		r = r<<1 | (v>>i)&1
	}
	return r
}

// ---- additive entry points (no reference equivalent) -----------------------

// FFTBatch transforms len(x)/n rows of n complex128 held in one flat slice
// in one call (one launch), the batched seam the reference lacks (SURVEY.md
// §8b). inverse selects IFFT semantics (1/n).
func FFTBatch(x []complex128, n int, inverse bool) []complex128 {
	if n <= 0 || len(x)%n != 0 {
		panic("arrays not of equal size")
	}
	r := make([]complex128, len(x))
	check(C.gdsp_fft_batch(cplx(x), cplx(r), C.int64_t(n), C.int64_t(len(x)/n), cbool(inverse)))
	return r
}

// FFTRealBatch: FFTReal of len(x)/n float64 rows of n in one call.
func FFTRealBatch(x []float64, n int) []complex128 {
	if n <= 0 || len(x)%n != 0 {
		panic("arrays not of equal size")
	}
	r := make([]complex128, len(x))
	check(C.gdsp_fft_real_batch(real64(x), cplx(r), C.int64_t(n), C.int64_t(len(x)/n)))
	return r
}

// SetDevices selects the GPUs that large FFTBatch / Pwelch calls split over
// (nil: every call stays on the calling thread's current device).
func SetDevices(ids []int) {
	var p *C.int
	c := make([]C.int, len(ids))
	for i, d := range ids {
		c[i] = C.int(d)
	}
	if len(c) > 0 {
		p = &c[0]
	}
	check(C.gdsp_set_devices(p, C.int(len(c))))
}

// FFTBatchMulti: FFTBatch always split into contiguous row shards over the
// device set, one host worker per device, no collective.
func FFTBatchMulti(x []complex128, n int, inverse bool) []complex128 {
	if n <= 0 || len(x)%n != 0 {
		panic("arrays not of equal size")
	}
	r := make([]complex128, len(x))
	check(C.gdsp_fft_batch_multi(cplx(x), cplx(r), C.int64_t(n), C.int64_t(len(x)/n),
		cbool(inverse), nil, 0))
	return r
}

func cbool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}
