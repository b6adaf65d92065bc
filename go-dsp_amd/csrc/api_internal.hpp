// api_internal.hpp — what the multi-device layer (multi.hip) uses of the
// single-device host path in gdsp_api.hip. Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace gdsp_api {

// Scratch slots the multi-device layer reuses (the Workspace slots of
// gdsp_api.hip, keyed by (device, stream)).
enum ScratchSlot { SCRATCH_SIGNAL = 0, SCRATCH_WINDOW = 1, SCRATCH_ACC = 2 };

// Record msg as the calling thread's gdsp_last_error and return st.
int set_error(int st, const std::string &msg);
// The calling thread's non-blocking stream on device dev (created once).
hipStream_t stream_for(int dev);
// Grow-only device scratch of the current device, ordered by stream s.
int scratch(size_t bytes, hipStream_t s, ScratchSlot slot, void **p);
// Host <-> device through the calling thread's pinned staging (current device).
int h2d(void *dst, const void *src, size_t bytes, hipStream_t s);
int d2h(void *dst, const void *src, size_t bytes, hipStream_t s);  // returns after s drained
// Host-pointer batched transform on the calling thread's current device.
int batch_on_current_device(const void *x, size_t in_elem_bytes, double *out, int64_t n,
                            int64_t batch, bool inv, int load);
// window.Hann table and spectral.Segment count (gdsp_api.hip).
void hann(int64_t L, double *out);
int segments(int64_t lx, int64_t size, int64_t noverlap, int64_t *count);

// Multi-device layer (multi.hip). Whether a host-pointer call of `bytes`
// input over `units` independent units (rows or segments) is split over the
// library's device set; then the split itself.
bool multi_wanted(size_t bytes, int64_t units);
int fft_batch_multi(const void *x, size_t in_elem_bytes, double *out, int64_t n, int64_t batch,
                    bool inv, int load, const int *devices, int ndev);
int pwelch_multi(const double *x, int64_t n, double fs, int64_t nfft, int64_t pad,
                 int64_t noverlap, const double *win_seg, const double *win_nfft, int scale_off,
                 double *pxx, double *freqs, int64_t *lp_out, const int *devices, int ndev);

}  // namespace gdsp_api
