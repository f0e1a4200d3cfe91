// Launchers for the error-detecting decode kernels (rs_correct.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace uplink_ec {
hipError_t launch_flag_columns(const uint8_t *shares, int64_t stride, const uint8_t *expected, int64_t estride, int k,
                               int ns, int64_t len, uint8_t *flags, hipStream_t s);
// changed (optional): [ncols][ns] bytes, 1 where BW rewrote share i of column ci
hipError_t launch_berlekamp_welch(uint8_t *shares, int64_t stride, int64_t len, const int *nums, int k, int n, int ns,
                                  const int64_t *cols, int ncols, int *status, hipStream_t s,
                                  uint8_t *changed = nullptr);
hipError_t launch_flag_rows(const uint8_t *shares, int64_t stride, const int *rows, int nrows, const uint8_t *expected,
                            int64_t estride, int64_t len, uint8_t *flags, hipStream_t s);
hipError_t launch_put_rows(uint8_t *shares, int64_t stride, const int *rows, int nrows, const uint8_t *expected,
                           int64_t estride, int64_t len, const uint8_t *skip, hipStream_t s);
}  // namespace uplink_ec
