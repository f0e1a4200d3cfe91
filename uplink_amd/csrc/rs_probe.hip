// On-box HBM ceilings for the bench line: plain streaming
// kernels, no GF arithmetic, in the access mixes of the erasure kernels, in
// the best shapes tools/exp/bw_probe.hip found on this part (DESIGN.md §4 HBM
// table): a one-shot grid, every wave moving R 1-KiB blocks in and W out
// (16 B per lane per block), non-temporal:
//   copy             R = 1, W = 1    (the rebuild's 1 : 1)
//   encode mix       R = 4, W = 11   (1 : 2.75; the full encode moves 1 : 80/29 = 2.76)
//   parity-only mix  R = 4, W = 7    (1 : 1.75; the parity-only encode 1 : 51/29 = 1.76)
// The written words depend on every word read (XOR), so nothing is dead code.
#include <hip/hip_runtime.h>

#include "../../include/uplink_ec.h"

namespace uplink_ec {
namespace {

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <int R, int W>
__global__ __launch_bounds__(256) void rs_bw_probe(const v4 *in, v4 *out, int64_t nwaves) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave >= nwaves) return;
    v4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; r++) acc ^= __builtin_nontemporal_load(in + (wave * R + r) * 64 + lane);
#pragma unroll
    for (int w = 0; w < W; w++) __builtin_nontemporal_store(acc ^ (uint32_t)w, out + (wave * W + w) * 64 + lane);
}

template <int R, int W>
hipError_t launch(const uint8_t *src, uint8_t *dst, size_t read_bytes, hipStream_t s) {
    const int64_t nwaves = (int64_t)(read_bytes / (1024 * R));
    if (nwaves <= 0) return hipErrorInvalidValue;
    const int64_t blocks = (nwaves + 3) / 4;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL((rs_bw_probe<R, W>), dim3((unsigned)blocks), dim3(256), 0, s, (const v4 *)src, (v4 *)dst,
                       nwaves);
    return hipGetLastError();
}

}  // namespace
}  // namespace uplink_ec

using namespace uplink_ec;

extern "C" int ec_bw_probe(int shape, const uint8_t *src, size_t read_bytes, uint8_t *dst, size_t *moved,
                           ec_stream stream) {
    if (!src || !dst || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return EC_ERR_INVALID_ARG;
    hipStream_t s = (hipStream_t)stream;
    hipError_t e;
    size_t r = 0, w = 0;
    switch (shape) {
    case EC_PROBE_COPY: e = launch<1, 1>(src, dst, read_bytes, s), r = read_bytes / 1024 * 1024, w = r; break;
    case EC_PROBE_ENCODE_MIX: e = launch<4, 11>(src, dst, read_bytes, s), r = read_bytes / 4096 * 4096, w = r / 4 * 11; break;
    case EC_PROBE_PARITY_MIX: e = launch<4, 7>(src, dst, read_bytes, s), r = read_bytes / 4096 * 4096, w = r / 4 * 7; break;
    default: return EC_ERR_INVALID_ARG;
    }
    if (e != hipSuccess) return e == hipErrorInvalidValue ? EC_ERR_INVALID_ARG : EC_ERR_DEVICE;
    if (moved) *moved = r + w;
    return EC_OK;
}
