// BLAKE3-256 piece hashing on the GPU: launch entry
// points used by the C-ABI.  Host-only header, plain pointers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace uplink_ec {

// npieces byte strings of piece_len bytes each.  Byte t of string j lives at
//   base + j*piece_stride + (t / run)*run_stride + t % run
// (run = piece_len for contiguous pieces; run = ess, run_stride = k*ess for
// the data pieces of a stripe-major segment).
struct B3View {
    const uint8_t *base;
    int64_t piece_stride;
    uint64_t piece_len;
    uint64_t run;
    int64_t run_stride;
    uint64_t npieces;
    int32_t run_shift;  // set by b3_launch: log2(run) when run is a power of two, else -1
};

// Device bytes of scratch b3_launch needs for this view (0 when every piece
// fits one 256-chunk group).
size_t b3_workspace_bytes(const B3View &v);

// hashes: npieces*32 bytes on the device.  `ws` has b3_workspace_bytes(v).
hipError_t b3_launch(const B3View &v, uint8_t *hashes, void *ws, hipStream_t stream);

}  // namespace uplink_ec
