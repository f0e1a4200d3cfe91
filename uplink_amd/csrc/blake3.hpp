// BLAKE3-256 piece hashing on the GPU: launch entry
// points used by the C-ABI.  Host-only header, plain pointers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace uplink_ec {

// npieces byte strings of piece_len bytes each, in sets of pieces_per_set
// (0 = one set).  Byte t of string j lives at
//   base + (j / pieces_per_set)*set_stride + (j % pieces_per_set)*piece_stride
//        + (t / run)*run_stride + t % run
// (run = piece_len for contiguous pieces; run = ess, run_stride = k*ess for
// the data pieces of a stripe-major segment).
struct B3View {
    const uint8_t *base;
    int64_t piece_stride;
    uint64_t piece_len;
    uint64_t run;
    int64_t run_stride;
    uint64_t npieces;
    uint64_t pieces_per_set;
    int64_t set_stride;
    int32_t run_shift;  // set by b3_launch: log2(run) when run is a power of two, else -1
};

// Device bytes of scratch b3_launch needs for this view (0 when every piece
// fits one 256-chunk group).
size_t b3_workspace_bytes(const B3View &v);

// hashes: npieces*32 bytes on the device.  `ws` has b3_workspace_bytes(v).
hipError_t b3_launch(const B3View &v, uint8_t *hashes, void *ws, hipStream_t stream);
// Both views in one launch (equal piece_len): hashes of `first`'s pieces,
// then `second`'s.  ws: b3_workspace_bytes of a view with the summed npieces.
hipError_t b3_launch2(const B3View &first, const B3View &second, uint8_t *hashes, void *ws, hipStream_t stream);
// Streamed form (pieces of >= 2 chunks): the chaining values of BLAKE3 chunks
// [c0, c1) of every piece of both views into cvs [npieces][nchunks][8 words],
// as the bytes of those chunks become available; then b3_launch_fold turns the
// complete cvs into the hashes (cvs is overwritten; ws: b3_fold_ws_bytes).
hipError_t b3_launch_chunk_range(const B3View &first, const B3View &second, uint64_t c0, uint64_t c1, uint32_t *cvs,
                                 hipStream_t stream);
size_t b3_fold_ws_bytes(uint64_t npieces, uint64_t nchunks);
hipError_t b3_launch_fold(uint32_t *cvs, uint64_t npieces, uint64_t nchunks, uint8_t *hashes, void *ws,
                          hipStream_t stream);

}  // namespace uplink_ec
