// Kernel argument block of the GF(2^8) Reed-Solomon stripe kernels (encode K1,
// rebuild K2 in SURVEY.md §2).  Plain integers and pointers; shared by the
// library build and the run-time-compiled encoders (rs_encoder_jit.cpp).
#pragma once
#include "rs_types.hpp"

namespace uplink_ec {

// Max inputs / outputs of one launch (inputs = the k source shares, outputs =
// the rows computed).  Larger row counts are split over several launches.
constexpr int kMaxOps = 128;

// RsArgs::queue points at a pair of counters: the launch's tile counter at
// word 0 and, at this word, the count of its workgroups that are done; both
// are zero when a launch starts, and its last workgroup zeroes them again.
constexpr int kQueueDoneWord = 32;

// One launch computes, for every byte column (stripe s, offset t < ess) of
// every segment g in the batch:
//   out_r[g, s, t] = XOR_j  M[r][j] * in_j[g, s, t]      (GF(2^8))
// with
//   in_j [g,s,t] = in_base  + g*in_seg_stride  + in_off[j]  + s*in_stripe_stride  + t
//   out_r[g,s,t] = out_base + g*out_seg_stride + out_off[r] + s*out_stripe_stride + t
// and, for inputs with copy_off[j] >= 0, the input bytes are also copied to
//   out_base + g*out_seg_stride + copy_off[j] + s*out_stripe_stride + t
// (the systematic pass-through of data shares: EncodeSingle num<k and
// Rebuild's present data shares).
//
// Encode of a segment [stripe][k][ess] into pieces [n][stripes*ess]:
//   in_off[j] = j*ess, in_stripe_stride = k*ess,
//   out_off[r] = (k+r)*piece_len, copy_off[j] = j*piece_len,
//   out_stripe_stride = ess.
// Rebuild from pieces into a stripe-major segment swaps the two layouts.
struct RsArgs {
    const uint8_t *in_base;
    uint8_t *out_base;
    const uint8_t *coef;      // runtime matrix, coef[j*coef_ld + r] (generic kernel)
    const uint64_t *jt_tgt;   // leaf addresses of coef (jt_targets_bytes; null: made per launch)
    int64_t in_stripe_stride;
    int64_t out_stripe_stride;
    int64_t in_seg_stride;
    int64_t out_seg_stride;
    int64_t nstripes;         // stripes per segment
    int64_t chunks_per_seg;   // nstripes * ess / 16
    int64_t tiles_per_seg;    // ceil(chunks_per_seg / 128)
    int64_t total_tiles;      // tiles_per_seg * nseg
    // compile-time encoder: 1-KiB column blocks (64 chunks of one share row),
    // paired across the batch (rs_tile.hpp pair_cols), handed out by a queue
    int64_t blocks_per_seg;   // ceil(chunks_per_seg / 64)
    int64_t total_blocks;     // blocks_per_seg * nseg
    uint32_t *queue;          // zero work counters of this launch, see kQueueDoneWord (null: static assignment)
    uint32_t *queue_host_done;  // with queue: the slot's completion word (pinned host memory)
    uint32_t queue_seq;       // stored there by the launch's last workgroup
    // runtime-matrix kernel: when set, the computed rows from nstore on are
    // checked for zero instead of stored (syndrome rows of ec_decode_segments);
    // each wave that finds a non-zero byte in a valid column adds 1 here
    uint32_t *zero_check;
    int32_t ess;              // erasure share size, multiple of 16 for the bit-sliced path
    int32_t cps;              // ess / 16 (16-byte chunks per share per stripe)
    int32_t nin;              // number of inputs (k)
    int32_t nout;             // number of computed rows
    int32_t coef_ld;          // leading dimension of coef (multiple of 16)
    int32_t nstore;           // with zero_check: rows below this are stored, the rest checked (fused Decode)
    // byte ranges every input read / output write of the launch must stay in
    // (set by the host from the geometry above; the checked build of the
    // library, UPLINK_EC_CHECKED, skips any access outside them and reports it)
    const uint8_t *chk_in_lo, *chk_in_hi;
    const uint8_t *chk_out_lo, *chk_out_hi;
    uint32_t *chk_flag;       // checked build: first violating site (0 = none)
    int64_t in_off[kMaxOps];  // bytes from in_base (16-byte aligned on the bit-sliced path)
    int64_t out_off[kMaxOps]; // bytes from out_base
    int64_t copy_off[kMaxOps];// bytes from out_base, -1 = no copy
    uint64_t *diag;           // diagnostic encoder forms only (rs_encoder.hpp kDiagStamp); null otherwise
};

}  // namespace uplink_ec
