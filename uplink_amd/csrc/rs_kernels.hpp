// Kernel argument block and launch entry points for the GF(2^8) Reed-Solomon
// stripe kernels (encode K1, rebuild K2 in SURVEY.md §2).  Host-only header:
// no torch types, plain pointers.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace uplink_ec {

// Max inputs / outputs of one launch (inputs = the k source shares, outputs =
// the rows computed).  Larger row counts are split over several launches.
constexpr int kMaxOps = 128;

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
    int32_t ess;              // erasure share size, multiple of 16 for the bit-sliced path
    int32_t cps;              // ess / 16 (16-byte chunks per share per stripe)
    int32_t nin;              // number of inputs (k)
    int32_t nout;             // number of computed rows
    int32_t coef_ld;          // leading dimension of coef (multiple of 16)
    int32_t pad_;
    int64_t in_off[kMaxOps];  // bytes from in_base (16-byte aligned on the bit-sliced path)
    int64_t out_off[kMaxOps]; // bytes from out_base
    int64_t copy_off[kMaxOps];// bytes from out_base, -1 = no copy
};

// Specialised compile-time-G encoders exist for these (k, n).
bool have_special_encoder(int k, int n);

// Launches.  `args.nout` rows of G (rows k..n-1) for the special encoder;
// any matrix for the generic kernel.  Return hipError_t.
hipError_t launch_encode_special(int k, int n, const RsArgs &args, int grid, hipStream_t stream);
hipError_t launch_matmul_generic(const RsArgs &args, int grid, hipStream_t stream);
// The generic kernel multiplies through a jump table whose leaf addresses
// depend on the matrix: launch_jt_targets writes them for args.coef / nin /
// nout into `targets` (jt_targets_bytes(args) bytes of device memory), after
// which args.jt_tgt = targets lets any number of launches of that matrix skip
// the per-launch preparation.
size_t jt_targets_bytes(const RsArgs &args);
hipError_t launch_jt_targets(const RsArgs &args, uint64_t *targets, hipStream_t stream);
// Byte-wise fallback (any ess, any alignment); coef as above.
hipError_t launch_matmul_bytes(const RsArgs &args, hipStream_t stream);

// Default grid (workgroups) for a launch over `total_tiles` tiles.
int default_grid(int64_t total_tiles, int wgs_per_cu);

}  // namespace uplink_ec
