// Rebuild / Decode of a batch of segments that each come with their own share
// set (a download's segment is decoded from whichever k pieces answered
// first: private/eestream/stripe.go:314-354, private/ecclient/client.go:273-308,
// several at once under prefetch, private/storage/streams/store.go:240-253).
//
// Nothing is prepared on the host beyond the share choice: per segment the
// host writes a SetStage into pinned memory (one DMA takes the call's records
// to device memory); one launch of rs_sets_prep (one
// workgroup per segment) copies its descriptor to the device, computes the
// segment's decode rows (Lagrange interpolation weights, closed form) and
// writes the jump-table leaf addresses of those rows; then rs_matmul_sets<NW> rebuilds every
// segment's stripes, one workgroup per 2048-column tile, each tile reading
// its segment's descriptor.  All of it is stream-ordered on the caller's
// stream: no host synchronisation, no module load, no shared setup stream.
#pragma once
#include "rs_args.hpp"

namespace uplink_ec {

// One segment of a sets launch, in device memory.
struct SetDesc {
    const uint8_t *in[kMaxOps];  // the segment's input shares (the k basis shares first), nstripes*ess bytes each
    uint8_t *out;                // the segment, stripe-major [stripe][k][ess]
    uint64_t *tgt;               // leaf addresses [pass][input][group][8] (rs_sets_prep)
    uint32_t *zero_check;        // Decode: this segment's syndrome counter (rows from nstore on); null: Rebuild
    int32_t nin, nout, nstore, status;  // status: 0, or EC_ERR_SINGULAR (nothing is written then)
    int32_t copy_off[kMaxOps];   // byte offset within a stripe of the output a basis data share is copied to, -1 none
    int32_t out_off[kMaxOps];    // byte offset within a stripe of computed row r (rows < nstore)
};
static_assert(sizeof(SetDesc) % 8 == 0, "copied as 8-byte words");

// What the host writes per segment (pinned memory, copied to the device, read once by rs_sets_prep).
// Inputs are the k basis shares (infectious' choice, position p holds share
// num[p]; a present data share d sits at position d) followed by the other
// shares (Decode).  Rows: the nstore missing data positions missing[r], then
// one syndrome row per non-basis input (rows nstore.., input k + r - nstore).
struct SetStage {
    SetDesc d;
    int32_t num[kMaxOps];
    int32_t missing[kMaxOps];
    int32_t k, nw, pad0, pad1;
};

// Kernel arguments of rs_matmul_sets (one launch per wave-count class).
struct SetsArgs {
    const SetDesc *desc;     // this launch's segments
    int64_t nstripes, chunks_per_seg, tiles_per_seg, total_tiles;
    int32_t ess, cps, k, pad;
    // completion of the whole call (every class launch): each workgroup adds 1
    // to *done_ctr when it has read everything it reads from the slot; the one
    // that brings it to total_wgs zeroes it and stores seq to *host_done
    // (pinned), which tells the host the slot's staging and tables are free
    uint32_t *done_ctr;
    uint32_t *host_done;
    uint32_t seq, total_wgs;
    uint32_t *chk_flag;  // checked build: first access outside a share / segment (site 8 or 9)
    uint64_t jt_base;    // rs_sets_fused1: address of leaf 0
};

constexpr int64_t kTileChunksHost = 128;  // 16-byte chunks per tile (rs_tile.hpp kTileChunks)

// waves per workgroup for `rows` computed rows (<= 14 -> 2, <= 24 -> 3, else 4,
// at most 8 rows per wave)
int sets_waves(int rows);
size_t sets_tgt_entries(int nin, int rows, int nw);  // 64-bit words of one segment's leaf table on nw waves
// most tiles one rs_matmul_sets launch on nw waves takes (one workgroup per tile, the grid's
// work-items below 2^32)
int64_t sets_max_tiles(int nw);
// one workgroup per segment; jt_base = address of leaf 0 (jt_table_base_addr);
// zeroes *done_ctr for the launches that follow
hipError_t launch_sets_prep(const SetStage *stage, SetDesc *desc, int nseg, uint64_t jt_base, uint32_t *done_ctr,
                            hipStream_t s);
// the same for one segment, its record passed in the launch's arguments
hipError_t launch_sets_prep1(const SetStage &stage, SetDesc *desc, uint64_t jt_base, uint32_t *done_ctr,
                             hipStream_t s);
static_assert(sizeof(SetStage) + 3 * sizeof(void *) <= 4096, "a launch's arguments are at most 4 KB");
hipError_t launch_matmul_sets(const SetsArgs &a, int nw, hipStream_t s);

// One segment's Rebuild in one launch (rs_sets_one): its record and its decode
// rows' coefficients, solved on the host, are the launch's arguments; every
// workgroup writes the leaf table (the same bytes) and reads it back.  Field
// names as SetDesc's (the tile body reads either).
constexpr int kOneMaxIn = 64, kOneMaxCoef = 2048;
struct SetOne {
    SetsArgs a;
    const uint8_t *in[kOneMaxIn];
    uint8_t *out;
    uint64_t *tgt;         // the leaf table [pass][input][group][8]
    uint32_t *zero_check;  // null (Rebuild)
    int32_t nin, nout, nstore, status;
    int32_t copy_off[kOneMaxIn];
    int32_t out_off[kOneMaxIn];
    uint8_t coef[kOneMaxCoef];  // coef[r * nin + j]: row r's coefficient of input j
};
static_assert(sizeof(SetOne) <= 4096, "a launch's arguments are at most 4 KB");
// *p.a.done_ctr must be 0 (every pass leaves it so)
hipError_t launch_sets_one(const SetOne &p, int nw, hipStream_t s);
// address of the jump table's leaf 0 on the current device (one small launch on
// s, synchronous; the table sits in rs_jt_targets' code)
hipError_t jt_table_base_addr(uint64_t *out, hipStream_t s);

}  // namespace uplink_ec
