// Device side of the runtime-matrix kernel (rebuild, and encode without a
// compile-time-G kernel): the jump-table multiply-accumulate body.  Included
// by rs_kernels.hip (and by developer experiments under tools/exp/).
#pragma once
#include "rs_tile.hpp"

namespace uplink_ec {
namespace dev {

// stage_inputs split in two, so the runtime-matrix kernel can issue the
// global loads of its next chunk of input shares before it multiplies in the
// current one: load_inputs fills registers, slice_inputs copies the present
// data shares through, bit-slices and writes LDS.
template <int PER>
struct StageRegs {
    uint4 A[PER], B[PER];
};

template <int NW, int PER, bool NT = false>
__device__ __forceinline__ void load_inputs(const RsArgs &a, int64_t seg, const TileCols &c, int wave, int j0, int jn,
                                            StageRegs<PER> &r) {
    // Columns past the end of the segment load column 0 of the same share
    // instead of branching; their planes are never stored (slice_inputs and
    // store_rows test vA / vB).
    const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
    const int64_t oA = c.vA ? c.inA : 0, oB = c.vB ? c.inB : 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const uint8_t *p = in_seg + a.in_off[j0 + j];
            const uint4 z = make_uint4(0, 0, 0, 0);
            r.A[i] = in_range(a, p + oA, false, 4) ? ld16<NT>(p + oA) : z;
            r.B[i] = in_range(a, p + oB, false, 4) ? ld16<NT>(p + oB) : z;
        }
    }
}

// WIDE: the straight-line body's layout -- per input 2 KiB, planes 0-3 of a
// lane as one 16-byte word at 16 lane, planes 4-7 at 1024 + 16 lane (two
// ds_read_b128 per input, conflict-free); otherwise plane p at 256 p + 4 lane.
template <int NW, int PER, bool NT = false, bool WIDE = false>
__device__ __forceinline__ void slice_inputs(const RsArgs &a, int64_t seg, const TileCols &c, uint32_t *lds, int lane,
                                             int wave, int j0, int jn, bool do_copy, const StageRegs<PER> &r) {
    uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const int64_t co = a.copy_off[j0 + j];
            if (do_copy && co >= 0) {
                uint8_t *p = out_seg + co;
                if (c.vA && in_range(a, p + c.outA, true, 5)) st16<NT>(p + c.outA, r.A[i].x, r.A[i].y, r.A[i].z, r.A[i].w);
                if (c.vB && in_range(a, p + c.outB, true, 5)) st16<NT>(p + c.outB, r.B[i].x, r.B[i].y, r.B[i].z, r.B[i].w);
            }
            uint32_t w[8] = {r.A[i].x, r.A[i].y, r.A[i].z, r.A[i].w, r.B[i].x, r.B[i].y, r.B[i].z, r.B[i].w};
            bitslice8(w);
            if constexpr (WIDE) {
                u32x4 *dst = (u32x4 *)(lds + j * 8 * 64) + lane;
                dst[0] = (u32x4){w[0], w[1], w[2], w[3]};
                dst[64] = (u32x4){w[4], w[5], w[6], w[7]};
            } else {
                uint32_t *dst = lds + j * 8 * 64 + lane;
#pragma unroll
                for (int p = 0; p < 8; p++) dst[p * 64] = w[p];
            }
        }
    }
}

// ------------------------------------------------ runtime-matrix body
// rs_jump_table.inc (tools/gen/gen_jump_table.py): 256 compile-time leaves,
// leaf c = "acc[row] ^= c * x" as one v_bitop3 per plane from the 4-plane
// XOR combinations lo[1..15] / hi[1..15] of the current input x, and the XORs
// that make those combinations (RS_JT_COMBOS_ASM).
#include "rs_jump_table.inc"

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// acc[O] ^= sum over the n inputs j of D[row O][j] * x_j, for the wave's
// 8 - skip accumulator rows.  xa = LDS byte address of the first input for
// this lane in the wide layout (slice_inputs WIDE: planes 0-3 of the lane as
// one 16-byte word at +0, planes 4-7 at +1024, the next input 2 KiB on); tp =
// the first input's 8 absolute leaf addresses of the wave's rows, right-aligned
// (entry skip + i holds row i), in global memory (rs_jt_targets), the next
// input's `tstride` bytes on.  Per input, one scalar load brings the leaf
// addresses straight into the call registers s[52:67] while two ds_read_b128
// put the planes in the single-bit slots lo[1,2,4,8] / hi[1,2,4,8] (v[96:103]);
// 22 XORs fill the other combinations; then, with VGPR index mode on for the accumulator operand
// (SRC0 and DST, M0 = 8 * row, stepped by each leaf), a jump enters the
// sequence of eight s_swappc_b64 (4 bytes each) at call site `skip`, so only
// the wave's rows are visited; the leaves return with s_setpc_b64.  The loop
// over the inputs is part of the asm, so the call-site entry and M0 are set
// up once per chunk.  Registers are fixed by the register contract of
// rs_jump_table.inc: acc in v[32:95] (pinned operands), combinations
// v[96:125], s[42:43], s[48:49], s51, s[52:67] scratch (the loop state lives
// in compiler-allocated operands, so the compiler keeps its own SGPRs without
// spilling).  n >= 1.
__device__ __forceinline__ void jt_inputs(u32x8 (&acc)[8], uint32_t xa, const uint64_t *tp, uint32_t tstride,
                                          uint32_t skip, uint32_t n) {
    uint32_t off = 0;  // byte offset of the current input's leaf addresses from tp
    asm volatile(
        "s_load_dwordx16 s[52:67], %[tp], 0x0\n"
        "s_mov_b32 s51, m0\n"
        "s_getpc_b64 s[42:43]\n"
        ".Ljt_pc%=:\n"
        "s_lshl_b32 s48, %[skip], 2\n"  // s48: scratch until the first call writes the return address
        "s_add_u32 s42, s42, s48\n"
        "s_addc_u32 s43, s43, 0\n"
        "s_add_u32 s42, s42, .Ljt_sites%=-.Ljt_pc%=\n"
        "s_addc_u32 s43, s43, 0\n"
        ".Ljt_loop%=:\n"
        "ds_read_b128 v[96:99], %[xa]\n"
        "ds_read_b128 v[100:103], %[xa] offset:1024\n"
        "v_add_u32 %[xa], 0x800, %[xa]\n"
        "s_add_u32 %[off], %[off], %[ts]\n"
        "s_sub_u32 %[n], %[n], 1\n"
        "s_waitcnt lgkmcnt(0)\n"
        RS_JT_COMBOS_ASM
        "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
        "s_setpc_b64 s[42:43]\n"
        ".Ljt_sites%=:\n"
        "s_swappc_b64 s[48:49], s[52:53]\n"
        "s_swappc_b64 s[48:49], s[54:55]\n"
        "s_swappc_b64 s[48:49], s[56:57]\n"
        "s_swappc_b64 s[48:49], s[58:59]\n"
        "s_swappc_b64 s[48:49], s[60:61]\n"
        "s_swappc_b64 s[48:49], s[62:63]\n"
        "s_swappc_b64 s[48:49], s[64:65]\n"
        "s_swappc_b64 s[48:49], s[66:67]\n"
        "s_set_gpr_idx_off\n"
        "s_cmp_eq_u32 %[n], 0\n"
        "s_cbranch_scc1 .Ljt_done%=\n"
        "s_load_dwordx16 s[52:67], %[tp], %[off]\n"
        "s_branch .Ljt_loop%=\n"
        ".Ljt_done%=:\n"
        "s_mov_b32 m0, s51\n"
        : "+{v[32:39]}"(acc[0]), "+{v[40:47]}"(acc[1]), "+{v[48:55]}"(acc[2]), "+{v[56:63]}"(acc[3]),
          "+{v[64:71]}"(acc[4]), "+{v[72:79]}"(acc[5]), "+{v[80:87]}"(acc[6]), "+{v[88:95]}"(acc[7]), [xa] "+v"(xa),
          [off] "+s"(off), [n] "+s"(n)
        : [tp] "s"(tp), [ts] "s"(tstride), [skip] "s"(skip)
        : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",
          "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
          "v122", "v123", "v124", "v125", "s42", "s43", "s48", "s49", "s51",
          "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",
          "s67", "scc", "memory");
}

// The straight-line form (rs_sl.hpp): one call into the plan's generated
// segment for this chunk, rows and wave; it reads the chunk's planes from LDS
// at xa (pinned to v126), uses v[96:125] as scratch, adds into the
// accumulators and returns through s[48:49].
// `tp` points at the segment's address in the plan's table (a scalar load
// inside the asm: the compiler would fetch it with a vector load).
__device__ __forceinline__ void sl_segment(u32x8 (&acc)[8], uint32_t xa, const uint64_t *tp) {
    asm volatile(
        "s_load_dwordx2 s[52:53], %[tp], 0x0\n"
        "s_waitcnt lgkmcnt(0)\n"
        "s_swappc_b64 s[48:49], s[52:53]"
        : "+{v[32:39]}"(acc[0]), "+{v[40:47]}"(acc[1]), "+{v[48:55]}"(acc[2]), "+{v[56:63]}"(acc[3]),
          "+{v[64:71]}"(acc[4]), "+{v[72:79]}"(acc[5]), "+{v[80:87]}"(acc[6]), "+{v[88:95]}"(acc[7])
        : [tp] "s"(tp), "{v126}"(xa)
        : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",
          "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",
          "v123", "v124", "v125", "s48", "s49", "s52", "s53", "memory");
}

// Absolute address of leaf 0 of the jump table.  The table itself sits here,
// behind a branch, in the code of the one kernel that calls this
// (rs_jt_targets); the leaves are position-independent code that any kernel
// honouring the register contract calls through the addresses it computes.
__device__ __forceinline__ uint64_t jt_table_base() {
    uint32_t lo, hi;
    asm volatile(
        "s_getpc_b64 s[40:41]\n"
        ".Ltb_pc%=:\n"
        "s_add_u32 s40, s40, .Ltb_tab%=-.Ltb_pc%=\n"
        "s_addc_u32 s41, s41, 0\n"
        "s_mov_b32 %0, s40\n"
        "s_mov_b32 %1, s41\n"
        "s_branch .Ltb_end%=\n"
        ".Ltb_tab%=:\n"
        RS_JUMP_TABLE_ASM
        ".Ltb_end%=:\n"
        : "=s"(lo), "=s"(hi)
        :
        : "s40", "s41", "scc");
    return ((uint64_t)hi << 32) | lo;
}

}  // namespace dev
}  // namespace uplink_ec
