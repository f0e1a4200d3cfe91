// Device-side building blocks of the bit-sliced GF(2^8) stripe kernels
// (tile geometry, bit-slice transposes, LDS staging, row output and the
// compile-time-G body).  Included by rs_kernels.hip (and by the developer
// experiments under tools/exp/).  See rs_kernels.hip for the design notes.
#pragma once
#include <utility>

#include "gf256.hpp"
#include "rs_kernels.hpp"

namespace uplink_ec {
namespace dev {

template <typename F, int... I>
__device__ __forceinline__ void sf_impl(F &&f, std::integer_sequence<int, I...>) {
    (f.template operator()<I>(), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    sf_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int kTileChunks = 128;  // 16-byte chunks per tile = 2048 byte columns

__device__ __forceinline__ void swapmove(uint32_t &a, uint32_t &b, int s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}

// 32 bytes (byte b of word w) -> 8 planes: plane p, bit 8b+w = bit p of byte (w,b).
__device__ __forceinline__ void bitslice8(uint32_t (&w)[8]) {
    swapmove(w[0], w[4], 4, 0x0F0F0F0Fu);
    swapmove(w[1], w[5], 4, 0x0F0F0F0Fu);
    swapmove(w[2], w[6], 4, 0x0F0F0F0Fu);
    swapmove(w[3], w[7], 4, 0x0F0F0F0Fu);
    swapmove(w[0], w[2], 2, 0x33333333u);
    swapmove(w[1], w[3], 2, 0x33333333u);
    swapmove(w[4], w[6], 2, 0x33333333u);
    swapmove(w[5], w[7], 2, 0x33333333u);
    swapmove(w[0], w[1], 1, 0x55555555u);
    swapmove(w[2], w[3], 1, 0x55555555u);
    swapmove(w[4], w[5], 1, 0x55555555u);
    swapmove(w[6], w[7], 1, 0x55555555u);
}

// inverse of bitslice8 (each swap-move is an involution; reverse the stages)
__device__ __forceinline__ void unbitslice8(uint32_t (&w)[8]) {
    swapmove(w[0], w[1], 1, 0x55555555u);
    swapmove(w[2], w[3], 1, 0x55555555u);
    swapmove(w[4], w[5], 1, 0x55555555u);
    swapmove(w[6], w[7], 1, 0x55555555u);
    swapmove(w[0], w[2], 2, 0x33333333u);
    swapmove(w[1], w[3], 2, 0x33333333u);
    swapmove(w[4], w[6], 2, 0x33333333u);
    swapmove(w[5], w[7], 2, 0x33333333u);
    swapmove(w[0], w[4], 4, 0x0F0F0F0Fu);
    swapmove(w[1], w[5], 4, 0x0F0F0F0Fu);
    swapmove(w[2], w[6], 4, 0x0F0F0F0Fu);
    swapmove(w[3], w[7], 4, 0x0F0F0F0Fu);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-byte global store; NT = non-temporal (streamed output written once,
// never re-read by this kernel: keeps it from displacing useful lines).
template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    if constexpr (NT) {
        __builtin_nontemporal_store((u32x4){x, y, z, w}, (u32x4 *)p);
    } else {
        *(uint4 *)p = make_uint4(x, y, z, w);
    }
}

template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *(const uint4 *)p;
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations but, unlike __syncthreads() (whose release fence emits
// s_waitcnt vmcnt(0)), does not drain outstanding global stores.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct TileCols {
    bool vA, vB;
    int64_t inA, inB;    // byte offsets of the two chunks in an input share
    int64_t outA, outB;  // byte offsets of the two chunks in an output row
};

__device__ __forceinline__ TileCols tile_cols(const RsArgs &a, int64_t tt, int lane) {
    TileCols c;
    const int64_t qA = tt * kTileChunks + lane;
    const int64_t qB = qA + 64;
    c.vA = qA < a.chunks_per_seg;
    c.vB = qB < a.chunks_per_seg;
    const uint32_t cps = (uint32_t)a.cps;
    const uint32_t sA = (uint32_t)qA / cps, tA = (uint32_t)qA - sA * cps;
    const uint32_t sB = (uint32_t)qB / cps, tB = (uint32_t)qB - sB * cps;
    c.inA = (int64_t)sA * a.in_stripe_stride + (int64_t)tA * 16;
    c.inB = (int64_t)sB * a.in_stripe_stride + (int64_t)tB * 16;
    c.outA = (int64_t)sA * a.out_stripe_stride + (int64_t)tA * 16;
    c.outB = (int64_t)sB * a.out_stripe_stride + (int64_t)tB * 16;
    return c;
}

// Phase A: inputs j0 .. j0+jn-1 (thread handles j = j0 + wave + NW*i), load
// two 16-byte chunks, optionally copy them through (systematic shares),
// bit-slice and write the planes to lds[(j-j0)*8 + p][lane].
template <int NW, int PER, bool NT = false>
__device__ __forceinline__ void stage_inputs(const RsArgs &a, int64_t seg, const TileCols &c, uint32_t *lds,
                                             int lane, int wave, int j0, int jn, bool do_copy) {
    uint4 bufA[PER], bufB[PER];
    const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
    const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const uint8_t *p = in_seg + a.in_off[j0 + j];
            bufA[i] = c.vA ? ld16<NT>(p + c.inA) : z;
            bufB[i] = c.vB ? ld16<NT>(p + c.inB) : z;
        }
    }
    uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const int64_t co = a.copy_off[j0 + j];
            if (do_copy && co >= 0) {
                uint8_t *p = out_seg + co;
                if (c.vA) st16<NT>(p + c.outA, bufA[i].x, bufA[i].y, bufA[i].z, bufA[i].w);
                if (c.vB) st16<NT>(p + c.outB, bufB[i].x, bufB[i].y, bufB[i].z, bufB[i].w);
            }
            uint32_t w[8] = {bufA[i].x, bufA[i].y, bufA[i].z, bufA[i].w,
                             bufB[i].x, bufB[i].y, bufB[i].z, bufB[i].w};
            bitslice8(w);
            uint32_t *dst = lds + j * 8 * 64 + lane;
#pragma unroll
            for (int p = 0; p < 8; p++) dst[p * 64] = w[p];
        }
    }
}

// Output: un-bit-slice each accumulated row and store its two chunks.
template <int OPW, bool NT = false>
__device__ __forceinline__ void store_rows(const RsArgs &a, int64_t seg, const TileCols &c, int rbase, int cnt,
                                           uint32_t (&acc)[OPW][8]) {
    uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
    static_for<OPW>([&]<int O>() {
        if (O < cnt) {
            uint32_t w[8];
#pragma unroll
            for (int p = 0; p < 8; p++) w[p] = acc[O][p];
            unbitslice8(w);
            uint8_t *p = out_seg + a.out_off[rbase + O];
            if (c.vA) st16<NT>(p + c.outA, w[0], w[1], w[2], w[3]);
            if (c.vB) st16<NT>(p + c.outB, w[4], w[5], w[6], w[7]);
        }
    });
}

// ------------------------------------------------ compile-time-G encoder body
template <int K, int N, int OPW, int W>
__device__ __forceinline__ void compute_special(const uint32_t *lds, int lane, uint32_t (&acc)[OPW][8]) {
    static_for<K>([&]<int J>() {
        uint32_t x[8];
        static_for<8>([&]<int P>() { x[P] = lds[(J * 8 + P) * 64 + lane]; });
        uint32_t lo[16], hi[16];
        lo[0] = 0;
        hi[0] = 0;
        static_for<15>([&]<int M1>() {
            constexpr int M = M1 + 1;
            constexpr int low = M & (-M);
            constexpr int bit = low == 1 ? 0 : low == 2 ? 1 : low == 4 ? 2 : 3;
            if constexpr (M == low) {
                lo[M] = x[bit];
                hi[M] = x[4 + bit];
            } else {
                lo[M] = lo[M ^ low] ^ x[bit];
                hi[M] = hi[M ^ low] ^ x[4 + bit];
            }
        });
        static_for<OPW>([&]<int O>() {
            constexpr int r = W * OPW + O;
            if constexpr (r < N - K) {
                constexpr uint8_t cval = gen_entry(K, K + r, J);
                static_for<8>([&]<int P>() {
                    constexpr uint8_t row = mul_bitrow(cval, P);
                    constexpr int L = row & 15, H = row >> 4;
                    if constexpr (L != 0 && H != 0)
                        acc[O][P] = __builtin_amdgcn_bitop3_b32(acc[O][P], lo[L], hi[H], 0x96);
                    else if constexpr (L != 0)
                        acc[O][P] ^= lo[L];
                    else if constexpr (H != 0)
                        acc[O][P] ^= hi[H];
                });
            }
        });
    });
}

// ------------------------------------------------ runtime-matrix body
// rs_jump_table.inc (tools/gen/gen_jump_table.py): 256 compile-time leaves,
// leaf c = "acc[row] ^= c * x" as one v_bitop3 per plane from the 4-plane
// XOR combinations lo[1..15] / hi[1..15] of the current input x.
#include "rs_jump_table.inc"

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// acc[O] ^= sum over the n inputs j of D[row O][j] * x_j, for the wave's
// 8 - skip accumulator rows.  xa = LDS byte address of plane 0 of the first
// input for this lane (plane p at +256 p, the next input 2 KiB on); tp = the
// first input's 8 absolute leaf addresses of the wave's rows, right-aligned
// (entry skip + i holds row i), in global memory (rs_jt_targets), the next
// input's `tstride` bytes on.  Per input, one scalar load brings the leaf
// addresses straight into the call registers s[52:67] while the planes land
// in the single-bit slots lo[1,2,4,8] / hi[1,2,4,8]; 22 XORs fill the other
// combinations; then, with VGPR index mode on for the accumulator operand
// (SRC0 and DST, M0 = 8 * row, stepped by each leaf), a jump enters the
// sequence of eight s_swappc_b64 (4 bytes each) at call site `skip`, so only
// the wave's rows are visited; the leaves return with s_setpc_b64.  The loop
// over the inputs is part of the asm, so the call-site entry and M0 are set
// up once per chunk.  Registers are fixed by the register contract of
// rs_jump_table.inc: acc in v[32:95] (pinned operands), combinations
// v[96:125], s[42:67] scratch.  n >= 1.
__device__ __forceinline__ void jt_inputs(u32x8 (&acc)[8], uint32_t xa, const uint64_t *tp, uint32_t tstride,
                                          uint32_t skip, uint32_t n) {
    asm volatile(
        "s_load_dwordx16 s[52:67], %[tp], 0x0\n"
        "s_mov_b64 s[44:45], %[tp]\n"
        "s_mov_b32 s46, %[n]\n"
        "s_mov_b32 s51, m0\n"
        "s_getpc_b64 s[42:43]\n"
        ".Ljt_pc%=:\n"
        "s_lshl_b32 s50, %[skip], 2\n"
        "s_add_u32 s42, s42, s50\n"
        "s_addc_u32 s43, s43, 0\n"
        "s_add_u32 s42, s42, .Ljt_sites%=-.Ljt_pc%=\n"
        "s_addc_u32 s43, s43, 0\n"
        ".Ljt_loop%=:\n"
        "ds_read_b32 v96, %[xa]\n"
        "ds_read_b32 v97, %[xa] offset:256\n"
        "ds_read_b32 v99, %[xa] offset:512\n"
        "ds_read_b32 v103, %[xa] offset:768\n"
        "ds_read_b32 v111, %[xa] offset:1024\n"
        "ds_read_b32 v112, %[xa] offset:1280\n"
        "ds_read_b32 v114, %[xa] offset:1536\n"
        "ds_read_b32 v118, %[xa] offset:1792\n"
        "v_add_u32 %[xa], 0x800, %[xa]\n"
        "s_add_u32 s44, s44, %[ts]\n"
        "s_addc_u32 s45, s45, 0\n"
        "s_sub_u32 s46, s46, 1\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_xor_b32 v98, v96, v97\n"
        "v_xor_b32 v100, v96, v99\n"
        "v_xor_b32 v101, v97, v99\n"
        "v_xor_b32 v102, v98, v99\n"
        "v_xor_b32 v104, v96, v103\n"
        "v_xor_b32 v105, v97, v103\n"
        "v_xor_b32 v106, v98, v103\n"
        "v_xor_b32 v107, v99, v103\n"
        "v_xor_b32 v108, v100, v103\n"
        "v_xor_b32 v109, v101, v103\n"
        "v_xor_b32 v110, v102, v103\n"
        "v_xor_b32 v113, v111, v112\n"
        "v_xor_b32 v115, v111, v114\n"
        "v_xor_b32 v116, v112, v114\n"
        "v_xor_b32 v117, v113, v114\n"
        "v_xor_b32 v119, v111, v118\n"
        "v_xor_b32 v120, v112, v118\n"
        "v_xor_b32 v121, v113, v118\n"
        "v_xor_b32 v122, v114, v118\n"
        "v_xor_b32 v123, v115, v118\n"
        "v_xor_b32 v124, v116, v118\n"
        "v_xor_b32 v125, v117, v118\n"
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
        "s_cmp_eq_u32 s46, 0\n"
        "s_cbranch_scc1 .Ljt_done%=\n"
        "s_load_dwordx16 s[52:67], s[44:45], 0x0\n"
        "s_branch .Ljt_loop%=\n"
        ".Ljt_done%=:\n"
        "s_mov_b32 m0, s51\n"
        : "+{v[32:39]}"(acc[0]), "+{v[40:47]}"(acc[1]), "+{v[48:55]}"(acc[2]), "+{v[56:63]}"(acc[3]),
          "+{v[64:71]}"(acc[4]), "+{v[72:79]}"(acc[5]), "+{v[80:87]}"(acc[6]), "+{v[88:95]}"(acc[7]), [xa] "+v"(xa)
        : [tp] "s"(tp), [ts] "s"(tstride), [skip] "s"(skip), [n] "s"(n)
        : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",
          "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
          "v122", "v123", "v124", "v125", "s42", "s43", "s44", "s45", "s46", "s48", "s49", "s50", "s51",
          "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66",
          "s67", "scc", "memory");
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
