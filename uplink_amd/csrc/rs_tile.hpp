// Device building blocks shared by the GF(2^8) stripe kernels: tile geometry,
// the bit-slice transposes, LDS staging of input shares and the output of
// computed rows.  Used by the compile-time-G encoders (rs_encoder.hpp, also
// compiled at run time by hiprtc) and the runtime-matrix kernel
// (rs_device.hpp / rs_kernels.hip); see rs_kernels.hip for the design notes.
#pragma once
#include "rs_args.hpp"

namespace uplink_ec {
namespace dev {

// static_for<N>(f): f.template operator()<I>() for I = 0 .. N-1, unrolled at
// compile time (clang's __make_integer_seq: no library header needed, so the
// same code compiles under hiprtc).
template <typename T, T... I>
struct iseq {};
template <typename F, int... I>
__device__ __forceinline__ void sf_impl(F &&f, iseq<int, I...>) {
    (f.template operator()<I>(), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    sf_impl(f, __make_integer_seq<iseq, int, N>{});
}

constexpr int kTileChunks = 128;  // 16-byte chunks per tile = 2048 byte columns

// Swap the bits m of b with the bits m << s of a (a "swap-move"), as two
// selects: b' = m ? a >> s : b, a' = (m << s) ? b << s : a.  v_bitop3 0xD8 is
// "S2 ? S1 : S0" (truth table over S0 = 0xF0, S1 = 0xCC, S2 = 0xAA), so this
// is 2 shifts + 2 bitop3 per pair instead of the classic 5-op
// t = ((a >> s) ^ b) & m; b ^= t; a ^= t << s, which the compiler does not
// fuse (49 instead of 67 VALU per 32-byte transpose).
__device__ __forceinline__ void swapmove(uint32_t &a, uint32_t &b, int s, uint32_t m) {
    const uint32_t na = __builtin_amdgcn_bitop3_b32(a, b << s, m << s, 0xD8);
    const uint32_t nb = __builtin_amdgcn_bitop3_b32(b, a >> s, m, 0xD8);
    a = na;
    b = nb;
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

// One 1-KiB LDS-DMA: 16 bytes per lane from g (per lane) to the LDS byte
// address lds (wave-uniform) + 16 lane, non-temporal.  Inline asm, so the
// compiler neither waits for it nor moves memory operations across it: the
// kernel's counted vmcnt waits retire it.  (M0 written by SALU and read by an
// LDS-DMA right after needs a wait state: the s_nop.)
// M0 is the compiler's, so the asm puts it back.
__device__ __forceinline__ void dma_1k(const uint8_t *g, uint32_t lds) {
    uint32_t save;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(save)
        : "v"(g), "s"(lds)
        : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 63] (gfx9's 6-bit counter).
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define UPLINK_WAIT_VM(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        UPLINK_WAIT_VM(1) UPLINK_WAIT_VM(2) UPLINK_WAIT_VM(3) UPLINK_WAIT_VM(4) UPLINK_WAIT_VM(5) UPLINK_WAIT_VM(6) UPLINK_WAIT_VM(7) UPLINK_WAIT_VM(8)
        UPLINK_WAIT_VM(9) UPLINK_WAIT_VM(10) UPLINK_WAIT_VM(11) UPLINK_WAIT_VM(12) UPLINK_WAIT_VM(13) UPLINK_WAIT_VM(14) UPLINK_WAIT_VM(15) UPLINK_WAIT_VM(16)
        UPLINK_WAIT_VM(17) UPLINK_WAIT_VM(18) UPLINK_WAIT_VM(19) UPLINK_WAIT_VM(20) UPLINK_WAIT_VM(21) UPLINK_WAIT_VM(22) UPLINK_WAIT_VM(23) UPLINK_WAIT_VM(24)
        UPLINK_WAIT_VM(25) UPLINK_WAIT_VM(26) UPLINK_WAIT_VM(27) UPLINK_WAIT_VM(28) UPLINK_WAIT_VM(29) UPLINK_WAIT_VM(30) UPLINK_WAIT_VM(31) UPLINK_WAIT_VM(32)
        UPLINK_WAIT_VM(33) UPLINK_WAIT_VM(34) UPLINK_WAIT_VM(35) UPLINK_WAIT_VM(36) UPLINK_WAIT_VM(37) UPLINK_WAIT_VM(38) UPLINK_WAIT_VM(39) UPLINK_WAIT_VM(40)
        UPLINK_WAIT_VM(41) UPLINK_WAIT_VM(42) UPLINK_WAIT_VM(43) UPLINK_WAIT_VM(44) UPLINK_WAIT_VM(45) UPLINK_WAIT_VM(46) UPLINK_WAIT_VM(47) UPLINK_WAIT_VM(48)
        UPLINK_WAIT_VM(49) UPLINK_WAIT_VM(50) UPLINK_WAIT_VM(51) UPLINK_WAIT_VM(52) UPLINK_WAIT_VM(53) UPLINK_WAIT_VM(54) UPLINK_WAIT_VM(55) UPLINK_WAIT_VM(56)
        UPLINK_WAIT_VM(57) UPLINK_WAIT_VM(58) UPLINK_WAIT_VM(59) UPLINK_WAIT_VM(60) UPLINK_WAIT_VM(61) UPLINK_WAIT_VM(62) UPLINK_WAIT_VM(63)
#undef UPLINK_WAIT_VM
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// Checked build (UPLINK_EC_CHECKED, tests/test_c_abi.py): every 16-byte
// global access of the stripe kernels is compared with the launch's declared
// byte ranges; one outside them is skipped and its site recorded in
// a.chk_flag, which the library reads after the launch.  In the product
// build this is `true` and compiles away.
__device__ __forceinline__ bool in_range(const RsArgs &a, const uint8_t *p, bool out, int site) {
#ifdef UPLINK_EC_CHECKED
    const uint8_t *lo = out ? a.chk_out_lo : a.chk_in_lo, *hi = out ? a.chk_out_hi : a.chk_in_hi;
    if (p < lo || p + 16 > hi) {
        if (a.chk_flag) atomicCAS(a.chk_flag, 0u, (uint32_t)site);
        return false;
    }
#else
    (void)a, (void)p, (void)out, (void)site;
#endif
    return true;
}

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

// The compile-time encoder's tile: two 1-KiB column blocks of the batch (64
// chunks of 16 B of every share row), block t and block t + ceil(B / 2) of the
// B blocks of all segments -- for a batch of segments, the same columns of
// segments g and g + nseg/2.  A lane's 32 bytes are chunk `lane` of each.
// Offsets are absolute (segment included).  Measured against two adjacent
// blocks (one 2-KiB tile of one segment): the encode's 80 piece streams are
// written at 5.6-6.5 instead of 4.5-4.7 TB/s (tools/exp/enc_shape_probe2.hip,
// DESIGN.md §4).
__device__ __forceinline__ void block_cols(const RsArgs &a, int64_t b, int lane, bool &v, int64_t &in, int64_t &out) {
    v = false;
    in = out = 0;
    if (b >= a.total_blocks) return;
    const uint32_t bps = (uint32_t)a.blocks_per_seg;
    const uint32_t seg = (uint32_t)b / bps;
    const int64_t q = (int64_t)((uint32_t)b - seg * bps) * 64 + lane;
    if (q >= a.chunks_per_seg) return;
    v = true;
    const uint32_t cps = (uint32_t)a.cps;
    const uint32_t s = (uint32_t)q / cps, t = (uint32_t)q - s * cps;
    in = (int64_t)seg * a.in_seg_stride + (int64_t)s * a.in_stripe_stride + (int64_t)t * 16;
    out = (int64_t)seg * a.out_seg_stride + (int64_t)s * a.out_stripe_stride + (int64_t)t * 16;
}

__device__ __forceinline__ int64_t pair_count(const RsArgs &a) { return (a.total_blocks + 1) >> 1; }

__device__ __forceinline__ TileCols pair_cols(const RsArgs &a, int64_t t, int lane) {
    TileCols c;
    block_cols(a, t, lane, c.vA, c.inA, c.outA);
    block_cols(a, t + pair_count(a), lane, c.vB, c.inB, c.outB);
    return c;
}

// Phase A: inputs j0 .. j0+jn-1 (thread handles j = j0 + wave + NW*i), load
// two 16-byte chunks, optionally copy them through (systematic shares),
// bit-slice and write the planes to lds[(j-j0)*8 + p][lane].  All loads are
// issued before the first is consumed (issuing them in smaller groups
// measured slower: tools/exp/enc_variants.py).
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
            bufA[i] = c.vA && in_range(a, p + c.inA, false, 1) ? ld16<NT>(p + c.inA) : z;
            bufB[i] = c.vB && in_range(a, p + c.inB, false, 1) ? ld16<NT>(p + c.inB) : z;
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
                if (c.vA && in_range(a, p + c.outA, true, 2)) st16<NT>(p + c.outA, bufA[i].x, bufA[i].y, bufA[i].z, bufA[i].w);
                if (c.vB && in_range(a, p + c.outB, true, 2)) st16<NT>(p + c.outB, bufB[i].x, bufB[i].y, bufB[i].z, bufB[i].w);
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
            if (c.vA && in_range(a, p + c.outA, true, 3)) st16<NT>(p + c.outA, w[0], w[1], w[2], w[3]);
            if (c.vB && in_range(a, p + c.outB, true, 3)) st16<NT>(p + c.outB, w[4], w[5], w[6], w[7]);
        }
    });
}

// Diagnostic stand-in for store_rows (rs_encoder.hpp kDiagNoParityStores):
// the rows are un-bit-sliced as for the store and kept live by an empty asm.
template <int OPW>
__device__ __forceinline__ void sink_rows(int cnt, uint32_t (&acc)[OPW][8]) {
    static_for<OPW>([&]<int O>() {
        if (O < cnt) {
            uint32_t w[8];
#pragma unroll
            for (int p = 0; p < 8; p++) w[p] = acc[O][p];
            unbitslice8(w);
            asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]), "v"(w[6]), "v"(w[7]));
        }
    });
}

}  // namespace dev
}  // namespace uplink_ec
