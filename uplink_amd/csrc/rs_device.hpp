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
__device__ __forceinline__ void mul2_planes(const uint32_t (&o)[8], uint32_t (&n)[8]) {
    // v*2 mod 0x11d on bit planes: bit0 <- b7, bit1 <- b0, bit2 <- b1^b7,
    // bit3 <- b2^b7, bit4 <- b3^b7, bit5 <- b4, bit6 <- b5, bit7 <- b6
    n[0] = o[7];
    n[1] = o[0];
    n[2] = o[1] ^ o[7];
    n[3] = o[2] ^ o[7];
    n[4] = o[3] ^ o[7];
    n[5] = o[4];
    n[6] = o[5];
    n[7] = o[6];
}

// add_nibble<B>(acc, y0..y3, c): acc ^= ((c >> B) & 15) * x on bit planes,
// y0..y3 = x*2^i (i = 0..3 of this nibble).  A 4-level tree of wave-uniform
// scalar bit tests picks one of 16 leaves; a leaf pairs the set bits so two
// multiples cost one v_bitop3 XOR3 per plane (expected 20 VALU per
// coefficient byte, vs 24 for fixed bit pairs and 32 for one branch per
// bit).  One asm block per nibble keeps the branches scalar (the compiler's
// structurizer turned the C++ forms into exec-masked code with extra moves).
#include "rs_nibble_tree.inc"

// Runtime-matrix body.  For input share j the multiples x*2^b are formed on
// the fly (3 XORs each on bit planes), four at a time; every output row then
// walks the nibble tree of its coefficient byte.  The wave's OPW coefficient
// bytes of input j sit in LDS (staged once per workgroup, zero-padded) and
// come in with one broadcast LDS read: no global load, and so no vmcnt wait
// behind outstanding stores, inside the j loop.  Forms measured in
// tools/exp/decode_exp.hip (RS(29,80), 64 MiB segments, m = 29 / 17 missing):
// one branch per bit 83/78 us, fixed bit pairs 71/55, nibble tree 66/52,
// + LDS coefficients 61.5/47.3.
template <int OPW>
__device__ __forceinline__ void compute_generic(const uint32_t *lds, const uint8_t *lcoef, int coef_stride, int lane,
                                                int jn, int cnt, uint32_t (&acc)[OPW][8]) {
    static_assert(OPW % 4 == 0, "coefficient slots are whole words");
    constexpr int NWORD = OPW / 4;
    for (int jj = 0; jj < jn; jj++) {
        uint32_t y0[8], y1[8], y2[8], y3[8];
#pragma unroll
        for (int p = 0; p < 8; p++) y0[p] = lds[(jj * 8 + p) * 64 + lane];
        const uint32_t *cp = (const uint32_t *)(lcoef + jj * coef_stride);
        uint32_t cw[NWORD];
#pragma unroll
        for (int q = 0; q < NWORD; q++) cw[q] = (uint32_t)__builtin_amdgcn_readfirstlane(cp[q]);
        mul2_planes(y0, y1);
        mul2_planes(y1, y2);
        mul2_planes(y2, y3);
        static_for<OPW>([&]<int O>() {
            if (O < cnt) add_nibble<8 * (O % 4)>(acc[O], y0, y1, y2, y3, cw[O / 4]);
        });
        mul2_planes(y3, y0);
        mul2_planes(y0, y1);
        mul2_planes(y1, y2);
        mul2_planes(y2, y3);
        static_for<OPW>([&]<int O>() {
            if (O < cnt) add_nibble<8 * (O % 4) + 4>(acc[O], y0, y1, y2, y3, cw[O / 4]);
        });
    }
}

}  // namespace dev
}  // namespace uplink_ec
