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

// acc ^= (bit B of c ? y : 0) ^ (bit B+1 of c ? z : 0), c wave-uniform.
// Two scalar tests pick one of three 8-instruction blocks: v_bitop3 XOR3 when
// both bits are set (one VALU per plane for two terms), v_xor otherwise.
// Written as one asm block so the branch structure stays scalar (the
// compiler's structurizer turned the C++ form into exec-masked code with
// ~300 extra v_mov per body: tools/exp/decode_exp.hip, MODE 7 vs 8).
template <int B>
__device__ __forceinline__ void add_bit_pair(uint32_t (&acc)[8], const uint32_t (&y)[8], const uint32_t (&z)[8],
                                             uint32_t c) {
#define UEC_PAIR_XOR(src)                                                                                      \
    "v_xor_b32 %[a0], %[a0], %[" src "0]\n v_xor_b32 %[a1], %[a1], %[" src "1]\n"                            \
    "v_xor_b32 %[a2], %[a2], %[" src "2]\n v_xor_b32 %[a3], %[a3], %[" src "3]\n"                            \
    "v_xor_b32 %[a4], %[a4], %[" src "4]\n v_xor_b32 %[a5], %[a5], %[" src "5]\n"                            \
    "v_xor_b32 %[a6], %[a6], %[" src "6]\n v_xor_b32 %[a7], %[a7], %[" src "7]\n"
#define UEC_PAIR_X3(i) "v_bitop3_b32 %[a" #i "], %[a" #i "], %[y" #i "], %[z" #i "] bitop3:0x96\n"
    asm volatile(
        "s_bitcmp1_b32 %[c], %[b0]\n"
        "s_cbranch_scc0 .Lpair_no0_%=\n"
        "s_bitcmp1_b32 %[c], %[b1]\n"
        "s_cbranch_scc0 .Lpair_only0_%=\n"
        UEC_PAIR_X3(0) UEC_PAIR_X3(1) UEC_PAIR_X3(2) UEC_PAIR_X3(3)
        UEC_PAIR_X3(4) UEC_PAIR_X3(5) UEC_PAIR_X3(6) UEC_PAIR_X3(7)
        "s_branch .Lpair_end_%=\n"
        ".Lpair_only0_%=:\n"
        UEC_PAIR_XOR("y")
        "s_branch .Lpair_end_%=\n"
        ".Lpair_no0_%=:\n"
        "s_bitcmp1_b32 %[c], %[b1]\n"
        "s_cbranch_scc0 .Lpair_end_%=\n"
        UEC_PAIR_XOR("z")
        ".Lpair_end_%=:\n"
        : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]),
          [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7])
        : [y0] "v"(y[0]), [y1] "v"(y[1]), [y2] "v"(y[2]), [y3] "v"(y[3]), [y4] "v"(y[4]), [y5] "v"(y[5]),
          [y6] "v"(y[6]), [y7] "v"(y[7]), [z0] "v"(z[0]), [z1] "v"(z[1]), [z2] "v"(z[2]), [z3] "v"(z[3]),
          [z4] "v"(z[4]), [z5] "v"(z[5]), [z6] "v"(z[6]), [z7] "v"(z[7]), [c] "s"(c), [b0] "i"(B),
          [b1] "i"(B + 1)
        : "scc");
#undef UEC_PAIR_XOR
#undef UEC_PAIR_X3
}

// Runtime-matrix body: for input share j the multiples x*2^b (b = 0..7) are
// formed on the fly (3 XORs each on bit planes), and for every output row
// the coefficient's bits are taken in pairs (b, b+1): wave-uniform scalar
// branches add x*2^b and/or x*2^(b+1) with 8 VALU (expected 6 per pair
// instead of 8 for one branch per bit).  Measured fastest of the runtime
// forms tried (per-bit branches, dense SGPR-masked bitop3, C++ 2-bit
// branches, two tiles per branch): tools/exp/decode_exp.hip.
template <int OPW>
__device__ __forceinline__ void compute_generic(const RsArgs &a, const uint32_t *lds, int lane, int jbase, int jn,
                                                int rbase, int cnt, uint32_t (&acc)[OPW][8]) {
    for (int jj = 0; jj < jn; jj++) {
        uint32_t y[8];
#pragma unroll
        for (int p = 0; p < 8; p++) y[p] = lds[(jj * 8 + p) * 64 + lane];
        const uint8_t *cp = a.coef + (int64_t)(jbase + jj) * a.coef_ld + rbase;
        uint32_t cw[(OPW + 3) / 4];
#pragma unroll
        for (int q = 0; q < (OPW + 3) / 4; q++)
            cw[q] = __builtin_amdgcn_readfirstlane(*(const uint32_t *)(cp + 4 * q));
        static_for<4>([&]<int G>() {
            uint32_t z[8];
            mul2_planes(y, z);
            static_for<OPW>([&]<int O>() {
                if (O < cnt) add_bit_pair<8 * (O % 4) + 2 * G>(acc[O], y, z, cw[O / 4]);
            });
            if constexpr (G < 3) mul2_planes(z, y);
        });
    }
}

}  // namespace dev
}  // namespace uplink_ec
