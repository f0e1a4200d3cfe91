// Developer experiment (not product): timing variants of the RS(29,80)
// encode kernel to locate its bottleneck.  Build: make -C tools/exp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../uplink_amd/csrc/rs_device.hpp"

using namespace uplink_ec;
using namespace uplink_ec::dev;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// MODE 0 normal, 1 all waves run group 0 code, 2 no XOR compute, 3 copy only (no LDS, no transposes)
template <int K, int N, int NW, int MODE>
__global__ __launch_bounds__(NW * 64, 2) void enc_var(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NW - 1) / NW;
    constexpr int PER = (K + NW - 1) / NW;
    __shared__ uint32_t lds[K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const int64_t tt = tile - seg * a.tiles_per_seg;
        const TileCols c = tile_cols(a, tt, lane);
        if constexpr (MODE == 3) {
            uint4 bufA[PER], bufB[PER];
            const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (j < K) {
                    const uint8_t *p = in_seg + a.in_off[j];
                    bufA[i] = c.vA ? *(const uint4 *)(p + c.inA) : make_uint4(0, 0, 0, 0);
                    bufB[i] = c.vB ? *(const uint4 *)(p + c.inB) : make_uint4(0, 0, 0, 0);
                }
            }
            uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (j < K) {
                    uint8_t *p = out_seg + a.copy_off[j];
                    if (c.vA) *(uint4 *)(p + c.outA) = bufA[i];
                    if (c.vB) *(uint4 *)(p + c.outB) = bufB[i];
                }
            }
            const int rbase = wave * OPW;
            static_for<OPW>([&]<int O>() {
                if (rbase + O < R) {
                    uint8_t *p = out_seg + a.out_off[rbase + O];
                    if (c.vA) *(uint4 *)(p + c.outA) = bufA[O % PER];
                    if (c.vB) *(uint4 *)(p + c.outB) = bufB[O % PER];
                }
            });
            continue;
        } else {
            stage_inputs<NW, PER>(a, seg, c, lds, lane, wave, 0, K, true);
            __syncthreads();
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            if constexpr (MODE == 0) {
                static_for<NW>([&]<int W>() {
                    if (wave == W) compute_special<K, N, OPW, W>(lds, lane, acc);
                });
            } else if constexpr (MODE == 1) {
                compute_special<K, N, OPW, 0>(lds, lane, acc);
            } else {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = lds[((o % K) * 8 + p) * 64 + lane];
            }
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            store_rows<OPW>(a, seg, c, rbase, cnt, acc);
            __syncthreads();
        }
    }
}


// warp-specialised: waves 0..3 compute (rows), waves 4..7 load/transpose into a
// double-buffered LDS tile ring; one barrier per tile.

// I-cache probe: the body of input 0 (compile-time coefficients) executed in a
// runtime loop over all K inputs (same VALU mix, 1/K of the code; wrong output)
template <int K, int N, int OPW, int W>
__device__ __forceinline__ void compute_looped(const uint32_t *lds, int lane, uint32_t (&acc)[OPW][8]) {
#pragma unroll 1
    for (int jr = 0; jr < K; jr++) {
        uint32_t x[8];
#pragma unroll
        for (int p = 0; p < 8; p++) x[p] = lds[(jr * 8 + p) * 64 + lane];
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
                constexpr uint8_t cval = gen_entry(K, K + r, (O * 7 + W) % K);
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
    }
}

template <int K, int N, bool NT, bool NTL = false, bool RAW = false, bool SAME = false, int PROBE = 0>
__global__ __launch_bounds__(512, 1) void enc_ws(const RsArgs a) {
    constexpr int NWC = 4;
    constexpr int R = N - K;
    constexpr int OPW = (R + NWC - 1) / NWC;
    constexpr int PER = (K + 3) / 4;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NWC;
    const int lw = wave - NWC;
    int64_t tile = blockIdx.x;
    if (loader && tile < a.total_tiles) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        stage_inputs<4, PER, NTL>(a, seg, c, lds[0], lane, lw, 0, K, true);
    }
    __syncthreads();
    int buf = 0;
    for (; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t next = tile + gridDim.x;
        if (loader) {
            if (next < a.total_tiles && PROBE != 1) {
                const int64_t seg = next / a.tiles_per_seg;
                const TileCols c = tile_cols(a, next - seg * a.tiles_per_seg, lane);
                stage_inputs<4, PER, NTL>(a, seg, c, lds[buf ^ 1], lane, lw, 0, K, true);
            }
        } else {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            if constexpr (PROBE == 2) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = lds[buf][((o % K) * 8 + p) * 64 + lane];
            } else {
            static_for<NWC>([&]<int W>() {
                if (wave == W) {
                    if constexpr (SAME) compute_looped<K, N, OPW, W>(lds[buf], lane, acc);
                    else compute_special<K, N, OPW, W>(lds[buf], lane, acc);
                }
            });
            }
            if constexpr (PROBE == 1) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) asm volatile("" ::"v"(acc[o][p]));
                if (RAW) lds_barrier(); else __syncthreads();
                buf ^= 1;
                continue;
            }
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            if constexpr (NT) {
                uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
                static_for<OPW>([&]<int O>() {
                    if (O < cnt) {
                        uint32_t w[8];
#pragma unroll
                        for (int p = 0; p < 8; p++) w[p] = acc[O][p];
                        unbitslice8(w);
                        uint8_t *p = out_seg + a.out_off[rbase + O];
                        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                        if (c.vA) __builtin_nontemporal_store((v4){w[0], w[1], w[2], w[3]}, (v4 *)(p + c.outA));
                        if (c.vB) __builtin_nontemporal_store((v4){w[4], w[5], w[6], w[7]}, (v4 *)(p + c.outB));
                    }
                });
            } else {
                store_rows<OPW>(a, seg, c, rbase, cnt, acc);
            }
        }
        if constexpr (RAW) lds_barrier(); else __syncthreads();
        buf ^= 1;
    }
}

__global__ void copy4_kernel(const uint4 *in, uint4 *out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        uint4 a0 = in[i], a1 = in[i + stride], a2 = in[i + 2 * stride], a3 = in[i + 3 * stride];
        out[i] = a0; out[i + stride] = a1; out[i + 2 * stride] = a2; out[i + 3 * stride] = a3;
    }
    for (; i < n; i += stride) out[i] = in[i];
}


// warp-specialised with the loaders' global loads issued one tile further
// ahead (register double buffer): loads of tile i+2 are in flight while the
// planes of tile i+1 are written to LDS and compute runs on tile i.
template <int K, int N, int PF, int NWC = 4>
__global__ __launch_bounds__((NWC + 4) * 64, 1) void enc_ws_pf(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NWC - 1) / NWC;
    constexpr int PER = (K + 3) / 4;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NWC;
    const int lw = wave - NWC;
    uint4 bA[PER], bB[PER];
    auto issue = [&](int64_t t) {
        if (t >= a.total_tiles) return;
        const int64_t seg = t / a.tiles_per_seg;
        const TileCols c = tile_cols(a, t - seg * a.tiles_per_seg, lane);
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + 4 * i;
            if (j < K) {
                const uint8_t *p = in_seg + a.in_off[j];
                bA[i] = c.vA ? ld16<true>(p + c.inA) : make_uint4(0, 0, 0, 0);
                bB[i] = c.vB ? ld16<true>(p + c.inB) : make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto consume = [&](int64_t t, uint32_t *dst_lds) {
        if (t >= a.total_tiles) return;
        const int64_t seg = t / a.tiles_per_seg;
        const TileCols c = tile_cols(a, t - seg * a.tiles_per_seg, lane);
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + 4 * i;
            if (j < K) {
                uint8_t *p = out_seg + a.copy_off[j];
                if (c.vA) st16<true>(p + c.outA, bA[i].x, bA[i].y, bA[i].z, bA[i].w);
                if (c.vB) st16<true>(p + c.outB, bB[i].x, bB[i].y, bB[i].z, bB[i].w);
                uint32_t w[8] = {bA[i].x, bA[i].y, bA[i].z, bA[i].w, bB[i].x, bB[i].y, bB[i].z, bB[i].w};
                bitslice8(w);
                uint32_t *d = dst_lds + j * 8 * 64 + lane;
#pragma unroll
                for (int p2 = 0; p2 < 8; p2++) d[p2 * 64] = w[p2];
            }
        }
    };
    int64_t tile = blockIdx.x;
    const int64_t G = gridDim.x;
    if (loader) {
        // loader role: its own loop, same number of barriers as the compute role
        issue(tile);
        consume(tile, lds[0]);
        if (PF) issue(tile + G);
        lds_barrier();
        int buf = 0;
        for (; tile < a.total_tiles; tile += G) {
            if (PF) {
                consume(tile + G, lds[buf ^ 1]);
                issue(tile + 2 * G);
            } else {
                issue(tile + G);
                consume(tile + G, lds[buf ^ 1]);
            }
            lds_barrier();
            buf ^= 1;
        }
    } else {
        lds_barrier();
        int buf = 0;
        for (; tile < a.total_tiles; tile += G) {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            static_for<NWC>([&]<int W>() {
                if (wave == W) compute_special<K, N, OPW, W>(lds[buf], lane, acc);
            });
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            store_rows<OPW, true>(a, seg, c, rbase, cnt, acc);
            lds_barrier();
            buf ^= 1;
        }
    }
}


// register-resident: every wave owns a whole tile (2048 columns); the k
// input shares' bit planes live in VGPRs (8k registers), the parity rows are
// produced in groups of OG rows; all waves execute the same instruction
// stream (I-cache shared), no LDS, no barriers.
template <int K, int N, int OG>
__device__ __forceinline__ void reg_group(const uint32_t (&x)[K][8], uint32_t (&acc)[OG][8], auto rowidx) {
}

template <int K, int N, int OG, int G0>
__device__ __forceinline__ void compute_group_regs(const uint32_t (&x)[K][8], uint32_t (&acc)[OG][8]) {
    static_for<K>([&]<int J>() {
        uint32_t lo[16], hi[16];
        lo[0] = 0;
        hi[0] = 0;
        static_for<15>([&]<int M1>() {
            constexpr int M = M1 + 1;
            constexpr int low = M & (-M);
            constexpr int bit = low == 1 ? 0 : low == 2 ? 1 : low == 4 ? 2 : 3;
            if constexpr (M == low) {
                lo[M] = x[J][bit];
                hi[M] = x[J][4 + bit];
            } else {
                lo[M] = lo[M ^ low] ^ x[J][bit];
                hi[M] = hi[M ^ low] ^ x[J][4 + bit];
            }
        });
        static_for<OG>([&]<int O>() {
            constexpr int r = G0 + O;
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

template <int K, int N, int OG>
__global__ __launch_bounds__(256, 1) void enc_reg(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int NG = (R + OG - 1) / OG;
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t tile = gw; tile < a.total_tiles; tile += nw) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
        uint32_t x[K][8];
        static_for<K>([&]<int J>() {
            const uint8_t *p = in_seg + a.in_off[J];
            const uint4 A = c.vA ? ld16<true>(p + c.inA) : make_uint4(0, 0, 0, 0);
            const uint4 B = c.vB ? ld16<true>(p + c.inB) : make_uint4(0, 0, 0, 0);
            uint8_t *q = out_seg + a.copy_off[J];
            if (c.vA) st16<true>(q + c.outA, A.x, A.y, A.z, A.w);
            if (c.vB) st16<true>(q + c.outB, B.x, B.y, B.z, B.w);
            uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
            bitslice8(w);
#pragma unroll
            for (int p2 = 0; p2 < 8; p2++) x[J][p2] = w[p2];
        });
        static_for<NG>([&]<int G>() {
            uint32_t acc[OG][8];
#pragma unroll
            for (int o = 0; o < OG; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            compute_group_regs<K, N, OG, G * OG>(x, acc);
            const int cnt = R - G * OG < OG ? R - G * OG : OG;
            store_rows<OG, true>(a, seg, c, G * OG, cnt, acc);
        });
    }
}



// software-pipelined, no role split: every wave (NW of them) prefetches its
// share of tile i+1's inputs into registers, computes its rows of tile i
// from LDS, then bit-slices the prefetched inputs into the other LDS slot.
template <int K, int N, int NW, int PROBE = 0>
__global__ __launch_bounds__(NW * 64, 1) void enc_sp(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NW - 1) / NW;
    constexpr int PER = (K + NW - 1) / NW;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 bA[PER], bB[PER];
    auto issue = [&](int64_t t) {
        const int64_t seg = t / a.tiles_per_seg;
        const TileCols c = tile_cols(a, t - seg * a.tiles_per_seg, lane);
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = wave + NW * i;
            if (j < K) {
                const uint8_t *p = in_seg + a.in_off[j];
                bA[i] = c.vA ? ld16<true>(p + c.inA) : make_uint4(0, 0, 0, 0);
                bB[i] = c.vB ? ld16<true>(p + c.inB) : make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto consume = [&](int64_t t, uint32_t *dst_lds) {
        const int64_t seg = t / a.tiles_per_seg;
        const TileCols c = tile_cols(a, t - seg * a.tiles_per_seg, lane);
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = wave + NW * i;
            if (j < K) {
                if (PROBE != 1) {
                    uint8_t *p = out_seg + a.copy_off[j];
                    if (c.vA) st16<true>(p + c.outA, bA[i].x, bA[i].y, bA[i].z, bA[i].w);
                    if (c.vB) st16<true>(p + c.outB, bB[i].x, bB[i].y, bB[i].z, bB[i].w);
                }
                uint32_t w[8] = {bA[i].x, bA[i].y, bA[i].z, bA[i].w, bB[i].x, bB[i].y, bB[i].z, bB[i].w};
                bitslice8(w);
                uint32_t *d = dst_lds + j * 8 * 64 + lane;
#pragma unroll
                for (int p2 = 0; p2 < 8; p2++) d[p2 * 64] = w[p2];
            }
        }
    };
    int64_t tile = blockIdx.x;
    const int64_t G = gridDim.x;
    if (tile < a.total_tiles) {
        if (PROBE != 1) issue(tile);
        consume(tile, lds[0]);
    }
    lds_barrier();
    int buf = 0;
    for (; tile < a.total_tiles; tile += G) {
        const int64_t next = tile + G;
        if (next < a.total_tiles && PROBE != 1) issue(next);
        {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            if constexpr (PROBE == 2) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = lds[buf][((o % K) * 8 + p) * 64 + lane];
            } else {
                static_for<NW>([&]<int W>() {
                    if (wave == W) compute_special<K, N, OPW, W>(lds[buf], lane, acc);
                });
            }
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            if (PROBE == 1) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) asm volatile("" ::"v"(acc[o][p]));
            } else {
                store_rows<OPW, true>(a, seg, c, rbase, cnt, acc);
            }
        }
        if (next < a.total_tiles) consume(next, lds[buf ^ 1]);
        lds_barrier();
        buf ^= 1;
    }
}

__global__ void fanout3_kernel(const uint4 *in, uint4 *o1, uint4 *o2, uint4 *o3, int64_t n, int nt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint4 v;
        if (nt) {
            typedef uint32_t v4 __attribute__((ext_vector_type(4)));
            v4 t = __builtin_nontemporal_load((const v4 *)(in + i));
            __builtin_nontemporal_store(t, (v4 *)(o1 + i));
            __builtin_nontemporal_store(t, (v4 *)(o2 + i));
            __builtin_nontemporal_store(t, (v4 *)(o3 + i));
        } else {
            v = in[i];
            o1[i] = v; o2[i] = v; o3[i] = v;
        }
    }
}

__global__ void copy_kernel(const uint4 *in, uint4 *out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0;
    const int k = 29, n = 80, ess = 256, nstripes = 9040, nseg = 8;
    const int64_t spad = (int64_t)nstripes * k * ess, plen = (int64_t)nstripes * ess;
    uint8_t *segs, *pieces;
    CK(hipMalloc(&segs, spad * nseg));
    CK(hipMalloc(&pieces, plen * n * nseg));
    std::vector<uint8_t> h(spad * nseg);
    for (auto &x : h) x = rand();
    CK(hipMemcpy(segs, h.data(), h.size(), hipMemcpyHostToDevice));
    RsArgs a{};
    a.in_base = segs; a.out_base = pieces;
    a.in_stripe_stride = k * ess; a.out_stripe_stride = ess;
    a.in_seg_stride = spad; a.out_seg_stride = plen * n;
    a.nin = k; a.nout = n - k;
    for (int j = 0; j < k; j++) { a.in_off[j] = (int64_t)j * ess; a.copy_off[j] = (int64_t)j * plen; }
    for (int r = 0; r < n - k; r++) a.out_off[r] = (int64_t)(k + r) * plen;
    a.ess = ess; a.cps = ess / 16; a.nstripes = nstripes;
    a.chunks_per_seg = (int64_t)nstripes * (ess / 16);
    a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
    a.total_tiles = a.tiles_per_seg * nseg;
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = (double)spad * nseg * (1.0 + (double)n / k);
    auto timeit = [&](const char *name, auto launch) {
        if (only >= 0 && vidx++ != only) return;
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-34s %9.1f us/8seg  %7.1f us/seg  %6.2f TB/s alg\n", name, us, us / nseg, bytes / us / 1e6);
        fflush(stdout);
    };
    const int grid2 = (int)std::min<int64_t>(a.total_tiles, (int64_t)cus * 2);
    {
        const int grid = (int)std::min<int64_t>(a.total_tiles, (int64_t)cus);
        for (int rep = 0; rep < 1; rep++) {
            timeit("ws nt (product)", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, true, true>), dim3(grid), dim3(512), 0, 0, a); });
            timeit("PROBE compute only (no HBM)", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, true, true, false, 1>), dim3(grid), dim3(512), 0, 0, a); });
            timeit("PROBE memory only (no XOR)", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, true, true, false, 2>), dim3(grid), dim3(512), 0, 0, a); });
        }
    }
    // plain copy of the same byte count (read spad*(1) write spad*(n/k)) approximated by read+write of equal halves
    const int64_t n16 = (int64_t)(bytes / 2) / 16;
    uint4 *cbuf; CK(hipMalloc(&cbuf, n16 * 16 * 2));
    for (int g : {4})
        for (int u : {1}) {
            char nm[64];
            snprintf(nm, 64, "copy unroll%d grid=%dx (same bytes)", u, g);
            if (u == 1) timeit(nm, [&] { hipLaunchKernelGGL(copy_kernel, dim3(cus * g), dim3(256), 0, 0, cbuf, cbuf + n16, n16); });
            else timeit(nm, [&] { hipLaunchKernelGGL(copy4_kernel, dim3(cus * g), dim3(256), 0, 0, cbuf, cbuf + n16, n16); });
        }
    {
        // same byte count as one encode launch, 1 read : 3 writes (encode is 1 : 2.76)
        const int64_t nr = (int64_t)(bytes / 4) / 16;
        uint4 *fb; CK(hipMalloc(&fb, nr * 16 * 4));
        for (int g : {2})
            for (int nt : {0}) {
                char nm[64];
                snprintf(nm, 64, "fanout 1r:3w grid=%dx nt=%d", g, nt);
                timeit(nm, [&] { hipLaunchKernelGGL(fanout3_kernel, dim3(cus * g), dim3(256), 0, 0, fb, fb + nr, fb + 2 * nr, fb + 3 * nr, nr, nt); });
            }
    }
    return 0;
}
