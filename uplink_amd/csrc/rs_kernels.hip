// GF(2^8) Reed-Solomon stripe kernels for MI355X (gfx950 / CDNA4).
//
// Reproduces, for whole segments at once, the per-stripe calls of the
// reference:
//   encode  rsScheme.EncodeSingle / Encode   private/eestream/rs.go:21-30
//           driven per piece per stripe by   segmentupload/encode.go:39-75
//   rebuild rsScheme.Rebuild                 private/eestream/rs.go:40-45
//           driven per stripe by             private/eestream/stripe.go:382-428
// The arithmetic itself (infectious addmul) is restated bit-sliced:
//
//  * A lane owns 32 byte columns (two 16-byte chunks of one share row) and
//    turns the 32 bytes into 8 bit planes (plane p, bit 8b+w = bit p of byte b
//    of word w) with a 3-stage swap-move network.
//  * Multiplication by a GF(2^8) constant is then an 8x8 GF(2) matrix on the
//    planes, i.e. pure VALU XORs (v_bitop3_b32 fuses three-input XORs) over
//    full 32-bit words: no table lookups, no MFMA (byte-field arithmetic).
//  * A workgroup stages the bit planes of all inputs of a 2048-column tile in
//    LDS once; its waves then compute disjoint groups of output rows from
//    them, so each input byte is read from HBM exactly once and every output
//    byte is written exactly once (all HBM traffic is the algorithmic bytes).
//  * Loads and stores are 16 B per lane; a wave instruction touches 1 KiB of
//    256-byte share rows (coalesced).
//
// Two bodies share that skeleton:
//  * rs_encode_special<K,N>: G is a compile-time constant (the same Lagrange
//    construction as infectious, gf256.hpp), and each output plane gets the
//    XOR of two precomputed 4-plane combinations ("four Russians"), one
//    v_bitop3 per (output plane, input share): 8 ops per GF multiply-add of a
//    32-byte column block instead of ~16 for the plain bit-matrix.
//  * rs_matmul_generic<OPW>: any runtime matrix (encode for arbitrary (k,n),
//    and the rebuild matrix (G_S)^-1 of a share set).  The input's multiples
//    x*2^b are formed once per input (21 XORs); each coefficient bit pair is
//    then a wave-uniform branch adding one or two of them.
#include <utility>

#include "gf256.hpp"
#include "rs_kernels.hpp"

namespace uplink_ec {
namespace {

template <typename F, int... I>
__device__ __forceinline__ void sf_impl(F &&f, std::integer_sequence<int, I...>) {
    (f.template operator()<I>(), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    sf_impl(f, std::make_integer_sequence<int, N>{});
}

__constant__ GfTables d_gf = make_gf_tables();

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
template <int NW, int PER>
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
            bufA[i] = c.vA ? *(const uint4 *)(p + c.inA) : z;
            bufB[i] = c.vB ? *(const uint4 *)(p + c.inB) : z;
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
                if (c.vA) *(uint4 *)(p + c.outA) = bufA[i];
                if (c.vB) *(uint4 *)(p + c.outB) = bufB[i];
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
template <int OPW>
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
            if (c.vA) *(uint4 *)(p + c.outA) = make_uint4(w[0], w[1], w[2], w[3]);
            if (c.vB) *(uint4 *)(p + c.outB) = make_uint4(w[4], w[5], w[6], w[7]);
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

template <int K, int N, int NW>
__global__ __launch_bounds__(NW * 64, 2) void rs_encode_special(const RsArgs a) {
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
        stage_inputs<NW, PER>(a, seg, c, lds, lane, wave, 0, K, true);
        __syncthreads();
        uint32_t acc[OPW][8];
#pragma unroll
        for (int o = 0; o < OPW; o++)
#pragma unroll
            for (int p = 0; p < 8; p++) acc[o][p] = 0;
        static_for<NW>([&]<int W>() {
            if (wave == W) compute_special<K, N, OPW, W>(lds, lane, acc);
        });
        const int rbase = wave * OPW;
        const int cnt = R - rbase < OPW ? R - rbase : OPW;
        store_rows<OPW>(a, seg, c, rbase, cnt, acc);
        __syncthreads();
    }
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

template <int OPW>
__device__ __forceinline__ void compute_generic(const RsArgs &a, const uint32_t *lds, int lane, int jbase, int jn,
                                                int rbase, int cnt, uint32_t (&acc)[OPW][8]) {
    for (int jj = 0; jj < jn; jj++) {
        uint32_t y[8][8];
#pragma unroll
        for (int p = 0; p < 8; p++) y[0][p] = lds[(jj * 8 + p) * 64 + lane];
#pragma unroll
        for (int b = 1; b < 8; b++) mul2_planes(y[b - 1], y[b]);
        const uint8_t *cp = a.coef + (int64_t)(jbase + jj) * a.coef_ld + rbase;
        static_for<OPW / 4>([&]<int Q>() {
            const uint32_t cw = __builtin_amdgcn_readfirstlane(*(const uint32_t *)(cp + 4 * Q));
            static_for<4>([&]<int B>() {
                constexpr int O = 4 * Q + B;
                if (O < cnt) {
                    const uint32_t cv = (cw >> (8 * B)) & 0xffu;
                    static_for<4>([&]<int G2>() {
                        const uint32_t two = (cv >> (2 * G2)) & 3u;
                        if (two == 3u) {
#pragma unroll
                            for (int p = 0; p < 8; p++)
                                acc[O][p] = __builtin_amdgcn_bitop3_b32(acc[O][p], y[2 * G2][p], y[2 * G2 + 1][p], 0x96);
                        } else if (two == 1u) {
#pragma unroll
                            for (int p = 0; p < 8; p++) acc[O][p] ^= y[2 * G2][p];
                        } else if (two == 2u) {
#pragma unroll
                            for (int p = 0; p < 8; p++) acc[O][p] ^= y[2 * G2 + 1][p];
                        }
                    });
                }
            });
        });
    }
}

constexpr int kGenericNW = 4;
constexpr int kGenericJC = 16;  // inputs staged per LDS chunk

template <int OPW>
__global__ __launch_bounds__(kGenericNW * 64) void rs_matmul_generic(const RsArgs a) {
    constexpr int NW = kGenericNW;
    constexpr int JC = kGenericJC;
    constexpr int PER = (JC + NW - 1) / NW;
    __shared__ uint32_t lds[JC * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rows_per_pass = NW * OPW;
    const int npass = (a.nout + rows_per_pass - 1) / rows_per_pass;
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const int64_t tt = tile - seg * a.tiles_per_seg;
        const TileCols c = tile_cols(a, tt, lane);
        for (int pass = 0; pass < (npass > 0 ? npass : 1); pass++) {
            const int rbase = pass * rows_per_pass + wave * OPW;
            int cnt = a.nout - rbase;
            cnt = cnt < 0 ? 0 : (cnt > OPW ? OPW : cnt);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            for (int j0 = 0; j0 < a.nin; j0 += JC) {
                const int jn = a.nin - j0 < JC ? a.nin - j0 : JC;
                stage_inputs<NW, PER>(a, seg, c, lds, lane, wave, j0, jn, pass == 0);
                __syncthreads();
                if (cnt > 0) compute_generic<OPW>(a, lds, lane, j0, jn, rbase, cnt, acc);
                __syncthreads();
            }
            store_rows<OPW>(a, seg, c, rbase, cnt, acc);
        }
    }
}

// ------------------------------------------------ byte-wise fallback
// Any ess / alignment: one thread per byte column, log/exp tables in LDS.
__global__ __launch_bounds__(256) void rs_matmul_bytes(const RsArgs a) {
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = d_gf.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = d_gf.log[i];
    __syncthreads();
    const int64_t cols = a.nstripes * a.ess;
    const int64_t total = cols * (a.total_tiles);  // total_tiles holds nseg for this kernel
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t seg = idx / cols;
        const int64_t col = idx - seg * cols;
        const int64_t s = col / a.ess, t = col - s * a.ess;
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
        for (int j = 0; j < a.nin; j++) {
            if (a.copy_off[j] >= 0)
                out_seg[a.copy_off[j] + s * a.out_stripe_stride + t] =
                    in_seg[a.in_off[j] + s * a.in_stripe_stride + t];
        }
        for (int r = 0; r < a.nout; r++) {
            uint8_t acc = 0;
            for (int j = 0; j < a.nin; j++) {
                const uint8_t x = in_seg[a.in_off[j] + s * a.in_stripe_stride + t];
                const uint8_t cv = a.coef[(int64_t)j * a.coef_ld + r];
                if (x && cv) acc ^= s_exp[s_log[x] + s_log[cv]];
            }
            out_seg[a.out_off[r] + s * a.out_stripe_stride + t] = acc;
        }
    }
}

}  // namespace
}  // namespace uplink_ec

// ------------------------------------------------ launch entry points
namespace uplink_ec {

namespace {
int g_cu_count = 0;
int cu_count() {
    if (g_cu_count == 0) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_cu_count = n;
        else
            g_cu_count = 256;
    }
    return g_cu_count;
}

template <int K, int N, int NW>
hipError_t launch_special_nw(const RsArgs &a, int grid, hipStream_t s) {
    if (grid <= 0) grid = default_grid(a.total_tiles, 2);
    hipLaunchKernelGGL((rs_encode_special<K, N, NW>), dim3(grid), dim3(NW * 64), 0, s, a);
    return hipGetLastError();
}
}  // namespace

int default_grid(int64_t total_tiles, int wgs_per_cu) {
    int64_t g = (int64_t)cu_count() * wgs_per_cu;
    if (total_tiles < g) g = total_tiles;
    return (int)(g > 0 ? g : 1);
}

bool have_special_encoder(int k, int n) {
    return (k == 29 && n == 80) || (k == 20 && n == 60) || (k == 4 && n == 10);
}

hipError_t launch_encode_special(int k, int n, const RsArgs &a, int grid, hipStream_t s) {
    if (k == 29 && n == 80) return launch_special_nw<29, 80, 4>(a, grid, s);
    if (k == 20 && n == 60) return launch_special_nw<20, 60, 4>(a, grid, s);
    if (k == 4 && n == 10) return launch_special_nw<4, 10, 4>(a, grid, s);
    return hipErrorInvalidValue;
}

hipError_t launch_matmul_generic(const RsArgs &a, int grid, hipStream_t s) {
    if (grid <= 0) grid = default_grid(a.total_tiles, 4);
    const dim3 block(kGenericNW * 64);
    if (a.nout <= kGenericNW * 4)
        hipLaunchKernelGGL(rs_matmul_generic<4>, dim3(grid), block, 0, s, a);
    else if (a.nout <= kGenericNW * 8)
        hipLaunchKernelGGL(rs_matmul_generic<8>, dim3(grid), block, 0, s, a);
    else
        hipLaunchKernelGGL(rs_matmul_generic<16>, dim3(grid), block, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_matmul_bytes(const RsArgs &a, hipStream_t s) {
    const int64_t total = a.nstripes * a.ess * a.total_tiles;
    int64_t blocks = (total + 255) / 256;
    const int64_t cap = (int64_t)cu_count() * 8;
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(rs_matmul_bytes, dim3((unsigned)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace uplink_ec
