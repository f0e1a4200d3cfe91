// Compile-time-G encoder kernel (K1 in SURVEY.md §2): every piece of whole
// segments, for one (k, n) fixed at compile time.
//
// Reproduces the per-piece, per-stripe loop of the reference
//   rsScheme.EncodeSingle / Encode  private/eestream/rs.go:21-30
//   driven by segmentupload/encode.go:39-75 (one reader per piece)
// for all n pieces of a tile of stripes at once.  Bit-sliced GF(2^8): a lane
// owns 32 byte columns as 8 bit planes (rs_tile.hpp); multiplying by the
// constant G[k+r][j] is an 8x8 GF(2) matrix on the planes, applied as one
// v_bitop3 per output plane that XORs a precomputed 4-plane combination of the
// low nibble with one of the high nibble ("four Russians").
//
// Warp-specialised: NC compute waves own the parity rows (rows_of); NL
// loader waves fetch the next work item's inputs (non-temporal 16-B loads),
// write the systematic data pieces straight from registers, bit-slice and
// fill the other slot of a 2-slot LDS ring.  A work item is a chunk of up to
// kMaxChunk input shares of one 2048-column tile, so any k fits the ring: the
// accumulators of a tile persist across its chunks and are stored after the
// last one.  One LDS-only barrier per item.
//
// Self-contained (no library headers): the same text is compiled into the
// library for the configurations in rs_encoder_registry.cpp and by hiprtc for
// any other (k, n) (rs_encoder_jit.cpp).
#pragma once
#include "gf256_field.hpp"
#include "rs_tile.hpp"

namespace uplink_ec {
namespace enc {

using namespace dev;

constexpr int kMaxChunk = 36;  // input shares per LDS slot: 2 slots x 36 x 2 KiB = 144 KiB
constexpr int chunks_of(int K) { return (K + kMaxChunk - 1) / kMaxChunk; }
constexpr int chunk_size(int K) { return (K + chunks_of(K) - 1) / chunks_of(K); }

// Parity rows of compute wave W of NC: R = N - K rows dealt as evenly as
// possible (the first R % NC waves take one more), so the two compute waves
// that share a SIMD in the 8-wave form carry 12-13 rows each for RS(29,80)
// instead of 14 and 9.
constexpr int rows_of(int R, int NC, int W) { return R / NC + (W < R % NC ? 1 : 0); }
constexpr int rbase_of(int R, int NC, int W) { return W * (R / NC) + (W < R % NC ? W : R % NC); }

// acc[O] ^= G[K + rbase + O][J] * x_J for the wave's rows and the inputs
// J0 .. J0+JN-1, whose bit planes sit in lds at slot J - J0.
template <int K, int N, int NC, int OPW, int W, int J0, int JN>
__device__ __forceinline__ void compute_chunk(const uint32_t *lds, int lane, uint32_t (&acc)[OPW][8]) {
    static_for<JN>([&]<int JJ>() {
        constexpr int J = J0 + JJ;
        uint32_t x[8];
        static_for<8>([&]<int P>() { x[P] = lds[(JJ * 8 + P) * 64 + lane]; });
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
            constexpr int r = rbase_of(N - K, NC, W) + O;
            if constexpr (O < rows_of(N - K, NC, W)) {
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

// Tile t for the n-th fetch of this workgroup: from the launch's work queue
// (a.queue, zeroed before the launch) or, without one, statically.  Only one
// lane calls it; a returning vector atomic, not a scalar one.
__device__ __forceinline__ int32_t take_tile(const RsArgs &a, int n) {
    if (a.queue) return (int32_t)atomicAdd(a.queue, 1u);
    return (int32_t)(blockIdx.x + (int64_t)n * gridDim.x);
}

template <int K, int N, int NC, int NL>
__global__ __launch_bounds__((NC + NL) * 64, 1) void rs_encode_special(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NC - 1) / NC;
    constexpr int NCH = chunks_of(K), KC = chunk_size(K);
    constexpr int PER = (KC + NL - 1) / NL;
    __shared__ uint32_t lds[2][KC * 8 * 64];
    __shared__ int32_t s_q[4];  // tiles taken from the queue, in order (ring)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NC;
    const int lw = wave - NC;
    // lane 0 of the first loader wave takes the tiles; the others learn them
    // from s_q after the next barrier
    const bool taker = wave == NC && lane == 0;
    const int64_t P = pair_count(a);
    auto stage = [&](int64_t t, int ch, uint32_t *slot) {
        const TileCols c = pair_cols(a, t, lane);
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
        stage_inputs<NL, PER, true>(a, 0, c, slot, lane, lw, j0, jn, true);
    };
    if (taker) {
        s_q[0] = take_tile(a, 0);
        s_q[1] = take_tile(a, 1);
    }
    lds_barrier();
    int64_t tile = s_q[0];  // tile of the item being computed
    int64_t q1 = s_q[1];    // the tile to start after it
    int taken = 2;
    int ch = 0;
    if (loader && tile < P) stage(tile, 0, lds[0]);
    lds_barrier();
    int buf = 0;
    uint32_t acc[OPW][8];
    while (tile < P) {
        int64_t ntile = tile;
        int nch = ch + 1;
        bool take = false;
        if (nch == NCH) {
            nch = 0;
            ntile = q1;
            take = ntile < P;  // q1 is consumed: take its successor (needed one item later)
        }
        if (loader) {
            int32_t got = 0;
            if (take && taker) got = take_tile(a, taken);  // issued before the loads, its result waited on after them
            if (ntile < P) stage(ntile, nch, lds[buf ^ 1]);
            if (take && taker) s_q[taken & 3] = got;
        } else {
            if (ch == 0) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = 0;
            }
            static_for<NCH>([&]<int C>() {
                if (ch == C) {
                    constexpr int J0 = C * KC, JN = K - J0 < KC ? K - J0 : KC;
                    static_for<NC>([&]<int W>() {
                        if (wave == W) compute_chunk<K, N, NC, OPW, W, J0, JN>(lds[buf], lane, acc);
                    });
                }
            });
            if (ch == NCH - 1) {
                const TileCols c = pair_cols(a, tile, lane);
                const int rbase = rbase_of(R, NC, wave), cnt = rows_of(R, NC, wave);
                store_rows<OPW, true>(a, 0, c, rbase, cnt, acc);
            }
        }
        lds_barrier();
        if (take) q1 = s_q[taken & 3], taken++;
        buf ^= 1;
        tile = ntile;
        ch = nch;
    }
}

// Limits of the compile-time encoder: 1 <= n - k <= 96 parity rows (24
// accumulator rows per compute wave), k <= kMaxOps inputs.
constexpr bool supported(int k, int n) { return k >= 1 && k <= kMaxOps && n - k >= 1 && n - k <= 96; }
// Compute waves of the parity-only variant: with no data pieces to write the
// loaders have less to do and one compute wave per SIMD, issuing at half rate
// on its own, is the limit: 8 + 4 waves once there are >= 32 parity rows
// (DESIGN.md §4).
constexpr int parity_compute_waves(int k, int n) { return n - k >= 32 ? 8 : 4; }
// Few parity rows (<= 32) for many chunk inputs (>= 16): the loaders' share
// of a tile (loads, data-piece stores, bit-slicing) is large next to the
// compute, and 8 loader waves carrying half as many inputs each are faster
// (RS(30,60) 6 %, RS(20,50) 3.5 %; with 40 or 51 parity rows 4 loaders stay
// ahead: DESIGN.md §4 "Encode kernel").
constexpr bool few_rows_many_inputs(int k, int n) { return n - k <= 32 && chunk_size(k) >= 16; }
// Compute waves of the full encode: 4, one per SIMD beside a loader wave,
// while a wave's rows fit its registers next to the loaders' (<= 13 rows:
// RS(29,80) runs at 198 VGPRs, two waves per SIMD); more parity rows would
// spill (RS(10,100) at 23 rows per wave: 120 B per lane to scratch), so
// 8 compute waves then.  A two-chunk tile with few rows and 8 loaders also
// takes 8 (RS(50,80): 4 + 8 spills, 8 + 8 is 4 % faster than 4 + 4).
constexpr int full_compute_waves(int k, int n) {
    return n - k > 52 || (few_rows_many_inputs(k, n) && chunks_of(k) > 1) ? 8 : 4;
}
constexpr int full_loader_waves(int k, int n) { return few_rows_many_inputs(k, n) ? 8 : 4; }
// Workgroups per CU: two when both LDS rings fit (<= 80 KiB each) and the
// two workgroups' waves fit the CU's 16 slots of this occupancy.
constexpr int wgs_per_cu(int k, int waves) {
    return 2 * chunk_size(k) * 2048 * 2 <= 160 * 1024 && 2 * waves <= 16 ? 2 : 1;
}

}  // namespace enc
}  // namespace uplink_ec
