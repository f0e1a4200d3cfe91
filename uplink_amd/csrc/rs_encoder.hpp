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
// One workgroup per CU, its tiles taken from the launch's work queue
// (take_tile); a tile is two 1-KiB column blocks half a batch apart
// (rs_tile.hpp pair_cols), a work item one chunk of its input shares.
// Warp-specialised around a 2-slot LDS ring: while the NC compute waves (two
// per SIMD) multiply item i, the NL loader waves bring item i+1 into the
// other slot raw by LDS-DMA (no registers held for the loads) and turn it
// into bit planes in place, writing the systematic data pieces on the way.
// One LDS-only barrier per item.  DESIGN.md §4 "Encode kernel".
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

constexpr int kSlots = 2;      // LDS ring: item i multiplied while item i+1 arrives and is bit-sliced
constexpr int kMaxChunk = 36;  // input shares per slot: 2 slots x 36 x 2 KiB = 144 KiB
constexpr int chunks_of(int K) { return (K + kMaxChunk - 1) / kMaxChunk; }
constexpr int chunk_size(int K) { return (K + chunks_of(K) - 1) / chunks_of(K); }

// Parity rows of compute wave W of NC: R = N - K rows dealt as evenly as
// possible (the first R % NC waves take one more).
constexpr int rows_of(int R, int NC, int W) { return R / NC + (W < R % NC ? 1 : 0); }
constexpr int rbase_of(int R, int NC, int W) { return W * (R / NC) + (W < R % NC ? W : R % NC); }

// acc[O] ^= G[K + rbase + O][J] * x_J for the wave's rows and the inputs
// J0 .. J0+JN-1, whose bit planes sit at slot position J - J0 (planes 0-3 of a
// lane as one 16-byte word at 16 lane, planes 4-7 at 1024 + 16 lane).
template <int K, int N, int NC, int OPW, int W, int J0, int JN>
__device__ __forceinline__ void compute_chunk(const u32x4 *slot, int lane, uint32_t (&acc)[OPW][8]) {
    // The plane reads are the same in every wave's arm of the caller's switch;
    // an offset the compiler cannot see through keeps it from hoisting them out
    // of the arms (all of a chunk's planes live at once would spill).  One
    // input's planes are read ahead of its multiply.
    uint32_t opq = 0;
    asm volatile("" : "+s"(opq));
    slot += opq;
    u32x4 nlo = slot[lane], nhi = slot[64 + lane];
    static_for<JN>([&]<int JJ>() {
        constexpr int J = J0 + JJ;
        const u32x4 lo4 = nlo, hi4 = nhi;
        if constexpr (JJ + 1 < JN) {
            nlo = slot[(JJ + 1) * 128 + lane];
            nhi = slot[(JJ + 1) * 128 + 64 + lane];
        }
        asm volatile("" ::: "memory");
        const uint32_t x[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
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

// Tile for the m-th take of this workgroup: from the launch's work queue
// (a.queue, zeroed before the launch) or, without one, statically.  Only one
// lane calls it; a returning vector atomic, not a scalar one.
__device__ __forceinline__ int32_t take_tile(const RsArgs &a, int m) {
    if (a.queue) return (int32_t)atomicAdd(a.queue, 1u);
    return (int32_t)(blockIdx.x + (int64_t)m * gridDim.x);
}

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

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 16].
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define UPLINK_WAIT_VM(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        UPLINK_WAIT_VM(1) UPLINK_WAIT_VM(2) UPLINK_WAIT_VM(3) UPLINK_WAIT_VM(4) UPLINK_WAIT_VM(5) UPLINK_WAIT_VM(6)
        UPLINK_WAIT_VM(7) UPLINK_WAIT_VM(8) UPLINK_WAIT_VM(9) UPLINK_WAIT_VM(10) UPLINK_WAIT_VM(11) UPLINK_WAIT_VM(12)
        UPLINK_WAIT_VM(13) UPLINK_WAIT_VM(14) UPLINK_WAIT_VM(15) UPLINK_WAIT_VM(16)
#undef UPLINK_WAIT_VM
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

template <int K, int N, int NC, int NL>
__global__ __launch_bounds__((NC + NL) * 64, 1) void rs_encode_special(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NC - 1) / NC;
    constexpr int NCH = chunks_of(K), KC = chunk_size(K);
    constexpr int PER = (KC + NL - 1) / NL;
    static_assert(2 * PER <= 63, "a loader's DMAs of one item must fit the vmcnt counter");
    constexpr int SLOT = KC * 2048;  // bytes
    // The first K0 tiles are taken before the loop; the loop takes tile m at
    // item m*NCH - 3 and publishes it one item later, before its first DMA at
    // item m*NCH - 1.
    constexpr int K0 = (3 + NCH - 1) / NCH;
    __shared__ __attribute__((aligned(16))) u32x4 ring[kSlots * SLOT / 16];
    __shared__ int32_t s_q[8];  // tile of the m-th take, at m & 7
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NC;
    const int lw = wave - NC;
    const bool taker = wave == NC && lane == 0;  // takes the tiles; the others read s_q after a barrier
    const bool do_copy = a.copy_off[0] >= 0;
    const int64_t P = pair_count(a);
    const uint32_t ring_addr = (uint32_t)(uint64_t)ring;  // LDS byte address (low bits of the generic pointer)

    // loader: LDS-DMA of this wave's inputs of item (t, ch) into slot sl; returns the DMAs issued
    auto issue = [&](int sl, int64_t t, int ch) {
        const TileCols c = pair_cols(a, t, lane);
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
        int n = 0;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + NL * i;
            if (j < jn) {
                // columns past the end of the batch read column 0 of the same share (their
                // planes are never stored)
                const uint8_t *p = a.in_base + a.in_off[j0 + j];
                const uint8_t *pa = p + (c.vA ? c.inA : 0), *pb = p + (c.vB ? c.inB : 0);
                if (!in_range(a, pa, false, 1)) pa = a.chk_in_lo;
                if (!in_range(a, pb, false, 1)) pb = a.chk_in_lo;
                const uint32_t d = __builtin_amdgcn_readfirstlane(ring_addr + (uint32_t)(sl * SLOT + j * 2048));
                dma_1k(pa, d);
                dma_1k(pb, d + 1024);
                n += 2;
            }
        }
        return n;
    };
    // loader: item (t, ch) in slot sl from raw bytes to bit planes, in place (each
    // lane rewrites its own 32 bytes); the systematic shares go to their data
    // pieces on the way
    auto slice = [&](int sl, int64_t t, int ch) {
        const TileCols c = pair_cols(a, t, lane);
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
        u32x4 *slot = ring + sl * (SLOT / 16);
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + NL * i;
            if (j < jn) {
                const u32x4 A = slot[j * 128 + lane], B = slot[j * 128 + 64 + lane];
                const int64_t co = a.copy_off[j0 + j];
                if (do_copy && co >= 0) {
                    uint8_t *p = a.out_base + co;
                    if (c.vA && in_range(a, p + c.outA, true, 2)) st16<true>(p + c.outA, A.x, A.y, A.z, A.w);
                    if (c.vB && in_range(a, p + c.outB, true, 2)) st16<true>(p + c.outB, B.x, B.y, B.z, B.w);
                }
                uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
                bitslice8(w);
                slot[j * 128 + lane] = (u32x4){w[0], w[1], w[2], w[3]};
                slot[j * 128 + 64 + lane] = (u32x4){w[4], w[5], w[6], w[7]};
            }
        }
    };
    auto tile_of = [&](int item) -> int64_t { return s_q[(item / NCH) & 7]; };

    if (taker)
#pragma unroll
        for (int m = 0; m < K0; m++) s_q[m] = take_tile(a, m);
    lds_barrier();
    if (loader) {
        const int64_t t0 = tile_of(0);
        if (t0 < P) {
            issue(0, t0, 0);
            wait_vm(0);
            slice(0, t0, 0);
        }
    }
    lds_barrier();
    uint32_t acc[OPW][8];
    int32_t pending = 0;  // the taker's last take, published one item later
    int pend_m = -1;
    for (int i = 0;; i++) {
        const int64_t ti = tile_of(i);
        if (ti >= P) break;
        const int ch = i % NCH;
        if (loader) {
            if (pend_m >= 0 && taker) s_q[pend_m & 7] = pending;
            const int64_t u1 = tile_of(i + 1);
            if (u1 < P) issue((i + 1) % kSlots, u1, (i + 1) % NCH);
            pend_m = -1;
            int took = 0;
            if ((i + 3) % NCH == 0 && (i + 3) / NCH >= K0) {
                pend_m = (i + 3) / NCH;
                if (taker) pending = take_tile(a, pend_m);
                took = wave == NC && a.queue ? 1 : 0;  // the taker's wave has its atomic in flight too
            }
            if (u1 < P) {
                wait_vm(took);  // item i+1 has landed
                slice((i + 1) % kSlots, u1, (i + 1) % NCH);
            }
        } else {
            if (ch == 0) {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = 0;
            }
            const u32x4 *slot = ring + (i % kSlots) * (SLOT / 16);
            static_for<NCH>([&]<int C>() {
                if (ch == C) {
                    constexpr int J0 = C * KC, JN = K - J0 < KC ? K - J0 : KC;
                    static_for<NC>([&]<int W>() {
                        if (wave == W) compute_chunk<K, N, NC, OPW, W, J0, JN>(slot, lane, acc);
                    });
                }
            });
            if (ch == NCH - 1) {
                const TileCols c = pair_cols(a, ti, lane);
                store_rows<OPW, true>(a, 0, c, rbase_of(R, NC, wave), rows_of(R, NC, wave), acc);
            }
        }
        lds_barrier();
    }
}

// Limits of the compile-time encoder: 1 <= n - k <= 96 parity rows (12
// accumulator rows per compute wave), k <= kMaxOps inputs.
constexpr bool supported(int k, int n) { return k >= 1 && k <= kMaxOps && n - k >= 1 && n - k <= 96; }
// Waves: 4 loaders and, from 16 parity rows on, 8 compute waves -- two per
// SIMD, so each issues VALU at the full rate (one wave alone on a SIMD issues
// every other cycle); the 4-plane combinations each compute wave rebuilds per
// input cost 14 % more VALU than with 4.
constexpr int compute_waves(int k, int n) { return n - k >= 16 ? 8 : 4; }
constexpr int loader_waves(int k, int n) { return 4; }
constexpr int parity_compute_waves(int k, int n) { return compute_waves(k, n); }
constexpr int full_compute_waves(int k, int n) { return compute_waves(k, n); }
constexpr int full_loader_waves(int k, int n) { return loader_waves(k, n); }
// One workgroup per CU: its ring takes up to 144 KiB of LDS.
constexpr int wgs_per_cu(int k, int waves) { return 1; }

}  // namespace enc
}  // namespace uplink_ec
