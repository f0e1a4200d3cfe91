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
// (rs_tile.hpp pair_cols), a work item one chunk of its input shares (all
// of them up to k = 36).  Warp-specialised around an LDS ring (2 slots):
// while the NC compute waves (two per SIMD) multiply item i, the NL loader
// waves bring item i+1 in raw by LDS-DMA (no registers held for the loads)
// and turn it into bit planes in place, writing the systematic data pieces on
// the way.  One LDS-only barrier per item.  DESIGN.md §4 "Encode kernel".
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

// LDS ring of kSlots items.  While the compute waves multiply item i, the
// loaders bit-slice item i+1 and the LDS-DMA loads of items i+2 .. i+kAhead
// are in flight (kAhead = kSlots - 1).  The product runs 2 slots of whole
// tiles (all k inputs, up to 36: 2 x 58 KiB for k = 29): 3 or 4 slots need
// items of at most 15 inputs to fit the LDS, and measured slower (RS(29,80)
// 51.2-51.8 vs 48.5 us per segment, DESIGN.md §4 "Encode kernel").  -D
// overrides are for A/B builds (tools/exp/build_enc_variants.sh).
#ifndef UPLINK_ENC_SLOTS
#define UPLINK_ENC_SLOTS 2
#endif
#ifndef UPLINK_ENC_MAX_CHUNK
#define UPLINK_ENC_MAX_CHUNK 36
#endif
// compute waves (from 16 parity rows on), loader waves and workgroups per CU
#ifndef UPLINK_ENC_NC
#define UPLINK_ENC_NC 8
#endif
#ifndef UPLINK_ENC_PARITY_NL
#define UPLINK_ENC_PARITY_NL 4
#endif
#ifndef UPLINK_ENC_WGS
#define UPLINK_ENC_WGS 1
#endif
// The loaders issue an item's copy-through stores one item late: after the
// next item's LDS-DMAs instead of while slicing (the raw bytes kept in
// registers meanwhile), so the counted vmcnt wait for those DMAs does not
// also wait for the item's own stores.  0 = store while slicing (A/B builds).
#ifndef UPLINK_ENC_DEFER_COPY
#define UPLINK_ENC_DEFER_COPY 1
#endif
// Each compute wave stores up to this many of a tile's parity rows one 16-byte
// store at a time between the next tile's first inputs instead of in the
// burst at the tile's end (the rows kept in registers meanwhile).
#ifndef UPLINK_ENC_DEFER_ROWS
#define UPLINK_ENC_DEFER_ROWS 0
#endif
// The compute waves meet the item's barrier right after their last read of
// the slot and store the tile's parity rows after it (while the loaders issue
// the next item's LDS-DMAs), instead of storing first and then meeting it.
#ifndef UPLINK_ENC_LATE_STORES
#define UPLINK_ENC_LATE_STORES 0
#endif
constexpr int kSlots = UPLINK_ENC_SLOTS;
constexpr int kAhead = kSlots - 1;               // items between a load's issue and that item's multiply
constexpr int kMaxChunk = UPLINK_ENC_MAX_CHUNK;  // input shares per item
constexpr int chunks_of(int K) { return (K + kMaxChunk - 1) / kMaxChunk; }
constexpr int chunk_size(int K) { return (K + chunks_of(K) - 1) / chunks_of(K); }

// Parity rows of compute wave W of NC: R = N - K rows dealt as evenly as
// possible (the first R % NC waves take one more).
constexpr int rows_of(int R, int NC, int W) { return R / NC + (W < R % NC ? 1 : 0); }
constexpr int rbase_of(int R, int NC, int W) { return W * (R / NC) + (W < R % NC ? W : R % NC); }

// acc[O] ^= G[K + rbase + O][J] * x_J for the wave's rows and the inputs
// J0 .. J0+JN-1, whose bit planes sit at slot position J - J0 (planes 0-3 of a
// lane as one 16-byte word at 16 lane, planes 4-7 at 1024 + 16 lane).
template <int K, int N, int NC, int OPW, int W, int J0, int JN, int DIAG = 0, typename Hook>
__device__ __forceinline__ void compute_chunk(const u32x4 *slot, int lane, uint32_t (&acc)[OPW][8], Hook &&hook) {
    // The plane reads are the same in every wave's arm of the caller's switch;
    // an offset the compiler cannot see through keeps it from hoisting them out
    // of the arms (all of a chunk's planes live at once would spill).  One
    // input's planes are read ahead of its multiply.
    uint32_t opq = 0;
    asm volatile("" : "+s"(opq));
    slot += opq;
    u32x4 nlo = slot[lane], nhi = slot[64 + lane];
    // kDiagLdsCombos: the 30 combination planes of the next input, read ahead from the LDS
    constexpr bool kLdsCombos = (DIAG & 64) != 0;
    constexpr int kCbSpan = JN * 128 > 1024 ? JN * 128 - 512 : 1;
    [[maybe_unused]] u32x4 ncb[8];
    if constexpr (kLdsCombos)
#pragma unroll
        for (int q = 0; q < 8; q++) ncb[q] = slot[(q * 64) % (JN * 128) + lane];
    static_for<JN>([&]<int JJ>() {
        constexpr int J = J0 + JJ;
        const u32x4 lo4 = nlo, hi4 = nhi;
        [[maybe_unused]] u32x4 cb[8];
        if constexpr (kLdsCombos)
#pragma unroll
            for (int q = 0; q < 8; q++) cb[q] = ncb[q];
        if constexpr (JJ + 1 < JN) {
            nlo = slot[(JJ + 1) * 128 + lane];
            nhi = slot[(JJ + 1) * 128 + 64 + lane];
            if constexpr (kLdsCombos)
#pragma unroll
                for (int q = 0; q < 8; q++) ncb[q] = slot[((JJ + 1) * 512 % kCbSpan + q * 64) % (JN * 128) + lane];
        }
        asm volatile("" ::: "memory");
        const uint32_t x[8] = {lo4.x, lo4.y, lo4.z, lo4.w, hi4.x, hi4.y, hi4.z, hi4.w};
        if constexpr ((DIAG & 16) != 0) {  // kDiagNoRowOps
            asm volatile("" ::"v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]));
            // the rows stored are the chunk's last input (random bytes, as real parity is)
            if constexpr (JJ + 1 == JN)
                static_for<OPW>([&]<int O>() { static_for<8>([&]<int P>() { acc[O][P] = x[P]; }); });
            hook.template operator()<JJ>();
            return;
        }
        uint32_t lo[16], hi[16];
        lo[0] = 0;
        hi[0] = 0;
        if constexpr (kLdsCombos) {  // timing only: every entry from the LDS reads (values meaningless)
            static_for<15>([&]<int M1>() {
                constexpr int a = M1, b = M1 + 15;
                lo[M1 + 1] = cb[a / 4][a % 4];
                hi[M1 + 1] = cb[b / 4][b % 4];
            });
        } else
        static_for<15>([&]<int M1>() {
            constexpr int M = M1 + 1;
            constexpr int low = M & (-M);
            constexpr int bit = low == 1 ? 0 : low == 2 ? 1 : low == 4 ? 2 : 3;
            // (kDiagNoCombos: every entry a single plane; kDiagHalfCombos: so for the odd inputs)
            if constexpr (M == low || (DIAG & 8) != 0 || ((DIAG & 32) != 0 && (J & 1) != 0)) {
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
        hook.template operator()<JJ>();
    });
}

// Tile for the m-th take of this workgroup: from the launch's work queue
// (a.queue, zero when the launch starts) or, without one, statically.  Only
// one lane calls it; a returning vector atomic, not a scalar one.
__device__ __forceinline__ int32_t take_tile(const RsArgs &a, int m) {
    if (a.queue) return (int32_t)atomicAdd(a.queue, 1u);
    return (int32_t)(blockIdx.x + (int64_t)m * gridDim.x);
}

// Diagnostic forms of the encoder body (DIAG != 0), instantiated only by the
// measurement harness tools/exp/enc_diag.hip, never by the library:
//   kDiagStamp            wave 0 of every workgroup stamps s_memtime and
//                         s_memrealtime around its tile loop, and compute wave 0
//                         and loader wave 0 count the cycles they spend waiting
//                         (barriers; the loader's counted vmcnt waits), into
//                         a.diag[8 * blockIdx.x ..]; nothing else reads them
//   kDiagNoParityStores   the parity rows are computed (and un-bit-sliced) but
//                         handed to an empty asm that keeps them live, not stored
//   kDiagNoCopyStores     the same for the loaders' copy-through of the data pieces
//                         (their vmcnt waits then count no stores)
//   kDiagNoCombos         timing only: the 22 combination planes per input are
//                         not built (every combination reads a single plane)
//   kDiagNoRowOps         timing only: no multiply-add at all (the inputs' planes
//                         are read from the LDS and kept live; each row stored is
//                         the tile's last input); the library builds this form
//                         for RS(29,80) as its on-box ceiling (rs_encode_probe.hip)
//   kDiagHalfCombos       timing only: kDiagNoCombos for the odd inputs (what
//                         building each input's combinations in half the waves saves)
//   kDiagLdsCombos        timing only: the 30 combination planes of each input read
//                         from the LDS (8 ds_read_b128 per lane, one input ahead)
//                         instead of built (what publishing them once per tile would cost)
constexpr int kDiagStamp = 1, kDiagNoParityStores = 2, kDiagNoCopyStores = 4, kDiagNoCombos = 8, kDiagNoRowOps = 16,
              kDiagHalfCombos = 32, kDiagLdsCombos = 64;

__device__ __forceinline__ void sink16(uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    asm volatile("" ::"v"(x), "v"(y), "v"(z), "v"(w));
}

// COPY: the full encode (the systematic data pieces written too); false: the
// parity-only form (EC_FLAG_PARITY_ONLY), a kernel of its own name.
template <int K, int N, int NC, int NL, bool COPY, int DIAG>
__device__ __forceinline__ void encode_body(const RsArgs &a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NC - 1) / NC;
    constexpr int NCH = chunks_of(K), KC = chunk_size(K);
    constexpr int PER = (KC + NL - 1) / NL;
    constexpr int A = kAhead;
    // a loader waits with at most 2(A-1) items of its DMAs and copy-through stores issued after the awaited ones
    static_assert(4 * (A - 1) * PER <= 63 && 2 * (2 * A - 1) * PER <= 63 && A >= 1,
                  "a loader's VMEM ops in flight must fit the vmcnt counter");
    constexpr int SLOT = KC * 2048;  // bytes
    static_assert(kSlots * SLOT <= 150 * 1024, "LDS ring too large");
    // Tile m (items m*NCH ..) is taken by compute wave 0 at the start of item
    // m*NCH - A - 1 and published in s_q before that item's barrier, so the
    // loaders know it when they issue its first DMAs at item m*NCH - A.  The
    // first K0 tiles are taken before the loop.
    constexpr int K0 = (A + 1 + NCH - 1) / NCH;
    __shared__ __attribute__((aligned(16))) u32x4 ring[kSlots * SLOT / 16];
    __shared__ int32_t s_q[8];  // tile of the m-th take, at m & 7
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NC;
    const int lw = wave - NC;
    const bool taker = wave == 0 && lane == 0;
    constexpr bool do_copy = COPY;
    const int64_t P = pair_count(a);
    const uint32_t ring_addr = (uint32_t)(uint64_t)ring;  // LDS byte address (low bits of the generic pointer)

    // loader: its DMAs for an item of chunk ch (two per input share it owns); with
    // do_copy its slice issues as many copy-through stores
    auto ops_of = [&](int ch) -> int {
        const int jn = K - ch * KC < KC ? K - ch * KC : KC;
        return lw < jn ? 2 * ((jn - lw + NL - 1) / NL) : 0;
    };
#ifdef UPLINK_EC_CHECKED
    constexpr bool kCountStores = false;  // the checked build may skip a store: count none (waits longer, never shorter)
#else
    constexpr bool kCountStores = !(DIAG & kDiagNoCopyStores);
#endif
    // kDiagStamp: cycles this wave spent waiting, and the stamps around the loop
    [[maybe_unused]] uint64_t d_wait = 0, d_t0 = 0, d_r0 = 0;
    auto d_now = [&]() -> uint64_t {
        if constexpr ((DIAG & kDiagStamp) != 0) return __builtin_amdgcn_s_memtime();
        return 0;
    };
    // loader: LDS-DMA of this wave's inputs of item (t, ch) into slot sl
    auto issue = [&](int sl, int64_t t, int ch) {
        const TileCols c = pair_cols(a, t, lane);
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + NL * i;
            if (j < jn) {
                // columns past the end of the batch read column 0 of the same share (their
                // planes are never stored; their copy-through rewrites column 0 with itself)
                const uint8_t *p = a.in_base + a.in_off[j0 + j];
                const uint8_t *pa = p + (c.vA ? c.inA : 0), *pb = p + (c.vB ? c.inB : 0);
                if (!in_range(a, pa, false, 1)) pa = a.chk_in_lo;
                if (!in_range(a, pb, false, 1)) pb = a.chk_in_lo;
                const uint32_t d = __builtin_amdgcn_readfirstlane(ring_addr + (uint32_t)(sl * SLOT + j * 2048));
                dma_1k(pa, d);
                dma_1k(pb, d + 1024);
            }
        }
    };
    // loader: the copy-through stores of item (t, ch), the raw bytes of this
    // wave's inputs -- two stores per input on every lane, so the wave's count of
    // VMEM ops is exact (a lane past the end of the batch holds column 0 of its
    // share, which it stores to column 0 of that share's piece: the bytes already
    // there)
    auto copy_out = [&](int64_t t, int ch, const u32x4 *rA, const u32x4 *rB) {
        const TileCols c = pair_cols(a, t, lane);
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + NL * i;
            if (j < jn) {
                if constexpr ((DIAG & kDiagNoCopyStores) != 0) {
                    sink16(rA[i].x, rA[i].y, rA[i].z, rA[i].w);
                    sink16(rB[i].x, rB[i].y, rB[i].z, rB[i].w);
                } else {
                    uint8_t *p = a.out_base + a.copy_off[j0 + j];
                    uint8_t *qa = p + (c.vA ? c.outA : 0), *qb = p + (c.vB ? c.outB : 0);
                    if (in_range(a, qa, true, 2)) st16<true>(qa, rA[i].x, rA[i].y, rA[i].z, rA[i].w);
                    if (in_range(a, qb, true, 2)) st16<true>(qb, rB[i].x, rB[i].y, rB[i].z, rB[i].w);
                }
            }
        }
    };
    constexpr bool kDefer = do_copy && UPLINK_ENC_DEFER_COPY != 0;
    // loader: item (t, ch) in slot sl from raw bytes to bit planes, in place (each
    // lane rewrites its own 32 bytes); the systematic shares go to their data
    // pieces on the way -- or, kDefer, the raw bytes are kept in rA / rB for
    // their stores one item later (the loop below)
    auto slice = [&](int sl, int64_t t, int ch, u32x4 *rA, u32x4 *rB) {
        const int j0 = ch * KC, jn = K - j0 < KC ? K - j0 : KC;
        u32x4 *slot = ring + sl * (SLOT / 16);
#pragma unroll
        for (int i = 0; i < PER; i++) {
            const int j = lw + NL * i;
            if (j < jn) {
                const u32x4 A4 = slot[j * 128 + lane], B4 = slot[j * 128 + 64 + lane];
                if constexpr (kDefer) {
                    rA[i] = A4;
                    rB[i] = B4;
                } else if constexpr (do_copy) {
                    const TileCols c = pair_cols(a, t, lane);
                    if constexpr ((DIAG & kDiagNoCopyStores) != 0) {
                        sink16(A4.x, A4.y, A4.z, A4.w);
                        sink16(B4.x, B4.y, B4.z, B4.w);
                    } else {
                        uint8_t *p = a.out_base + a.copy_off[j0 + j];
                        uint8_t *qa = p + (c.vA ? c.outA : 0), *qb = p + (c.vB ? c.outB : 0);
                        if (in_range(a, qa, true, 2)) st16<true>(qa, A4.x, A4.y, A4.z, A4.w);
                        if (in_range(a, qb, true, 2)) st16<true>(qb, B4.x, B4.y, B4.z, B4.w);
                    }
                }
                uint32_t w[8] = {A4.x, A4.y, A4.z, A4.w, B4.x, B4.y, B4.z, B4.w};
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
    if constexpr ((DIAG & kDiagStamp) != 0) {
        d_t0 = __builtin_amdgcn_s_memtime();
        d_r0 = __builtin_amdgcn_s_memrealtime();
    }
    // kDiagStamp: a barrier, its wait counted
    auto barrier_w = [&]() {
        const uint64_t t = d_now();
        lds_barrier();
        if constexpr ((DIAG & kDiagStamp) != 0) d_wait += d_now() - t;
    };
    // kDiagStamp: the stamps of wave w (compute wave 0 at slots 0-3, loader wave 0 at 4-7)
    auto stamp_out = [&](int at) {
        if constexpr ((DIAG & kDiagStamp) != 0) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            if (lane == 0 && a.diag) {
                uint64_t *d = a.diag + 8 * (int64_t)blockIdx.x + at;
                d[0] = t1 - d_t0;
                d[1] = r1 - d_r0;
                d[2] = d_wait;
                d[3] = 1;
            }
        }
    };
    static_assert(!kDefer || A == 1, "deferred copy-through stores are counted for a ring of 2 slots");
    if (loader) {
        // items 0 .. A-1 in flight, item 0 bit-sliced
        int after = 0;
#pragma unroll
        for (int y = 0; y < A; y++) {
            const int64_t t = tile_of(y);
            if (t < P) {
                issue(y % kSlots, t, y % NCH);
                if (y > 0) after += ops_of(y % NCH);
            }
        }
        const int64_t t0 = tile_of(0);
        if (t0 < P) {
            wait_vm(after);
            // (item 0's copy-through stores at once: nothing of the loader's is
            // live across the barrier below)
            u32x4 rA0[kDefer ? PER : 1], rB0[kDefer ? PER : 1];
            slice(0, t0, 0, rA0, rB0);
            if constexpr (kDefer) copy_out(t0, 0, rA0, rB0);
        }
    }
    barrier_w();
    if (loader) {
        // (kDefer) the raw bytes of the item sliced last (from item 1 on), its tile and chunk
        [[maybe_unused]] u32x4 rawA[kDefer ? PER : 1], rawB[kDefer ? PER : 1];
        [[maybe_unused]] int64_t raw_t = 0;
        [[maybe_unused]] int raw_ch = 0;
        for (int i = 0;; i++) {
            if (tile_of(i) >= P) break;
            const int64_t ua = tile_of(i + A);
            if (ua < P) issue((i + A) % kSlots, ua, (i + A) % NCH);
            // (kDefer) item i's copy-through stores, behind item i+1's DMAs
            if constexpr (kDefer)
                if (i > 0) copy_out(raw_t, raw_ch, rawA, rawB);
            const int64_t u1 = tile_of(i + 1);
            if (u1 < P) {
                // this wave's VMEM ops issued after item i+1's DMAs: the copy-through
                // stores of items i+2-A .. i (sliced since; kDefer: item i's, issued
                // just now, from item 1 on) and the DMAs of items i+2 .. i+A;
                // completion is in order, so waiting down to that many means item i+1
                // has landed
                int after = 0;
                if constexpr (do_copy && kCountStores && kDefer) {
                    if (i > 0) after += ops_of(i % NCH);
                } else if constexpr (do_copy && kCountStores) {
#pragma unroll
                    for (int y = i + 2 - A; y <= i; y++)
                        if (y >= 0) after += ops_of(y % NCH);
                }
#pragma unroll
                for (int y = i + 2; y <= i + A; y++)
                    if (tile_of(y) < P) after += ops_of(y % NCH);
                const uint64_t tw = d_now();
                wait_vm(after);
                if constexpr ((DIAG & kDiagStamp) != 0) d_wait += d_now() - tw;
                slice((i + 1) % kSlots, u1, (i + 1) % NCH, rawA, rawB);
                raw_t = u1;
                raw_ch = (i + 1) % NCH;
            }
            barrier_w();
        }
        if (lw == 0) stamp_out(4);
        return;
    }
    // compute waves: per tile, the chunks in order with a barrier after each (the
    // loaders' per-item barrier); the accumulators live across the chunks
    uint32_t acc[OPW][8];
    // deferred parity rows (UPLINK_ENC_DEFER_ROWS): the first DR rows of the
    // previous tile, un-bit-sliced, stored between the next tile's first 2 DR inputs
    constexpr int DR = (DIAG & kDiagNoParityStores) != 0 ? 0
                       : UPLINK_ENC_DEFER_ROWS < OPW ? UPLINK_ENC_DEFER_ROWS : OPW;
    [[maybe_unused]] uint32_t dfr[DR > 0 ? DR : 1][8];
    [[maybe_unused]] TileCols dc{};
    [[maybe_unused]] int dcnt = 0;  // deferred rows held (0: none)
    const int w_rbase = rbase_of(R, NC, wave), w_rows = rows_of(R, NC, wave);
    constexpr bool kLateStores = UPLINK_ENC_LATE_STORES != 0;
    auto store_half = [&](const uint32_t (&w)[8], int row, const TileCols &c, bool second) __attribute__((always_inline)) {
        uint8_t *p = a.out_base + a.out_off[row];
        if (!second) {
            if (c.vA && in_range(a, p + c.outA, true, 3)) st16<true>(p + c.outA, w[0], w[1], w[2], w[3]);
        } else {
            if (c.vB && in_range(a, p + c.outB, true, 3)) st16<true>(p + c.outB, w[4], w[5], w[6], w[7]);
        }
    };
    for (int m = 0;; m++) {
        const int64_t ti = tile_of(m * NCH);
        if (ti >= P) break;
#pragma unroll
        for (int o = 0; o < OPW; o++)
#pragma unroll
            for (int p = 0; p < 8; p++) acc[o][p] = 0;
        static_for<NCH>([&]<int C>() __attribute__((always_inline)) {
            const int i = m * NCH + C;
            // the tile of item i+A+1 onwards (when one starts there): its queue atomic
            // returns during this item's multiply and is published before the barrier
            int pend_m = -1;
            int32_t pending = 0;
            if (taker && (i + A + 1) % NCH == 0 && (i + A + 1) / NCH >= K0) {
                pend_m = (i + A + 1) / NCH;
                pending = take_tile(a, pend_m);
            }
            constexpr int J0 = C * KC, JN = K - J0 < KC ? K - J0 : KC;
            const u32x4 *slot = ring + (i % kSlots) * (SLOT / 16);
            // (DR) the previous tile's deferred rows, half a row after each of the first 2 DR inputs
            auto hook = [&]<int JJ>() __attribute__((always_inline)) {
                if constexpr (DR > 0 && C == 0 && JJ < 2 * DR)
                    if (JJ / 2 < dcnt) store_half(dfr[JJ / 2], w_rbase + JJ / 2, dc, (JJ & 1) != 0);
            };
            static_for<NC>([&]<int W>() __attribute__((always_inline)) {
                if (wave == W) compute_chunk<K, N, NC, OPW, W, J0, JN, DIAG>(slot, lane, acc, hook);
            });
            if (pend_m >= 0) s_q[pend_m & 7] = pending;
            // (kLateStores) the barrier first: the slot is read to the end, so the
            // loaders' next LDS-DMAs go out before this tile's burst of parity stores
            if constexpr (kLateStores) barrier_w();
            if constexpr (C == NCH - 1) {
                const TileCols c = pair_cols(a, ti, lane);
                if constexpr ((DIAG & kDiagNoParityStores) != 0) {
                    sink_rows<OPW>(w_rows, acc);
                } else if constexpr (DR > 0) {
                    static_for<OPW>([&]<int O>() {
                        if (O < w_rows) {
                            uint32_t w[8];
#pragma unroll
                            for (int p = 0; p < 8; p++) w[p] = acc[O][p];
                            unbitslice8(w);
                            if constexpr (O < DR) {
#pragma unroll
                                for (int p = 0; p < 8; p++) dfr[O][p] = w[p];
                            } else {
                                store_half(w, w_rbase + O, c, false);
                                store_half(w, w_rbase + O, c, true);
                            }
                        }
                    });
                    dc = c;
                    dcnt = w_rows < DR ? w_rows : DR;
                } else {
                    store_rows<OPW, true>(a, 0, c, w_rbase, w_rows, acc);
                }
            }
            if constexpr (!kLateStores) barrier_w();
        });
    }
    if constexpr (DR > 0)  // the last tile's deferred rows
        static_for<DR>([&]<int O>() {
            if (O < dcnt) {
                store_half(dfr[O], w_rbase + O, dc, false);
                store_half(dfr[O], w_rbase + O, dc, true);
            }
        });
    if (wave == 0) stamp_out(0);
    // The launch's last workgroup to finish zeroes the queue for the next launch
    // that gets it (so none needs a memset before it).  Every take of this
    // workgroup has returned (its value was used above) before its done count
    // is added, so when the count reaches gridDim.x no take of the launch is left.
    // Then it tells the host, through the slot's completion word, that the slot
    // may go to a launch on another stream.
    if (taker && a.queue) {
        if (atomicAdd(a.queue + kQueueDoneWord, 1u) == gridDim.x - 1) {
            atomicExch(a.queue, 0u);
            atomicExch(a.queue + kQueueDoneWord, 0u);
            if (a.queue_host_done)
                __hip_atomic_store(a.queue_host_done, a.queue_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <int K, int N, int NC, int NL, bool COPY>
__global__ __launch_bounds__((NC + NL) * 64, UPLINK_ENC_WGS > 1 ? (NC + NL) * UPLINK_ENC_WGS / 4 : 1) void rs_encode_special(
    const RsArgs a) {
    encode_body<K, N, NC, NL, COPY, 0>(a);
}

// Limits of the compile-time encoder: 1 <= n - k <= 96 parity rows (12
// accumulator rows per compute wave), k <= kMaxOps inputs.
constexpr bool supported(int k, int n) { return k >= 1 && k <= kMaxOps && n - k >= 1 && n - k <= 96; }
// Waves: 4 loaders and, from 16 parity rows on, 8 compute waves -- two per
// SIMD, so each issues VALU at the full rate (one wave alone on a SIMD issues
// every other cycle); the 4-plane combinations each compute wave rebuilds per
// input cost 14 % more VALU than with 4.
constexpr int compute_waves(int k, int n) { return n - k >= 16 ? UPLINK_ENC_NC : 4; }  // -D override: A/B builds
constexpr int loader_waves(int k, int n) { return UPLINK_ENC_PARITY_NL; }  // -D override: A/B builds
constexpr int parity_compute_waves(int k, int n) { return compute_waves(k, n); }
// The full encode with at most 40 parity rows keeps 4 compute waves: its
// loaders' copy-through share of a tile is large enough that the 4 extra
// waves' combinations cost more than their issue rate gains (RS(20,60) 47.2
// vs 49.8 us per segment; RS(29,80) 50.0 vs 47.8 the other way).
constexpr int full_compute_waves(int k, int n) { return n - k <= 40 ? 4 : compute_waves(k, n); }
constexpr int full_loader_waves(int k, int n) { return loader_waves(k, n); }
// One workgroup per CU: its ring takes up to 144 KiB of LDS.
constexpr int wgs_per_cu(int k, int waves) { return UPLINK_ENC_WGS; }

}  // namespace enc
}  // namespace uplink_ec
