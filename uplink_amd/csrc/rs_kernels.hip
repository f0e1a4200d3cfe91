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
//  * rs_encode_special<K,N,..> (rs_encoder.hpp): G is a compile-time constant
//    (the same Lagrange construction as infectious, gf256_field.hpp), and each
//    output plane gets the XOR of two precomputed 4-plane combinations ("four
//    Russians"), one v_bitop3 per (output plane, input share): 8 ops per GF
//    multiply-add of a 32-byte column block instead of ~16 for the plain
//    bit-matrix.  Library-built for the configurations of
//    rs_encoder_aot.def, compiled by hiprtc for any other (k, n).
//  * rs_matmul_jt<NW> (this file): any runtime matrix (the rebuild matrix
//    (G_S)^-1 of a share set, re-encoding for error detection, per-stripe
//    EncodeSingle).  Same four-Russians body, but the coefficient is data:
//    each (row, input) pair is one call into a table of 256 compile-time
//    leaves (rs_jump_table.inc), the accumulator row picked by VGPR index
//    mode -- no per-bit branches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "gf256_field.hpp"
#include "rs_device.hpp"
#include "rs_kernels.hpp"
#include "rs_sets.hpp"
#include "rs_sl.hpp"

namespace uplink_ec {
namespace {

using namespace dev;

__constant__ GfTables d_gf = make_gf_tables();

// Runtime-matrix kernel (rebuild, and encode for (k, n) without a
// specialised kernel).  Every wave computes (no loader waves) and several
// workgroups share a CU; inputs are staged in LDS chunks of 2*NW shares.
// The rows of a pass are spread evenly over the NW waves (<= 8 each, the
// accumulators of jt_inputs), each wave stages two inputs of a chunk of 2*NW,
// and the row group of a wave is rotated by
// blockIdx so the SIMDs of a CU, which host waves of several workgroups, get
// equal VALU work.  Each coefficient is multiplied in through the jump table
// (jt_inputs), whose 8 leaf addresses per (pass, j, wave row group) come
// from the table rs_jt_targets made (a.jt_tgt, [pass][j][group][8] 64-bit
// words; leaf 0 = empty for padded rows); jt_lds_bytes() gives the dynamic
// LDS size.
constexpr int kJtRows = 8;  // accumulator rows per wave

// SL: the straight-line form (rs_sl.hpp): instead of the jump table, each
// wave calls the plan's generated code segment for (pass, chunk, row group)
// once per chunk; a.jt_tgt then holds those segments' absolute addresses,
// [pass][chunk][group].
template <int NW, bool SL>
__global__ __launch_bounds__(NW * 64, 4) void rs_matmul_jt(const RsArgs a) {
    constexpr int JC = SL ? sl::chunk_inputs(NW) : 2 * NW, OPW = kJtRows, PER = (JC + NW - 1) / NW;
    // the inputs in as few chunks of at most JC as they need, dealt evenly
    // (29 inputs on 7 waves: 10 + 10 + 9, not 14 + 14 + 1)
    const int nchunks = (a.nin + JC - 1) / JC;
    const int CH = (a.nin + nchunks - 1) / nchunks;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *lds = smem;                                  // 2 x [JC][8 planes][64 lanes]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int group = (wave + (int)(blockIdx.x % NW)) % NW;
    const int npass = a.nout > 0 ? (a.nout + NW * OPW - 1) / (NW * OPW) : 1;
    const uint32_t lds_addr = (uint32_t)(uintptr_t)lds + (uint32_t)lane * 16;  // the wide layout, both bodies
    // Plane chunks alternate between two LDS buffers, so one barrier per chunk
    // suffices: a wave staging chunk c+1 has passed barrier c, which every wave
    // reached only after it finished reading chunk c-1 from that buffer.
    int buf = 0;
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        for (int pass = 0; pass < npass; pass++) {
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rbase = p0 + group * prow / NW;
            const int cnt = p0 + (group + 1) * prow / NW - rbase;
            u32x8 acc[OPW];
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
            StageRegs<PER> r;
            load_inputs<NW, PER, true>(a, seg, c, wave, 0, a.nin < CH ? a.nin : CH, r);
            for (int j0 = 0; j0 < a.nin; j0 += CH) {
                const int jn = a.nin - j0 < CH ? a.nin - j0 : CH;
                slice_inputs<NW, PER, true, true>(a, seg, c, lds + buf * (JC * 8 * 64), lane, wave, j0, jn, pass == 0, r);
                lds_barrier();
                // the next chunk's loads are in flight while this chunk is multiplied in
                if (j0 + CH < a.nin) {
                    const int j1 = j0 + CH;
                    load_inputs<NW, PER, true>(a, seg, c, wave, j1, a.nin - j1 < CH ? a.nin - j1 : CH, r);
                }
                if (cnt > 0) {
                    const uint32_t xa = lds_addr + (uint32_t)(buf * JC * 8 * 64 * 4);
                    if constexpr (SL)
                        sl_segment(acc, xa, a.jt_tgt + (pass * nchunks + j0 / CH) * NW + group);
                    else
                        jt_inputs(acc, xa, a.jt_tgt + ((pass * a.nin + j0) * NW + group) * OPW,
                                  (uint32_t)(NW * OPW * 8), (uint32_t)(OPW - cnt), (uint32_t)jn);
                }
                buf ^= 1;
            }
            uint32_t rows[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) rows[o][p] = acc[o][p];
            // with zero_check, rows from a.nstore on are syndrome rows (the rows below
            // it, a fused Decode's rebuilt data shares, are stored): any set bit of a
            // valid column is an error (zero is zero in the bit-sliced layout too;
            // plane bits 0-3 of each byte are chunk A, bits 4-7 chunk B)
            const int nst = a.zero_check ? a.nstore : rbase + cnt;
            if (a.zero_check) {
                uint32_t any = 0;
#pragma unroll
                for (int o = 0; o < OPW; o++)
                    if (o < cnt && rbase + o >= nst)
#pragma unroll
                        for (int p = 0; p < 8; p++) any |= rows[o][p];
                any &= (c.vA ? 0x0F0F0F0Fu : 0u) | (c.vB ? 0xF0F0F0F0u : 0u);
                if (__ballot(any != 0) != 0 && lane == 0) atomicAdd(a.zero_check, 1u);
            }
            if (rbase < nst) store_rows<OPW, true>(a, seg, c, rbase, nst - rbase < cnt ? nst - rbase : cnt, rows);
        }
    }
}

// rs_matmul_jt's straight-line form with the input shares requested straight
// into LDS (LDS-DMA, no registers held): the DMAs of chunk c+D are issued
// after chunk c's barrier, so D chunks of every wave's loads are in flight
// while it multiplies (rs_matmul_jt: one, in registers).  A ring of D+1 slots
// of 2*NW inputs each; the issuing wave waits for its own DMAs by a counted
// vmcnt and bit-slices them in place (the wide layout the straight-line
// code reads), copying the present data shares through on the way.  Every
// lane issues the copy-through stores (a lane past the end of the segment
// rewrites column 0 with the bytes already there), so each wave's count of
// VMEM operations is exact.  Each pass's pipeline starts and drains within
// the pass.
// SL = false: the same pipeline around the jump-table body (per-stripe calls,
// or a plan before its generated code is ready), reading the same wide layout.
template <int NW, int D, bool SL = true>
__global__ __launch_bounds__(NW * 64, 4) void rs_matmul_dma(const RsArgs a) {
    constexpr int JC = SL ? sl::chunk_inputs(NW) : 2 * NW, PER = (JC + NW - 1) / NW, OPW = kJtRows, S = D + 1,
                  SLOT = JC * 2048;
    static_assert(D >= 1 && D <= 3, "store ring below holds at most 2 chunks");
#ifdef UPLINK_EC_CHECKED
    constexpr bool kCountStores = false;  // the checked build may skip a store: count none (waits longer)
#else
    constexpr bool kCountStores = true;
#endif
    const int nchunks = (a.nin + JC - 1) / JC;
    const int CH = (a.nin + nchunks - 1) / nchunks;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    u32x4 *ring = (u32x4 *)smem;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int group = (wave + (int)(blockIdx.x % NW)) % NW;
    const int npass = a.nout > 0 ? (a.nout + NW * OPW - 1) / (NW * OPW) : 1;
    const uint32_t ring_addr = (uint32_t)(uintptr_t)smem;
    // inputs of chunk ch this wave owns (j = wave, wave + NW, ...; CH <= JC)
    auto owned = [&](int ch) -> int {
        const int jn = a.nin - ch * CH < CH ? a.nin - ch * CH : CH;
        return wave < jn ? (jn - wave + NW - 1) / NW : 0;
    };
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
        const int64_t iA = c.vA ? c.inA : 0, iB = c.vB ? c.inB : 0;
        const int64_t oA = c.vA ? c.outA : 0, oB = c.vB ? c.outB : 0;
        auto issue = [&](int ch) {
            const uint32_t d0 = ring_addr + (uint32_t)((ch % S) * SLOT);
            const int j0 = ch * CH;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (i < owned(ch)) {
                    const uint8_t *p = in_seg + a.in_off[j0 + j];
                    const uint8_t *pa = p + iA, *pb = p + iB;
                    if (!in_range(a, pa, false, 4)) pa = a.chk_in_lo;
                    if (!in_range(a, pb, false, 4)) pb = a.chk_in_lo;
                    const uint32_t d = __builtin_amdgcn_readfirstlane(d0 + (uint32_t)(j * 2048));
                    dma_1k(pa, d);
                    dma_1k(pb, d + 1024);
                }
            }
        };
        for (int pass = 0; pass < npass; pass++) {
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rbase = p0 + group * prow / NW;
            const int cnt = p0 + (group + 1) * prow / NW - rbase;
            const bool do_copy = pass == 0;
            u32x8 acc[OPW];
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
            for (int y = 0; y < D && y < nchunks; y++) issue(y);
            int st1 = 0, st2 = 0;  // copy-through stores of the last two slices (newest first)
            for (int ch = 0; ch < nchunks; ch++) {
                // this wave's VMEM operations issued after chunk ch's DMAs: the stores of
                // slices ch-D+1 .. ch-1 and the DMAs of chunks ch+1 .. ch+D-1 (in order
                // of completion, so waiting down to that many means chunk ch has landed)
                int after = 0;
                if constexpr (kCountStores) after += (D >= 2 ? st1 : 0) + (D >= 3 ? st2 : 0);
#pragma unroll
                for (int y = 1; y < D; y++)
                    if (ch + y < nchunks) after += 2 * owned(ch + y);
                wait_vm(after);
                // bit-slice this wave's inputs of chunk ch in place
                const int j0 = ch * CH;
                u32x4 *slot = ring + (ch % S) * (SLOT / 16);
                int st = 0;
#pragma unroll
                for (int i = 0; i < PER; i++) {
                    const int j = wave + NW * i;
                    if (i < owned(ch)) {
                        const u32x4 A4 = slot[j * 128 + lane], B4 = slot[j * 128 + 64 + lane];
                        const int64_t co = a.copy_off[j0 + j];
                        if (do_copy && co >= 0) {
                            uint8_t *p = out_seg + co;
                            if (in_range(a, p + oA, true, 5)) st16<true>(p + oA, A4.x, A4.y, A4.z, A4.w);
                            if (in_range(a, p + oB, true, 5)) st16<true>(p + oB, B4.x, B4.y, B4.z, B4.w);
                            st += 2;
                        }
                        uint32_t w[8] = {A4.x, A4.y, A4.z, A4.w, B4.x, B4.y, B4.z, B4.w};
                        bitslice8(w);
                        // (in place: the wide layout both bodies read puts a lane's planes where its bytes were)
                        slot[j * 128 + lane] = (u32x4){w[0], w[1], w[2], w[3]};
                        slot[j * 128 + 64 + lane] = (u32x4){w[4], w[5], w[6], w[7]};
                    }
                }
                st2 = st1;
                st1 = st;
                lds_barrier();
                // chunk ch+D into the slot chunk ch-1 left (every wave is past its multiply)
                if (ch + D < nchunks) issue(ch + D);
                if (cnt > 0) {
                    if constexpr (SL) {
                        sl_segment(acc, ring_addr + (uint32_t)((ch % S) * SLOT) + (uint32_t)lane * 16,
                                   a.jt_tgt + (pass * nchunks + ch) * NW + group);
                    } else {
                        const int jn = a.nin - j0 < CH ? a.nin - j0 : CH;
                        jt_inputs(acc, ring_addr + (uint32_t)((ch % S) * SLOT) + (uint32_t)lane * 16,
                                  a.jt_tgt + ((pass * a.nin + j0) * NW + group) * OPW, (uint32_t)(NW * OPW * 8),
                                  (uint32_t)(OPW - cnt), (uint32_t)jn);
                    }
                }
            }
            uint32_t rows[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) rows[o][p] = acc[o][p];
            const int nst = a.zero_check ? a.nstore : rbase + cnt;
            if (a.zero_check) {
                uint32_t any = 0;
#pragma unroll
                for (int o = 0; o < OPW; o++)
                    if (o < cnt && rbase + o >= nst)
#pragma unroll
                        for (int p = 0; p < 8; p++) any |= rows[o][p];
                any &= (c.vA ? 0x0F0F0F0Fu : 0u) | (c.vB ? 0xF0F0F0F0u : 0u);
                if (__ballot(any != 0) != 0 && lane == 0) atomicAdd(a.zero_check, 1u);
            }
            if (rbase < nst) store_rows<OPW, true>(a, seg, c, rbase, nst - rbase < cnt ? nst - rbase : cnt, rows);
            // the slot the next pass's first DMAs go to may still be read by a wave's multiply
            lds_barrier();
        }
    }
}

template <int NW, int D, bool SL = true>
size_t dma_lds_bytes() {
    return (size_t)(D + 1) * (SL ? sl::chunk_inputs(NW) : 2 * NW) * 2048;
}

// Rebuild with nothing to compute (every data share present): a copy of the
// data shares into the stripe-major segment, with no bit planes or barriers.
// Each of the 2 waves loads all of its (up to 16) inputs of the tile before
// it stores any, and the launch asks for kCopyLds bytes of LDS it never
// touches, so only 2 workgroups share a CU: RS(29,80) 23.8 us per segment,
// against 24.8-24.9 through rs_matmul_jt and 26.0-26.3 for this kernel at
// full occupancy (more workgroups per CU, more write streams open at once;
// DESIGN.md §4 "Rebuild, round 3").
template <int NW>
__global__ __launch_bounds__(NW * 64) void rs_copy_shares(const RsArgs a) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int G = 16;
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
        uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
        const int64_t oA = c.vA ? c.inA : 0, oB = c.vB ? c.inB : 0;
        for (int j0 = wave; j0 < a.nin; j0 += NW * G) {
            uint4 A[G], B[G];
#pragma unroll
            for (int i = 0; i < G; i++) {
                const int j = j0 + NW * i;
                if (j < a.nin) {
                    const uint8_t *p = in_seg + a.in_off[j];
                    const uint4 z = make_uint4(0, 0, 0, 0);
                    A[i] = in_range(a, p + oA, false, 6) ? ld16<true>(p + oA) : z;
                    B[i] = in_range(a, p + oB, false, 6) ? ld16<true>(p + oB) : z;
                }
            }
#pragma unroll
            for (int i = 0; i < G; i++) {
                const int j = j0 + NW * i;
                if (j < a.nin && a.copy_off[j] >= 0) {
                    uint8_t *p = out_seg + a.copy_off[j];
                    if (c.vA && in_range(a, p + c.outA, true, 7)) st16<true>(p + c.outA, A[i].x, A[i].y, A[i].z, A[i].w);
                    if (c.vB && in_range(a, p + c.outB, true, 7)) st16<true>(p + c.outB, B[i].x, B[i].y, B[i].z, B[i].w);
                }
            }
        }
    }
}

template <int NW, bool SL = true>
size_t jt_lds_bytes(const RsArgs &) {
    return (size_t)2 * (SL ? sl::chunk_inputs(NW) : 2 * NW) * 8 * 64 * 4;
}

int jt_waves(int nout) { return nout <= 2 * kJtRows ? 2 : nout <= 3 * kJtRows ? 3 : 4; }

// Leaf addresses of the matrix for rs_matmul_jt<nw>: the rows of each pass
// split over the nw row groups exactly as that kernel splits them, right-
// aligned in 8 slots (jt_inputs enters at call site 8 - count).
__global__ __launch_bounds__(256) void rs_jt_targets(const RsArgs a, int nw, uint64_t *tgt) {
    const uint64_t base = jt_table_base();
    if (nw == 0) {  // jt_table_base_addr: only the address of leaf 0
        if (threadIdx.x == 0) tgt[0] = base;
        return;
    }
    constexpr int OPW = kJtRows;
    const int npass = a.nout > 0 ? (a.nout + nw * OPW - 1) / (nw * OPW) : 1;
    const int per_pass = a.nin * nw * OPW;
    for (int t = threadIdx.x; t < npass * per_pass; t += blockDim.x) {
        const int pass = t / per_pass, r = t - pass * per_pass;
        const int j = r / (nw * OPW), g = (r / OPW) % nw, o = r % OPW;
        const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
        const int rb = p0 + g * prow / nw, cn = p0 + (g + 1) * prow / nw - rb;
        const int oo = o - (OPW - cn);
        const uint32_t c = oo >= 0 ? a.coef[(int64_t)j * a.coef_ld + rb + oo] : 0u;
        tgt[t] = base + (uint64_t)c * RS_JT_SLOT;
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

// Batched EncodeSingle (ec_encode_single's coalesced calls): share nums[r]
// of stripe r, from the stripe itself (a data share) or from the parity
// pieces of the batch ([n-k][B*bs]), into out[r]; 16-byte units when bs allows.
__global__ __launch_bounds__(256) void rs_gather_shares(const uint8_t *stripes, const uint8_t *parity, const int *nums,
                                                        int k, int64_t nreq, int64_t bs, uint8_t *out) {
    const bool wide = (bs & 15) == 0;
    const int64_t unit = wide ? 16 : 1, per = bs / unit, total = nreq * per;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / per, t = (i - r * per) * unit;
        const int num = nums[r];
        const uint8_t *src = num < k ? stripes + (r * k + num) * bs + t : parity + ((int64_t)(num - k) * nreq + r) * bs + t;
        if (wide) *(uint4 *)(out + r * bs + t) = *(const uint4 *)src;
        else out[r * bs + t] = *src;
    }
}

}  // namespace
}  // namespace uplink_ec

// ------------------------------------------------ launch entry points
namespace uplink_ec {

namespace {
int g_cu_count = 0;
}  // namespace

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

int default_grid(int64_t total_tiles, int wgs_per_cu) {
    int64_t g = (int64_t)cu_count() * wgs_per_cu;
    if (total_tiles < g) g = total_tiles;
    return (int)(g > 0 ? g : 1);
}

size_t jt_targets_bytes(const RsArgs &a) {
    const int nw = jt_waves(a.nout);
    const int npass = a.nout > 0 ? (a.nout + nw * kJtRows - 1) / (nw * kJtRows) : 1;
    return (size_t)npass * a.nin * nw * kJtRows * sizeof(uint64_t);
}

hipError_t launch_jt_targets(const RsArgs &a, uint64_t *targets, hipStream_t s) {
    hipLaunchKernelGGL(rs_jt_targets, dim3(1), dim3(256), 0, s, a, jt_waves(a.nout), targets);
    return hipGetLastError();
}

hipError_t jt_table_base_addr(uint64_t *out, hipStream_t s) {
    uint64_t *d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(uint64_t));
    if (e != hipSuccess) return e;
    RsArgs a{};
    hipLaunchKernelGGL(rs_jt_targets, dim3(1), dim3(64), 0, s, a, 0, d);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    return e;
}

namespace {
// chunks of LDS-DMA prefetch of the straight-line rebuild (rs_matmul_dma); 0 =
// rs_matmul_jt's register-staged form.  Set at ec_create (UPLINK_EC_REBUILD_DEPTH)
// for A/B builds of the library in one process.  One chunk ahead measured
// fastest: 16 RS(29,80) segments per launch, rebuild 399.7 us at depth 1,
// 409.4 at 2, 443.5 at 3 (each deeper slot costs the CU workgroups) and 418.5
// register-staged (profiles/r04/exp/ab_rebuild_dma.log).
std::atomic<int> g_rebuild_depth{1};  // written by ec_create, read by launches on any thread

template <int NW, int D, bool SL = true>
void launch_dma(const RsArgs &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((rs_matmul_dma<NW, D, SL>), dim3(grid), dim3(NW * 64), (dma_lds_bytes<NW, D, SL>()), s, a);
}

template <int NW>
void launch_dma_depth(const RsArgs &a, int grid, hipStream_t s, int depth) {
    // above 4 waves the ring stays within the 64 KiB of dynamic LDS a launch gets by default
    if constexpr (NW > 4) {
        launch_dma<NW, 1>(a, grid, s);
    } else {
        if (depth <= 1) launch_dma<NW, 1>(a, grid, s);
        else if (depth == 2) launch_dma<NW, 2>(a, grid, s);
        else launch_dma<NW, 3>(a, grid, s);
    }
}
}  // namespace

void configure_rebuild(int depth) { g_rebuild_depth.store(depth < 0 ? 0 : depth > 3 ? 3 : depth); }

template <bool SL>
hipError_t launch_matmul(const RsArgs &a, int grid, hipStream_t s) {
    if (!a.jt_tgt || a.nout > kMaxOps || a.nin > kMaxOps) return hipErrorInvalidValue;
    // up to 16 waves per CU (4 per SIMD: the jump-table body holds ~126
    // VGPRs); as few waves per workgroup as the rows need, since every wave
    // rebuilds the 4-plane combinations of each input for its own rows.
    // One workgroup per tile (not a persistent grid): while a workgroup waits
    // for its first chunk, the CU runs the others the dispatcher has placed
    // there -- the next-tile prefetch the kernel's registers have no room for
    // (rebuild of 16 RS(29,80) segments 419 -> 398 us, m = 29 28.1 -> 24.8 us
    // per segment).  The encoder keeps its persistent grid (one
    // workgroup per tile: 809 -> 1248 us).
    // (the kernels loop over tiles past the grid; grid x workgroup size stays below 2^32 work-items)
    if (grid <= 0) grid = (int)std::min<int64_t>(std::max<int64_t>(a.total_tiles, 1), 1 << 22);
    if (a.nout == 0 && !a.zero_check) {
        constexpr size_t kCopyLds = 58 * 1024;  // an occupancy cap: 2 workgroups per CU
        hipLaunchKernelGGL(rs_copy_shares<2>, dim3(grid), dim3(2 * 64), kCopyLds, s, a);
        return hipGetLastError();
    }
    const int depth = g_rebuild_depth.load(std::memory_order_relaxed);
    if (!SL && depth > 0) {  // the jump-table body (2-4 waves), one chunk ahead
        switch (jt_waves(a.nout)) {
        case 2: launch_dma<2, 1, false>(a, grid, s); break;
        case 3: launch_dma<3, 1, false>(a, grid, s); break;
        default: launch_dma<4, 1, false>(a, grid, s);
        }
        return hipGetLastError();
    }
    if (SL && depth > 0) {
        switch (sl::split_for(a.nout).nw) {
        case 8: launch_dma_depth<8>(a, grid, s, depth); break;
        case 7: launch_dma_depth<7>(a, grid, s, depth); break;
        case 6: launch_dma_depth<6>(a, grid, s, depth); break;
        case 5: launch_dma_depth<5>(a, grid, s, depth); break;
        case 2: launch_dma_depth<2>(a, grid, s, depth); break;
        case 3: launch_dma_depth<3>(a, grid, s, depth); break;
        default: launch_dma_depth<4>(a, grid, s, depth);
        }
        return hipGetLastError();
    }
    switch (SL ? sl::split_for(a.nout).nw : jt_waves(a.nout)) {
    case 8:
        hipLaunchKernelGGL((rs_matmul_jt<8, true>), dim3(grid), dim3(8 * 64), jt_lds_bytes<8>(a), s, a);
        break;
    case 7:
        hipLaunchKernelGGL((rs_matmul_jt<7, true>), dim3(grid), dim3(7 * 64), jt_lds_bytes<7>(a), s, a);
        break;
    case 6:
        hipLaunchKernelGGL((rs_matmul_jt<6, true>), dim3(grid), dim3(6 * 64), jt_lds_bytes<6>(a), s, a);
        break;
    case 5:
        hipLaunchKernelGGL((rs_matmul_jt<5, true>), dim3(grid), dim3(5 * 64), jt_lds_bytes<5>(a), s, a);
        break;
    case 2:
        hipLaunchKernelGGL((rs_matmul_jt<2, SL>), dim3(grid), dim3(2 * 64), (jt_lds_bytes<2, SL>(a)), s, a);
        break;
    case 3:
        hipLaunchKernelGGL((rs_matmul_jt<3, SL>), dim3(grid), dim3(3 * 64), (jt_lds_bytes<3, SL>(a)), s, a);
        break;
    default:
        hipLaunchKernelGGL((rs_matmul_jt<4, SL>), dim3(grid), dim3(4 * 64), (jt_lds_bytes<4, SL>(a)), s, a);
    }
    return hipGetLastError();
}

hipError_t launch_matmul_generic(const RsArgs &a, int grid, hipStream_t s) { return launch_matmul<false>(a, grid, s); }

hipError_t launch_matmul_sl(const RsArgs &a, int grid, hipStream_t s) { return launch_matmul<true>(a, grid, s); }

hipError_t launch_gather_shares(const uint8_t *stripes, const uint8_t *parity, const int *nums, int k, int64_t nreq,
                               int64_t bs, uint8_t *out, hipStream_t s) {
    const int64_t units = nreq * ((bs & 15) == 0 ? bs / 16 : bs);
    int64_t blocks = (units + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(rs_gather_shares, dim3((unsigned)blocks), dim3(256), 0, s, stripes, parity, nums, k, nreq, bs, out);
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
