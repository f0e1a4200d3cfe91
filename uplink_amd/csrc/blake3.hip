// BLAKE3-256 of erasure pieces, on the GPU.
//
// Replaces the piece hash the upload computes byte by byte in a TeeReader
// (private/piecestore/upload.go:133 NewHashFromAlgorithm(BLAKE3), :155
// io.TeeReader(data, client.hash), :270 Hash: client.hash.Sum(nil); the
// default algorithm is BLAKE3, hash.go:20-26).  The hash function itself is
// github.com/zeebo/blake3 v0.2.3 (go.mod:29), restated on the CPU in
// oracle/blake3_oracle.c and pinned there by the official test vectors.
//
// Layout of the work:
//   b3_chunks   one lane per 1 KiB chunk (16 sequential compressions of
//               64-byte blocks), 256 chunks per workgroup.  The chunk CVs go
//               to LDS and the workgroup folds its aligned group of 256 into
//               one subtree CV, level by level: pairs (2i, 2i+1) -> parent i,
//               an odd last node moves up unchanged.  Because every group
//               starts on a multiple of 256 chunks, this is exactly BLAKE3's
//               left-complete tree restricted to the group.
//   b3_parents  the same fold over the subtree CVs of a piece (256 per
//               workgroup), repeated until one workgroup holds the whole
//               piece; that one applies ROOT to its last parent and writes
//               the 32-byte hash.
// A piece of one chunk takes ROOT on the chunk's last block; a piece of one
// group is finished inside b3_chunks.
//
// Cost: 7 rounds x 8 G x ~12 VALU per 64-byte block (v_add3_u32,
// v_xor_b32, v_alignbit_b32 / v_perm_b32), ~11 VALU per input byte: the
// kernel is VALU-bound, not HBM-bound.
#include <hip/hip_runtime.h>

#include "blake3.hpp"
#include "blake3_device.hpp"

namespace uplink_ec {
namespace {

using namespace b3;

// Start of piece j: pieces come in sets of `pieces_per_set` (one set per
// segment), set_stride apart.
__device__ __forceinline__ const uint8_t *piece_base(const B3View &v, uint64_t j) {
    return v.base + (int64_t)(j / v.pieces_per_set) * v.set_stride + (int64_t)(j % v.pieces_per_set) * v.piece_stride;
}

// byte t of a piece starting at pb
template <bool kFast>
__device__ __forceinline__ const uint8_t *at(const B3View &v, const uint8_t *pb, uint64_t t) {
    if (kFast)  // power-of-two runs: no 64-bit division
        return pb + (int64_t)(t >> v.run_shift) * v.run_stride + (t & (v.run - 1));
    return pb + (int64_t)(t / v.run) * v.run_stride + (t % v.run);
}

// `n` 16-byte words at p (plain loads: the second half of each 128-byte
// line is read by the next block, so non-temporal loads, which let the line
// go, cost 2x here -- tools/exp/b3_probe.hip)
template <int n>
__device__ __forceinline__ void load_words(const uint8_t *p, uint32_t *m) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
    for (int i = 0; i < n; i++) {
        u32x4 w = q[i];
        m[4 * i] = w[0], m[4 * i + 1] = w[1], m[4 * i + 2] = w[2], m[4 * i + 3] = w[3];
    }
}

// 64-byte block starting at byte t, `len` valid bytes (zero padded)
template <bool kFast>
__device__ __forceinline__ void load_block(const B3View &v, const uint8_t *pb, uint64_t t, uint32_t len,
                                           uint32_t (&m)[16]) {
    if (kFast && len == 64) {  // the block lies in one run, 16-byte aligned
        load_words<4>(at<kFast>(v, pb, t), m);
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = 0;
    for (uint32_t b = 0; b < len; b++) m[b >> 2] |= (uint32_t)*at<kFast>(v, pb, t + b) << (8 * (b & 3));
}

// CV of a full 1 KiB chunk whose 128-byte lines each lie in one run: one
// whole line (two blocks) per load step, the next line in flight meanwhile
__device__ __forceinline__ void full_chunk_lines(const B3View &v, const uint8_t *pb, uint64_t t0, uint64_t c,
                                                 uint32_t last_flags, uint32_t (&h)[8]) {
    uint32_t m[32], nx[32];
    load_words<8>(at<true>(v, pb, t0), m);
    for (int pr = 0; pr < 8; pr++) {
        if (pr < 7) load_words<8>(at<true>(v, pb, t0 + 128 * (pr + 1)), nx);
        uint32_t lo[16], hi[16];
#pragma unroll
        for (int i = 0; i < 16; i++) lo[i] = m[i], hi[i] = m[16 + i];
        compress(h, lo, (uint32_t)c, (uint32_t)(c >> 32), 64, pr == 0 ? kChunkStart : 0);
        compress(h, hi, (uint32_t)c, (uint32_t)(c >> 32), 64, pr == 7 ? last_flags : 0);
#pragma unroll
        for (int i = 0; i < 32; i++) m[i] = nx[i];
    }
}

// Two views of pieces with the same length hashed in one launch (the data
// and the parity pieces of a batch of segments): piece p < split is piece p
// of v[0], else piece p - split of v[1]; hashes and tree nodes are indexed
// by p.
struct B3Pair {
    B3View v[2];
    uint64_t split;
};

// chunks per lane (two per lane, folding the first tree level in registers,
// halved the waves in flight and measured slower: DESIGN.md §4b)
constexpr int kPerLane = 1;
constexpr int kGroupChunks = kGroup * kPerLane;  // chunks per workgroup

// CV of chunk c of a piece (ROOT on its last block when `root`)
template <bool kFast>
__device__ __forceinline__ void chunk_cv(const B3View &v, const uint8_t *pb, uint64_t c, bool root, uint32_t (&h)[8]) {
    const uint64_t t0 = c * 1024;
    const uint64_t clen = v.piece_len - t0 < 1024 ? v.piece_len - t0 : 1024;  // 0 only for an empty piece
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = kIV[i];
    if (kFast && clen == 1024 && v.run_shift >= 7) {
        full_chunk_lines(v, pb, t0, c, kChunkEnd | (root ? kRoot : 0), h);
        return;
    }
    // partial chunk, 64-byte runs, or the byte path: block by block
    const uint32_t nb = clen ? (uint32_t)((clen + 63) >> 6) : 1;
    uint32_t m[16], nx[16];
    load_block<kFast>(v, pb, t0, nb == 1 ? (uint32_t)clen : 64, m);
    for (uint32_t b = 0; b < nb; b++) {
        const bool last = b + 1 == nb;
        const uint32_t blen = last ? (uint32_t)(clen - 64ull * b) : 64;
        if (!last) {  // prefetch the next block while this one compresses
            const uint32_t nlen = b + 2 == nb ? (uint32_t)(clen - 64ull * (b + 1)) : 64;
            load_block<kFast>(v, pb, t0 + 64ull * (b + 1), nlen, nx);
        }
        const uint32_t flags = (b == 0 ? kChunkStart : 0) | (last ? kChunkEnd : 0) | (last && root ? kRoot : 0);
        compress(h, m, (uint32_t)c, (uint32_t)(c >> 32), blen, flags);
        if (!last) {
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = nx[i];
        }
    }
}

template <bool kFast>
__global__ __launch_bounds__(kGroup) void b3_chunks(B3Pair pv, uint64_t nchunks, uint32_t groups, uint32_t *nodes,
                                                     uint8_t *hashes) {
    __shared__ uint32_t lds[2][8][kGroup];
    const uint64_t piece = blockIdx.x / groups;
    const uint32_t group = blockIdx.x % groups;
    const uint64_t c0 = (uint64_t)group * kGroupChunks + (uint64_t)threadIdx.x * kPerLane;
    const bool second = piece >= pv.split;
    const B3View &v = pv.v[second];
    const uint8_t *pb = piece_base(v, second ? piece - pv.split : piece);
    if (nchunks <= (uint64_t)kPerLane) {  // the whole piece is this lane's: it also applies ROOT
        if (threadIdx.x == 0 && group == 0) {
            uint32_t h[8];
            chunk_cv<kFast>(v, pb, 0, nchunks == 1, h);
            if (nchunks == 2) {
                uint32_t r[8], p[8];
                chunk_cv<kFast>(v, pb, 1, false, r);
                parent(p, h, r, true);
                store_hash(hashes + 32 * piece, p);
            } else {
                store_hash(hashes + 32 * piece, h);
            }
        }
        return;
    }
    if (c0 < nchunks) {
        uint32_t h[8];
        chunk_cv<kFast>(v, pb, c0, false, h);
        if (kPerLane == 2 && c0 + 1 < nchunks) {  // the level-1 parent of this lane's pair
            uint32_t r[8], p[8];
            chunk_cv<kFast>(v, pb, c0 + 1, false, r);
            parent(p, h, r, false);
#pragma unroll
            for (int i = 0; i < 8; i++) h[i] = p[i];
        }  // an odd last chunk moves up unchanged
#pragma unroll
        for (int i = 0; i < 8; i++) lds[0][i][threadIdx.x] = h[i];
    }
    __syncthreads();
    const uint64_t left = nchunks - (uint64_t)group * kGroupChunks;  // chunks in this group
    const uint64_t nodes1 = (left < (uint64_t)kGroupChunks ? left : kGroupChunks) + kPerLane - 1;
    const int cnt = (int)(nodes1 / kPerLane);
    uint32_t h[8];
    fold(lds, cnt, groups == 1, h);
    if (threadIdx.x == 0) {
        if (groups == 1)
            store_hash(hashes + 32 * piece, h);
        else {
            uint4 *o = reinterpret_cast<uint4 *>(nodes + ((uint64_t)piece * groups + group) * 8);
            o[0] = make_uint4(h[0], h[1], h[2], h[3]);
            o[1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
    }
}

// nodes_in: [piece][nin][8] subtree CVs (nin >= 2); folds groups of 256
__global__ __launch_bounds__(kGroup) void b3_parents(const uint32_t *nodes_in, uint32_t nin, uint32_t groups,
                                                      uint32_t *nodes_out, uint8_t *hashes) {
    __shared__ uint32_t lds[2][8][kGroup];
    const uint64_t piece = blockIdx.x / groups;
    const uint32_t group = blockIdx.x % groups;
    const uint32_t i0 = group * kGroup;
    const int cnt = nin - i0 < (uint32_t)kGroup ? (int)(nin - i0) : kGroup;
    if ((int)threadIdx.x < cnt) {
        const uint4 *p = reinterpret_cast<const uint4 *>(nodes_in + ((uint64_t)piece * nin + i0 + threadIdx.x) * 8);
        uint4 a = p[0], b = p[1];
        lds[0][0][threadIdx.x] = a.x, lds[0][1][threadIdx.x] = a.y, lds[0][2][threadIdx.x] = a.z;
        lds[0][3][threadIdx.x] = a.w, lds[0][4][threadIdx.x] = b.x, lds[0][5][threadIdx.x] = b.y;
        lds[0][6][threadIdx.x] = b.z, lds[0][7][threadIdx.x] = b.w;
    }
    __syncthreads();
    uint32_t h[8];
    fold(lds, cnt, groups == 1, h);
    if (threadIdx.x == 0) {
        if (groups == 1)
            store_hash(hashes + 32 * piece, h);
        else {
            uint4 *o = reinterpret_cast<uint4 *>(nodes_out + ((uint64_t)piece * groups + group) * 8);
            o[0] = make_uint4(h[0], h[1], h[2], h[3]);
            o[1] = make_uint4(h[4], h[5], h[6], h[7]);
        }
    }
}

// Streamed hashing (ec_upload with EC_FLAG_HASH_PIECES): the CVs of chunks
// [c0, c1) of every piece, written to cvs[piece][c][8] of pieces of nchunks
// >= 2 chunks (so no chunk is the root), one lane per chunk.  Once every range
// is in, b3_parents folds cvs level by level exactly as b3_chunks folds a
// group (pairs, an odd last node moving up).
template <bool kFast>
__global__ __launch_bounds__(kGroup) void b3_chunk_range(B3Pair pv, uint64_t c0, uint64_t c1, uint32_t groups,
                                                         uint64_t nchunks, uint32_t *cvs) {
    const uint64_t piece = blockIdx.x / groups;
    const uint64_t c = c0 + (uint64_t)(blockIdx.x % groups) * kGroup + threadIdx.x;
    if (c >= c1) return;
    const bool second = piece >= pv.split;
    const B3View &v = pv.v[second];
    const uint8_t *pb = piece_base(v, second ? piece - pv.split : piece);
    uint32_t h[8];
    chunk_cv<kFast>(v, pb, c, false, h);
    uint4 *o = reinterpret_cast<uint4 *>(cvs + (piece * nchunks + c) * 8);
    o[0] = make_uint4(h[0], h[1], h[2], h[3]);
    o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

uint64_t chunks_of(const B3View &v) { return v.piece_len ? (v.piece_len + 1023) / 1024 : 1; }
uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

}  // namespace

size_t b3_workspace_bytes(const B3View &v) {
    // two ping-pong node arrays: level 1 (ceil(chunks/256) per piece) and level 2
    const uint64_t g1 = ceil_div(chunks_of(v), kGroupChunks);
    if (g1 <= 1) return 0;
    const uint64_t g2 = ceil_div(g1, kGroup);
    return (size_t)(v.npieces * (g1 + (g2 > 1 ? g2 : 0)) * 32);
}

static B3View normalized(const B3View &view) {
    B3View v = view;
    if (v.run == 0 || v.run >= v.piece_len || v.run_stride == (int64_t)v.run) {  // contiguous pieces
        v.run = 1ull << 62;
        v.run_stride = 0;
    }
    v.run_shift = (v.run & (v.run - 1)) == 0 ? __builtin_ctzll(v.run) : -1;
    if (v.pieces_per_set == 0 || v.pieces_per_set > v.npieces) {  // one set
        v.pieces_per_set = v.npieces;
        v.set_stride = 0;
    }
    return v;
}

static bool fast_ok(const B3View &v) {
    return v.npieces == 0 || (v.run_shift >= 6 && (reinterpret_cast<uintptr_t>(v.base) & 15) == 0 &&
                              (v.piece_stride & 15) == 0 && (v.run_stride & 15) == 0 && (v.set_stride & 15) == 0);
}

hipError_t b3_launch2(const B3View &first, const B3View &second, uint8_t *hashes, void *ws, hipStream_t stream) {
    if (second.npieces && first.npieces && second.piece_len != first.piece_len) return hipErrorInvalidValue;
    B3Pair pv{{normalized(first), normalized(second)}, first.npieces};
    const uint64_t npieces = first.npieces + second.npieces;
    if (npieces == 0) return hipSuccess;
    for (const B3View &v : pv.v)
        if (v.npieces && !v.base && v.piece_len) return hipErrorInvalidValue;
    const uint64_t nchunks = chunks_of(first.npieces ? first : second);
    uint64_t groups = ceil_div(nchunks, kGroupChunks);
    if (groups > 0xFFFFFFFFull / kGroup || npieces * groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
    uint32_t *a = static_cast<uint32_t *>(ws);
    uint32_t *b = groups > 1 ? a + npieces * groups * 8 : nullptr;
    const dim3 grid((uint32_t)(npieces * groups));
    if (fast_ok(pv.v[0]) && fast_ok(pv.v[1]))
        b3_chunks<true><<<grid, kGroup, 0, stream>>>(pv, nchunks, (uint32_t)groups, a, hashes);
    else
        b3_chunks<false><<<grid, kGroup, 0, stream>>>(pv, nchunks, (uint32_t)groups, a, hashes);
    hipError_t e = hipGetLastError();
    while (e == hipSuccess && groups > 1) {
        const uint64_t next = ceil_div(groups, kGroup);
        b3_parents<<<dim3((uint32_t)(npieces * next)), kGroup, 0, stream>>>(a, (uint32_t)groups, (uint32_t)next, b,
                                                                          hashes);
        e = hipGetLastError();
        groups = next;
        uint32_t *t = a;
        a = b;
        b = t;
    }
    return e;
}

hipError_t b3_launch_chunk_range(const B3View &first, const B3View &second, uint64_t c0, uint64_t c1, uint32_t *cvs,
                                 hipStream_t stream) {
    if (second.npieces && first.npieces && second.piece_len != first.piece_len) return hipErrorInvalidValue;
    B3Pair pv{{normalized(first), normalized(second)}, first.npieces};
    const uint64_t npieces = first.npieces + second.npieces;
    const uint64_t nchunks = chunks_of(first.npieces ? first : second);
    if (npieces == 0 || c1 <= c0) return hipSuccess;
    if (nchunks < 2 || c1 > nchunks || !cvs) return hipErrorInvalidValue;
    const uint64_t groups = ceil_div(c1 - c0, kGroup);
    if (npieces * groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)(npieces * groups));
    if (fast_ok(pv.v[0]) && fast_ok(pv.v[1]))
        b3_chunk_range<true><<<grid, kGroup, 0, stream>>>(pv, c0, c1, (uint32_t)groups, nchunks, cvs);
    else
        b3_chunk_range<false><<<grid, kGroup, 0, stream>>>(pv, c0, c1, (uint32_t)groups, nchunks, cvs);
    return hipGetLastError();
}

size_t b3_fold_ws_bytes(uint64_t npieces, uint64_t nchunks) { return (size_t)(npieces * ceil_div(nchunks, kGroup) * 32); }

hipError_t b3_launch_fold(uint32_t *cvs, uint64_t npieces, uint64_t nchunks, uint8_t *hashes, void *ws,
                          hipStream_t stream) {
    if (npieces == 0) return hipSuccess;
    if (nchunks < 2) return hipErrorInvalidValue;
    uint32_t *a = cvs, *b = static_cast<uint32_t *>(ws);  // (after the first level, cvs is the scratch)
    uint64_t groups = nchunks;
    hipError_t e = hipSuccess;
    while (e == hipSuccess && groups > 1) {
        const uint64_t next = ceil_div(groups, kGroup);
        if (npieces * next > 0x7FFFFFFFull) return hipErrorInvalidValue;
        b3_parents<<<dim3((uint32_t)(npieces * next)), kGroup, 0, stream>>>(a, (uint32_t)groups, (uint32_t)next, b,
                                                                          hashes);
        e = hipGetLastError();
        groups = next;
        uint32_t *t = a;
        a = b;
        b = t;
    }
    return e;
}

hipError_t b3_launch(const B3View &v, uint8_t *hashes, void *ws, hipStream_t stream) {
    B3View none{};
    return b3_launch2(v, none, hashes, ws, stream);
}

}  // namespace uplink_ec
