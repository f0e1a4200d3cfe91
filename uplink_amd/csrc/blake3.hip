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

namespace uplink_ec {
namespace {

constexpr uint32_t kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8;
constexpr int kGroup = 256;  // chunks (or nodes) folded per workgroup
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                        0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

// message word schedule: kSched[r][i] = index of the word used in slot i of
// round r (the fixed permutation applied r times)
struct Sched {
    uint8_t s[7][16];
    constexpr Sched() : s{} {
        constexpr uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
        for (int i = 0; i < 16; i++) s[0][i] = (uint8_t)i;
        for (int r = 1; r < 7; r++)
            for (int i = 0; i < 16; i++) s[r][i] = s[r - 1][perm[i]];
    }
};
constexpr Sched kSched{};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

__device__ __forceinline__ void G(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t x, uint32_t y) {
    a = a + b + x;
    d = rotr(d ^ a, 16);
    c = c + d;
    b = rotr(b ^ c, 12);
    a = a + b + y;
    d = rotr(d ^ a, 8);
    c = c + d;
    b = rotr(b ^ c, 7);
}

// h <- first 8 words of compress(h, m, counter, blen, flags) (the new CV, or
// the 32-byte hash when flags has ROOT)
__device__ __forceinline__ void compress(uint32_t (&h)[8], const uint32_t (&m)[16], uint32_t ctr_lo, uint32_t ctr_hi,
                                         uint32_t blen, uint32_t flags) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = h[i];
#pragma unroll
    for (int i = 0; i < 4; i++) v[8 + i] = kIV[i];
    v[12] = ctr_lo;
    v[13] = ctr_hi;
    v[14] = blen;
    v[15] = flags;
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint8_t *s = kSched.s[r];
        G(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
        G(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
        G(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
        G(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
        G(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
        G(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
        G(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
        G(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = v[i] ^ v[i + 8];
}

__device__ __forceinline__ void parent(uint32_t (&h)[8], const uint32_t (&l)[8], const uint32_t (&r)[8], bool root) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        m[i] = l[i];
        m[8 + i] = r[i];
        h[i] = kIV[i];
    }
    compress(h, m, 0, 0, 64, kParent | (root ? kRoot : 0));
}

// byte address of byte t of piece j
template <bool kFast>
__device__ __forceinline__ const uint8_t *at(const B3View &v, uint64_t j, uint64_t t) {
    if (kFast)  // power-of-two runs: no 64-bit division
        return v.base + (int64_t)j * v.piece_stride + (int64_t)(t >> v.run_shift) * v.run_stride + (t & (v.run - 1));
    return v.base + (int64_t)j * v.piece_stride + (int64_t)(t / v.run) * v.run_stride + (t % v.run);
}

// 64-byte block starting at byte t of piece j, `len` valid bytes (zero padded)
template <bool kFast>
__device__ __forceinline__ void load_block(const B3View &v, uint64_t j, uint64_t t, uint32_t len, uint32_t (&m)[16]) {
    if (kFast && len == 64) {  // the block lies in one run, 16-byte aligned
        const u32x4 *p = reinterpret_cast<const u32x4 *>(at<kFast>(v, j, t));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            u32x4 w = __builtin_nontemporal_load(p + q);
            m[4 * q] = w[0], m[4 * q + 1] = w[1], m[4 * q + 2] = w[2], m[4 * q + 3] = w[3];
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = 0;
    for (uint32_t b = 0; b < len; b++) m[b >> 2] |= (uint32_t)*at<kFast>(v, j, t + b) << (8 * (b & 3));
}

__device__ __forceinline__ void store_hash(uint8_t *out, const uint32_t (&h)[8]) {
    uint4 *o = reinterpret_cast<uint4 *>(out);
    o[0] = make_uint4(h[0], h[1], h[2], h[3]);
    o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

// Folds `cnt` nodes held in lds[0] (layout [word][kGroup]) into one.  If
// `whole` (the nodes are every node of the piece), the last parent is the
// root and the function returns with the hash in `out` of thread 0; else
// thread 0 gets the subtree CV.  cnt >= 2 when whole.
__device__ void fold(uint32_t (*lds)[8][kGroup], int cnt, bool whole, uint32_t (&out)[8]) {
    const int t = threadIdx.x;
    int cur = 0;
    while (cnt > 1) {
        const int pairs = cnt >> 1;
        if (t < pairs) {
            uint32_t l[8], r[8], h[8];
#pragma unroll
            for (int i = 0; i < 8; i++) l[i] = lds[cur][i][2 * t], r[i] = lds[cur][i][2 * t + 1];
            parent(h, l, r, whole && cnt == 2);
#pragma unroll
            for (int i = 0; i < 8; i++) lds[cur ^ 1][i][t] = h[i];
        } else if (t == pairs && (cnt & 1)) {
#pragma unroll
            for (int i = 0; i < 8; i++) lds[cur ^ 1][i][t] = lds[cur][i][cnt - 1];
        }
        __syncthreads();
        cnt = (cnt + 1) >> 1;
        cur ^= 1;
    }
    if (t == 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) out[i] = lds[cur][i][0];
    }
}

template <bool kFast>
__global__ __launch_bounds__(kGroup) void b3_chunks(B3View v, uint64_t nchunks, uint32_t groups, uint32_t *nodes,
                                                     uint8_t *hashes) {
    __shared__ uint32_t lds[2][8][kGroup];
    const uint64_t piece = blockIdx.x / groups;
    const uint32_t group = blockIdx.x % groups;
    const uint64_t c = (uint64_t)group * kGroup + threadIdx.x;
    const bool single = nchunks == 1;
    if (c < nchunks) {
        const uint64_t t0 = c * 1024;
        const uint64_t clen = v.piece_len - t0 < 1024 ? v.piece_len - t0 : 1024;  // 0 only for an empty piece
        const uint32_t nb = clen ? (uint32_t)((clen + 63) >> 6) : 1;
        uint32_t h[8];
#pragma unroll
        for (int i = 0; i < 8; i++) h[i] = kIV[i];
        uint32_t m[16], nx[16];
        load_block<kFast>(v, piece, t0, nb == 1 ? (uint32_t)clen : 64, m);
        for (uint32_t b = 0; b < nb; b++) {
            const bool last = b + 1 == nb;
            const uint32_t blen = last ? (uint32_t)(clen - 64ull * b) : 64;
            if (!last) {  // prefetch the next block while this one compresses
                const uint32_t nlen = b + 2 == nb ? (uint32_t)(clen - 64ull * (b + 1)) : 64;
                load_block<kFast>(v, piece, t0 + 64ull * (b + 1), nlen, nx);
            }
            const uint32_t flags = (b == 0 ? kChunkStart : 0) | (last ? kChunkEnd : 0) | (last && single ? kRoot : 0);
            compress(h, m, (uint32_t)c, (uint32_t)(c >> 32), blen, flags);
            if (!last) {
#pragma unroll
                for (int i = 0; i < 16; i++) m[i] = nx[i];
            }
        }
        if (single) {
            store_hash(hashes + 32 * piece, h);
            return;  // the only lane of a one-chunk piece
        }
#pragma unroll
        for (int i = 0; i < 8; i++) lds[0][i][threadIdx.x] = h[i];
    }
    if (single) return;
    __syncthreads();
    const uint64_t left = nchunks - (uint64_t)group * kGroup;
    const int cnt = left < kGroup ? (int)left : kGroup;
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

uint64_t chunks_of(const B3View &v) { return v.piece_len ? (v.piece_len + 1023) / 1024 : 1; }
uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

}  // namespace

size_t b3_workspace_bytes(const B3View &v) {
    // two ping-pong node arrays: level 1 (ceil(chunks/256) per piece) and level 2
    const uint64_t g1 = ceil_div(chunks_of(v), kGroup);
    if (g1 <= 1) return 0;
    const uint64_t g2 = ceil_div(g1, kGroup);
    return (size_t)(v.npieces * (g1 + (g2 > 1 ? g2 : 0)) * 32);
}

hipError_t b3_launch(const B3View &view, uint8_t *hashes, void *ws, hipStream_t stream) {
    if (view.npieces == 0) return hipSuccess;
    if (!view.base && view.piece_len) return hipErrorInvalidValue;
    B3View v = view;
    if (v.run == 0 || v.run >= v.piece_len || v.run_stride == (int64_t)v.run) {  // contiguous pieces
        v.run = 1ull << 62;
        v.run_stride = 0;
    }
    v.run_shift = (v.run & (v.run - 1)) == 0 ? __builtin_ctzll(v.run) : -1;
    const uint64_t nchunks = chunks_of(v);
    uint64_t groups = ceil_div(nchunks, kGroup);
    if (groups > 0xFFFFFFFFull / kGroup || v.npieces * groups > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const bool aligned = v.run_shift >= 6 && (reinterpret_cast<uintptr_t>(v.base) & 15) == 0 &&
                         (v.piece_stride & 15) == 0 && (v.run_stride & 15) == 0;
    uint32_t *a = static_cast<uint32_t *>(ws);
    uint32_t *b = groups > 1 ? a + v.npieces * groups * 8 : nullptr;
    const dim3 grid((uint32_t)(v.npieces * groups));
    if (aligned)
        b3_chunks<true><<<grid, kGroup, 0, stream>>>(v, nchunks, (uint32_t)groups, a, hashes);
    else
        b3_chunks<false><<<grid, kGroup, 0, stream>>>(v, nchunks, (uint32_t)groups, a, hashes);
    hipError_t e = hipGetLastError();
    while (e == hipSuccess && groups > 1) {
        const uint64_t next = ceil_div(groups, kGroup);
        b3_parents<<<dim3((uint32_t)(v.npieces * next)), kGroup, 0, stream>>>(a, (uint32_t)groups, (uint32_t)next, b,
                                                                            hashes);
        e = hipGetLastError();
        groups = next;
        uint32_t *t = a;
        a = b;
        b = t;
    }
    return e;
}

}  // namespace uplink_ec
