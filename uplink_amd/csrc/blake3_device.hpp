// BLAKE3 device primitives shared by the piece-hash kernels (blake3.hip)
// and the experiments under tools/exp/.  Algorithm: BLAKE3 paper §2
// (restated on the CPU in oracle/blake3_oracle.c).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace uplink_ec {
namespace b3 {

constexpr uint32_t kChunkStart = 1, kChunkEnd = 2, kParent = 4, kRoot = 8;
constexpr int kGroup = 256;  // chunks (or nodes) folded per workgroup (256 measured best)
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

}  // namespace b3
}  // namespace uplink_ec
