// Experiment: where does the BLAKE3 chunk kernel's time go?  Chunk CVs of
// 640 contiguous pieces of 2,314,240 B (8 RS(29,80) segments' pieces),
// one lane per 1 KiB chunk, CVs written to global (no tree fold).
//   mode 0  64-B block per step, non-temporal loads (product as first written)
//   mode 1  64-B block per step, plain loads
//   mode 2  128-B line per step (two blocks), plain loads
//   mode 3  compute only (message words from registers, no loads)
//   mode 4  loads only (64-B steps, XOR-reduced), no compression
//   mode 5  128-B line per step, non-temporal loads
//   mode 6  compute only, two chunks per lane interleaved G by G (ILP 8)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 b3_probe.hip -o b3_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../uplink_amd/csrc/blake3_device.hpp"

using namespace uplink_ec::b3;
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

template <bool NT>
__device__ __forceinline__ void ld16(const uint8_t *p, uint32_t *m) {
    const u32x4v *q = reinterpret_cast<const u32x4v *>(p);
    u32x4v w = NT ? __builtin_nontemporal_load(q) : *q;
    m[0] = w[0], m[1] = w[1], m[2] = w[2], m[3] = w[3];
}

// two independent compressions interleaved G by G
__device__ __forceinline__ void compress2(uint32_t (&h)[8], const uint32_t (&m)[16], uint32_t (&h2)[8],
                                          const uint32_t (&m2)[16], uint32_t ctr, uint32_t flags) {
    uint32_t v[16], w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = h[i], w[i] = h2[i];
#pragma unroll
    for (int i = 0; i < 4; i++) v[8 + i] = w[8 + i] = kIV[i];
    v[12] = w[12] = ctr;
    v[13] = w[13] = 0;
    v[14] = w[14] = 64;
    v[15] = w[15] = flags;
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint8_t *s = kSched.s[r];
#define GG(A, B, C, D, X, Y) G(v[A], v[B], v[C], v[D], m[s[X]], m[s[Y]]); G(w[A], w[B], w[C], w[D], m2[s[X]], m2[s[Y]]);
        GG(0, 4, 8, 12, 0, 1) GG(1, 5, 9, 13, 2, 3) GG(2, 6, 10, 14, 4, 5) GG(3, 7, 11, 15, 6, 7)
        GG(0, 5, 10, 15, 8, 9) GG(1, 6, 11, 12, 10, 11) GG(2, 7, 8, 13, 12, 13) GG(3, 4, 9, 14, 14, 15)
#undef GG
    }
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = v[i] ^ v[i + 8], h2[i] = w[i] ^ w[i + 8];
}

template <int MODE>
__global__ __launch_bounds__(256) void chunks(const uint8_t *base, uint64_t nchunks, uint32_t *cvs) {
    const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= nchunks) return;
    const uint8_t *p = base + c * 1024;
    uint32_t h[8];
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = kIV[i];
    if constexpr (MODE == 0 || MODE == 1) {
        uint32_t m[16], nx[16];
#pragma unroll
        for (int q = 0; q < 4; q++) ld16<MODE == 0>(p + 16 * q, m + 4 * q);
        for (int b = 0; b < 16; b++) {
            if (b < 15)
#pragma unroll
                for (int q = 0; q < 4; q++) ld16<MODE == 0>(p + 64 * (b + 1) + 16 * q, nx + 4 * q);
            compress(h, m, (uint32_t)c, 0, 64, (b == 0 ? kChunkStart : 0) | (b == 15 ? kChunkEnd : 0));
#pragma unroll
            for (int i = 0; i < 16; i++) m[i] = nx[i];
        }
    } else if constexpr (MODE == 2 || MODE == 5) {
        uint32_t m[32], nx[32];
#pragma unroll
        for (int q = 0; q < 8; q++) ld16<MODE == 5>(p + 16 * q, m + 4 * q);
        for (int pr = 0; pr < 8; pr++) {
            if (pr < 7)
#pragma unroll
                for (int q = 0; q < 8; q++) ld16<MODE == 5>(p + 128 * (pr + 1) + 16 * q, nx + 4 * q);
            uint32_t a[16], b2[16];
#pragma unroll
            for (int i = 0; i < 16; i++) a[i] = m[i], b2[i] = m[16 + i];
            compress(h, a, (uint32_t)c, 0, 64, pr == 0 ? kChunkStart : 0);
            compress(h, b2, (uint32_t)c, 0, 64, pr == 7 ? kChunkEnd : 0);
#pragma unroll
            for (int i = 0; i < 32; i++) m[i] = nx[i];
        }
    } else if constexpr (MODE == 3) {
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = (uint32_t)c * 0x9E3779B9u + i;
        for (int b = 0; b < 16; b++) {
            compress(h, m, (uint32_t)c, 0, 64, (b == 0 ? kChunkStart : 0) | (b == 15 ? kChunkEnd : 0));
            m[b & 15] ^= h[b & 7];
        }
    } else if constexpr (MODE == 6) {  // compute only, two chunks per lane interleaved (ILP 8)
        uint32_t m[16], m2[16], h2[8];
#pragma unroll
        for (int i = 0; i < 8; i++) h2[i] = kIV[i];
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = (uint32_t)c * 0x9E3779B9u + i, m2[i] = (uint32_t)c * 0x7F4A7C15u + i;
        for (int b = 0; b < 16; b++) {
            compress2(h, m, h2, m2, (uint32_t)c, (b == 0 ? kChunkStart : 0) | (b == 15 ? kChunkEnd : 0));
            m[b & 15] ^= h[b & 7];
            m2[b & 15] ^= h2[b & 7];
        }
#pragma unroll
        for (int i = 0; i < 8; i++) h[i] ^= h2[i];
    } else {
        uint32_t m[16];
        for (int b = 0; b < 16; b++) {
#pragma unroll
            for (int q = 0; q < 4; q++) ld16<false>(p + 64 * b + 16 * q, m + 4 * q);
#pragma unroll
            for (int i = 0; i < 8; i++) h[i] ^= m[i] ^ m[i + 8];
        }
    }
    uint4 *o = reinterpret_cast<uint4 *>(cvs + c * 8);
    o[0] = make_uint4(h[0], h[1], h[2], h[3]);
    o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

template <int MODE>
float run(const uint8_t *d, uint64_t nchunks, uint32_t *cvs, int iters) {
    dim3 grid((unsigned)((nchunks + 255) / 256));
    for (int i = 0; i < 20; i++) chunks<MODE><<<grid, 256>>>(d, nchunks, cvs);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; i++) chunks<MODE><<<grid, 256>>>(d, nchunks, cvs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main() {
    const uint64_t bytes = 640ull * 2314240ull, nchunks = bytes / 1024;
    uint8_t *d;
    uint32_t *cvs;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&cvs, nchunks * 32));
    CK(hipMemset(d, 0x5a, bytes));
    const int it = 20;
    float t[7] = {run<0>(d, nchunks, cvs, it), run<1>(d, nchunks, cvs, it), run<2>(d, nchunks, cvs, it),
                  run<3>(d, nchunks, cvs, it), run<4>(d, nchunks, cvs, it), run<5>(d, nchunks, cvs, it),
                  run<6>(d, nchunks / 2, cvs, it)};  // half the lanes, two chunks each: same bytes
    const char *name[7] = {"64B NT", "64B plain", "128B line plain", "compute only", "loads only", "128B line NT",
                           "compute 2/lane"};
    for (int m = 0; m < 7; m++)
        printf("mode %d %-16s %8.1f us/launch  %7.1f GB/s\n", m, name[m], t[m] * 1e3, bytes / (t[m] * 1e-3) / 1e9);
    return 0;
}
