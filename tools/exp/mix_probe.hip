// Developer experiment (not product): which shape of the encode's HBM traffic
// (29 x 256-B share reads per stripe, 80 piece streams written) moves the
// most bytes on MI355X?  No GF arithmetic: every piece row is the XOR of the
// tile's inputs (plus the row number), so the compiler keeps every load.
// Sweeps stripes per tile (TS = output run per piece per tile = TS*256 B),
// the piece pitch (padding between pieces) and the load / store policy.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4 ld(const uint8_t *p) {
    if constexpr (NT) return __builtin_nontemporal_load((const v4 *)p);
    else return *(const v4 *)p;
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t *p, v4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (v4 *)p);
    else *(v4 *)p = v;
}

constexpr int K = 29, N = 80, ESS = 256, NSTRIPES = 9040;

// one thread per 16-B chunk of a tile of TS stripes (blockDim = TS*16)
template <int TS, bool NTL, bool NTS>
__global__ void enc_shape(const uint8_t *segs, uint8_t *pieces, int64_t pitch, int nseg, int64_t spad) {
    constexpr int tiles_per_seg = (NSTRIPES + TS - 1) / TS;
    const int64_t tiles = (int64_t)tiles_per_seg * nseg;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t sg = t / tiles_per_seg, tt = t - sg * tiles_per_seg;
        const int q = threadIdx.x;
        const int64_t s = tt * TS + (q >> 4);
        if (s >= NSTRIPES) continue;
        const int c = (q & 15) * 16;
        const uint8_t *in = segs + sg * spad + s * (K * ESS) + c;
        uint8_t *out = pieces + sg * pitch * N + s * ESS + c;
        v4 x[K];
#pragma unroll
        for (int j = 0; j < K; j++) x[j] = ld<NTL>(in + j * ESS);
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < K; j++) {
            acc ^= x[j];
            st<NTS>(out + j * pitch, x[j]);
        }
#pragma unroll
        for (int r = 0; r < N - K; r++) st<NTS>(out + (K + r) * pitch, acc ^ (uint32_t)r);
    }
}

// plain 1:1 copy for calibration (U consecutive 1 KiB pieces per wave)
template <int U, bool NT>
__global__ void copy_k(const uint8_t *in, uint8_t *out, int64_t n16) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t chunk = (int64_t)blockDim.x * U;
    for (int64_t base = (int64_t)blockIdx.x * chunk; base < n16; base += (int64_t)gridDim.x * chunk) {
        const int64_t wb = base + (int64_t)wave * 64 * U;
        v4 t[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t i = wb + u * 64 + lane;
            t[u] = i < n16 ? ld<NT>(in + i * 16) : v4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t i = wb + u * 64 + lane;
            if (i < n16) st<NT>(out + i * 16, t[u]);
        }
    }
}

int main(int argc, char **argv) {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nseg = 16;
    const int64_t spad = (int64_t)NSTRIPES * K * ESS, plen = (int64_t)NSTRIPES * ESS;
    const int64_t max_pitch = plen + 65536;
    uint8_t *A, *B;
    CK(hipMalloc(&A, spad * nseg));
    CK(hipMalloc(&B, max_pitch * N * nseg));
    CK(hipMemset(A, 0x5a, spad * nseg));
    CK(hipMemset(B, 0x33, max_pitch * N * nseg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double enc_bytes = (double)spad * nseg * (1.0 + (double)N / K);
    auto timeit = [&](const char *name, double bytes, auto launch) {
        for (int i = 0; i < 5; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-52s %9.1f us  %6.3f TB/s\n", name, us, bytes / us / 1e6);
        fflush(stdout);
    };
    char nm[128];
    const int64_t n16 = spad * nseg / 16;  // copy A (its whole size) into B
    for (int g : {1, 2, 4}) {
        snprintf(nm, sizeof nm, "copy U4 nt grid=%dx bs=256", g);
        timeit(nm, n16 * 32.0, [&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(cus * g), dim3(256), 0, 0, A, B, n16); });
        snprintf(nm, sizeof nm, "copy U8 plain grid=%dx bs=512", g);
        timeit(nm, n16 * 32.0, [&] { hipLaunchKernelGGL((copy_k<8, false>), dim3(cus * g), dim3(512), 0, 0, A, B, n16); });
    }
#define ENC(TS, NTL, NTS, G, PAD)                                                                              \
    snprintf(nm, sizeof nm, "enc TS=%d ntl=%d nts=%d grid=%dx pad=%d", TS, NTL, NTS, G, PAD);                  \
    timeit(nm, enc_bytes, [&] {                                                                                \
        hipLaunchKernelGGL((enc_shape<TS, NTL, NTS>), dim3(cus * G), dim3(TS * 16), 0, 0, A, B,                \
                           (int64_t)(plen + PAD), nseg, spad);                                                 \
    });
    ENC(8, 1, 1, 2, 0) ENC(8, 1, 1, 4, 0) ENC(8, 1, 1, 8, 0) ENC(8, 0, 0, 4, 0) ENC(8, 1, 0, 4, 0)
    ENC(16, 1, 1, 2, 0) ENC(16, 1, 1, 4, 0) ENC(16, 0, 0, 2, 0)
    ENC(32, 1, 1, 1, 0) ENC(32, 1, 1, 2, 0) ENC(32, 0, 0, 1, 0)
    ENC(64, 1, 1, 1, 0)
    ENC(8, 1, 1, 4, 256) ENC(8, 1, 1, 4, 1024) ENC(8, 1, 1, 4, 2048) ENC(8, 1, 1, 4, 4096) ENC(8, 1, 1, 4, 12288)
    ENC(32, 1, 1, 1, 256) ENC(32, 1, 1, 1, 4096)
    return 0;
}
