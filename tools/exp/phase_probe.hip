// Developer experiment (not product): does separating reads and writes in
// time (chip-wide, by the global 100 MHz s_memrealtime clock) raise the HBM
// rate of the encode's byte mix?  Every workgroup issues its tile's loads
// only inside a read window [0, R) of each period P (in 10-ns ticks) and its
// stores only outside it.  Encode access pattern, no GF arithmetic.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));
constexpr int K = 29, N = 80, ESS = 256, NSTR = 9040;
constexpr int64_t SPAD = (int64_t)NSTR * K * ESS, PLEN = (int64_t)NSTR * ESS;

__device__ __forceinline__ void wait_window(uint32_t P, uint32_t lo, uint32_t hi) {
    if (P == 0) return;
    for (;;) {
        const uint32_t t = (uint32_t)(__builtin_amdgcn_s_memrealtime() % P);
        if (t >= lo && t < hi) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

// 8 stripes per tile, 128 column lanes x 2 halves (256 threads); half h
// loads inputs h, h+2, ... and stores their copies and parity rows h, h+2, ...
__global__ __launch_bounds__(256) void enc_phase(const uint8_t *segs, uint8_t *pieces, int nseg, uint32_t P,
                                                 uint32_t R) {
    const int tps = (NSTR + 7) / 8;
    const int64_t tiles = (int64_t)tps * nseg;
    const int c = threadIdx.x & 127, h = threadIdx.x >> 7;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t sg = t / tps, tt = t - sg * tps;
        const int64_t s = tt * 8 + c / 16;
        const bool ok = s < NSTR;
        const int col = (c % 16) * 16;
        const uint8_t *in = segs + sg * SPAD + (ok ? s : 0) * (K * ESS) + col;
        uint8_t *out = pieces + sg * PLEN * N + (ok ? s : 0) * ESS + col;
        v4 x[15];
        wait_window(P, 0, R);
#pragma unroll
        for (int i = 0; i < 15; i++) {
            const int j = h + 2 * i;
            x[i] = j < K ? __builtin_nontemporal_load((const v4 *)(in + j * ESS)) : v4{0, 0, 0, 0};
        }
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 15; i++) acc ^= x[i];
        wait_window(P, R, P);
        if (ok) {
#pragma unroll
            for (int i = 0; i < 15; i++) {
                const int j = h + 2 * i;
                if (j < K) __builtin_nontemporal_store(x[i], (v4 *)(out + j * PLEN));
            }
            for (int r = h; r < N - K; r += 2) __builtin_nontemporal_store(acc ^ (uint32_t)r, (v4 *)(out + (K + r) * PLEN));
        }
    }
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nseg = 8;
    uint8_t *segs, *pieces;
    CK(hipMalloc(&segs, SPAD * nseg));
    CK(hipMalloc(&pieces, PLEN * N * nseg));
    CK(hipMemset(segs, 0x5a, SPAD * nseg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)SPAD * nseg * (1.0 + (double)N / K);
    auto run = [&](int g, uint32_t P, uint32_t R) {
        auto L = [&] { hipLaunchKernelGGL(enc_phase, dim3(cus * g), dim3(256), 0, 0, segs, pieces, nseg, P, R); };
        for (int i = 0; i < 60; i++) L();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; i++) L();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / 20;
        printf("grid=%dx P=%4u R=%4u ticks  %7.1f us/8seg %6.1f us/seg %6.3f TB/s\n", g, P, R, us, us / nseg,
               bytes / us / 1e6);
        fflush(stdout);
    };
    for (int g : {2, 4}) {
        run(g, 0, 0);
        run(g, 200, 60);
        run(g, 400, 110);
        run(g, 800, 220);
        run(g, 1600, 430);
        run(g, 800, 300);
    }
    return 0;
}
