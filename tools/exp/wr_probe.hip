// Developer experiment (not product): write-bandwidth shapes on MI355X.
// The encode kernel writes 2.76 bytes for every byte it reads, so the HBM
// write rate sets its ceiling.  Sweeps grid, block size, unroll, store
// policy and per-wave contiguity of pure streaming stores.
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

// POL 0 plain, 1 nontemporal, 2 sc1 (write-through, agent relaxed atomic store of 16B not possible: use asm)
template <int POL>
__device__ __forceinline__ void st(v4 *p, v4 v) {
    if constexpr (POL == 0) *p = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

// grid-stride: element i = one 16 B lane store; U independent stores per iteration
// spaced by the grid stride (SPREAD=1) or adjacent per wave (SPREAD=0: a wave
// writes U KiB contiguous).
template <int POL, int U, int SPREAD>
__global__ void wr_kernel(v4 *out, int64_t n) {
    const int64_t T = (int64_t)gridDim.x * blockDim.x;
    if constexpr (SPREAD) {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += T * U) {
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i + u * T < n) st<POL>(out + i + u * T, v4{(uint32_t)i, 1u, 2u, (uint32_t)u});
        }
    } else {
        // block b handles chunks of blockDim*U elements; within a wave, U consecutive 1 KiB pieces
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
        const int64_t chunk = (int64_t)blockDim.x * U;
        for (int64_t base = (int64_t)blockIdx.x * chunk; base < n; base += (int64_t)gridDim.x * chunk) {
            const int64_t wb = base + (int64_t)wave * 64 * U;
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int64_t i = wb + u * 64 + lane;
                if (i < n) st<POL>(out + i, v4{(uint32_t)i, 1u, 2u, (uint32_t)u});
            }
            (void)nw;
        }
    }
}

// 80 streams (pieces of 2,314,240 B): a block writes 2 KiB into each of R
// pieces per tile (like encode), or 8 KiB runs (4 tiles merged).
template <int POL, int RUN>
__global__ void pieces_kernel(uint8_t *out, int64_t plen, int npieces, int64_t nseg) {
    // one tile = RUN bytes of every piece; tiles per seg = plen / RUN
    const int64_t tps = plen / RUN;
    const int64_t tiles = tps * nseg;
    const int per_piece_lanes = RUN / 16;  // lanes needed per piece
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t sg = t / tps, tt = t - sg * tps;
        uint8_t *o = out + sg * plen * npieces + tt * RUN;
        for (int idx = threadIdx.x; idx < per_piece_lanes * npieces; idx += blockDim.x) {
            const int p = idx / per_piece_lanes, c = idx - p * per_piece_lanes;
            st<POL>((v4 *)(o + p * plen + c * 16), v4{(uint32_t)t, (uint32_t)p, 2u, 3u});
        }
    }
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t plen = 9040LL * 256;
    const int nseg = 8;
    const int64_t bytes = plen * 80 * nseg;  // 1.48 GB: the pieces of one encode launch
    const int64_t n = bytes / 16;
    v4 *B;
    CK(hipMalloc(&B, bytes + 4096));
    CK(hipMemset(B, 0x33, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        if (only >= 0 && vidx++ != only) return;
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-48s %9.1f us  %6.3f TB/s\n", name, us, bytes / us / 1e6);
        fflush(stdout);
    };
    char nm[128];
#define W(POL, U, SP, G, BS)                                                                             \
    snprintf(nm, 128, "write pol=%d U=%d spread=%d grid=%dx bs=%d", POL, U, SP, G, BS);                 \
    timeit(nm, [&] { hipLaunchKernelGGL((wr_kernel<POL, U, SP>), dim3(cus * G), dim3(BS), 0, 0, B, n); });
    W(0, 1, 1, 1, 256) W(0, 1, 1, 2, 256) W(0, 1, 1, 4, 256) W(0, 1, 1, 8, 256) W(0, 1, 1, 16, 256)
    W(1, 1, 1, 4, 256) W(2, 1, 1, 4, 256) W(3, 1, 1, 4, 256)
    W(0, 4, 0, 1, 256) W(0, 4, 0, 2, 256) W(0, 4, 0, 4, 256) W(1, 4, 0, 2, 256) W(2, 4, 0, 2, 256)
    W(0, 8, 0, 1, 512) W(0, 8, 0, 2, 512) W(1, 8, 0, 1, 512) W(2, 8, 0, 1, 512)
    W(0, 16, 0, 1, 256) W(1, 16, 0, 1, 256) W(2, 16, 0, 1, 256) W(0, 16, 0, 2, 1024)
    W(0, 1, 1, 1, 1024) W(0, 1, 1, 2, 1024)
#define P(POL, RUN, G, BS)                                                                                \
    snprintf(nm, 128, "pieces pol=%d run=%d grid=%dx bs=%d", POL, RUN, G, BS);                            \
    timeit(nm, [&] { hipLaunchKernelGGL((pieces_kernel<POL, RUN>), dim3(cus * G), dim3(BS), 0, 0, (uint8_t *)B, plen, 80, (int64_t)nseg); });
    P(0, 2048, 1, 512) P(1, 2048, 1, 512) P(2, 2048, 1, 512) P(0, 2048, 2, 256) P(1, 2048, 4, 256)
    P(0, 4096, 1, 512) P(1, 4096, 1, 512) P(1, 8192, 1, 512) P(0, 8192, 1, 1024)
    P(1, 1024, 2, 256) P(1, 512, 4, 256)
    return 0;
}
