// Developer experiment (not product): the encode's HBM access pattern alone
// (no LDS, no GF arithmetic), varying the tile shape and the tile->workgroup
// mapping, to find the layout of work that the HBM write path likes best.
// Reads 29 x (S stripes x 256 B) per tile from the stripe-major segment,
// writes S*256 B into each of the 80 pieces (data pieces = copies, parity =
// XOR-fold of the inputs).  RS(29,80), 8 x 64 MiB segments.
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

template <bool NT>
__device__ __forceinline__ v4 ld(const v4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4 *p, v4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// S stripes per tile; the block has S*16 column lanes x H row groups.
// MAP 0: grid-stride over tiles; 1: each block a contiguous range of tiles.
template <int S, int H, int MAP, bool NT>
__global__ __launch_bounds__(S * 16 * H) void enc_shape(const uint8_t *segs, uint8_t *pieces, int nseg) {
    const int tps = (NSTR + S - 1) / S;
    const int64_t tiles = (int64_t)tps * nseg;
    const int c = threadIdx.x % (S * 16), h = threadIdx.x / (S * 16);
    int64_t t0, t1, step;
    if (MAP == 0) {
        t0 = blockIdx.x; t1 = tiles; step = gridDim.x;
    } else {
        const int64_t per = (tiles + gridDim.x - 1) / gridDim.x;
        t0 = blockIdx.x * per; t1 = t0 + per < tiles ? t0 + per : tiles; step = 1;
    }
    for (int64_t t = t0; t < t1; t += step) {
        const int64_t sg = t / tps, tt = t - sg * tps;
        const int64_t s = tt * S + c / 16;
        if (s >= NSTR) continue;
        const int col = (c % 16) * 16;
        const uint8_t *in = segs + sg * SPAD + s * (K * ESS) + col;
        uint8_t *out = pieces + sg * PLEN * N + s * ESS + col;
        v4 acc = {0, 0, 0, 0};
        for (int j = h; j < K; j += H) {
            const v4 x = ld<NT>((const v4 *)(in + j * ESS));
            acc ^= x;
            st<NT>((v4 *)(out + j * PLEN), x);
        }
        for (int r = h; r < N - K; r += H) st<NT>((v4 *)(out + (K + r) * PLEN), acc ^ (uint32_t)r);
    }
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0, cus = 0;
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
        printf("%-44s %8.1f us/8seg %6.1f us/seg %6.3f TB/s\n", name, us, us / nseg, bytes / us / 1e6);
        fflush(stdout);
    };
    char nm[128];
#define E(S, H, MAP, NT, G)                                                                       \
    snprintf(nm, 128, "S=%d H=%d map=%d nt=%d grid=%dx", S, H, MAP, NT, G);                      \
    timeit(nm, [&] { hipLaunchKernelGGL((enc_shape<S, H, MAP, NT>), dim3(cus * G), dim3(S * 16 * H), 0, 0, segs, pieces, nseg); });
    E(8, 2, 0, 1, 2) E(8, 2, 0, 1, 1) E(8, 2, 0, 1, 4) E(8, 4, 0, 1, 1) E(8, 4, 0, 1, 2)
    E(8, 2, 1, 1, 1) E(8, 2, 1, 1, 2) E(8, 4, 1, 1, 1)
    E(16, 2, 0, 1, 1) E(16, 2, 0, 1, 2) E(16, 4, 0, 1, 1) E(16, 2, 1, 1, 1)
    E(32, 1, 0, 1, 1) E(32, 2, 0, 1, 1) E(32, 2, 0, 1, 2) E(32, 2, 1, 1, 1)
    E(64, 1, 0, 1, 1) E(64, 1, 1, 1, 1)
    E(8, 2, 0, 0, 2) E(16, 2, 0, 0, 1) E(32, 2, 0, 0, 1)
    E(4, 4, 0, 1, 2) E(4, 4, 0, 1, 4) E(4, 2, 0, 1, 8)
    return 0;
}
