// Developer experiment (not product): does the cache policy of the vector
// stores (and loads) move the HBM rate of the encode's access pattern?  The
// encode writes every output byte once and never reads it back, so the
// policies that keep a line in the XCD's L2 (plain, sc0, nt) and those that
// drop it (sc1, sc0 sc1; MI355X_MICROARCH.md, "stores of each flavour") are
// both candidates.  Shapes: the encode's (29 reads then 80 writes of 1 KiB
// per wave block, one-shot grid and persistent 4 waves per CU) and a 1:1 copy.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 store_policy_probe.hip -o spp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

// vector global stores with an explicit cache policy
template <int P>
__device__ __forceinline__ void st(v4 *p, v4 v) {
    if constexpr (P == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
}
template <int Q>
__device__ __forceinline__ v4 ld(const v4 *p) {
    if constexpr (Q == 0) return *p;
    else if constexpr (Q == 1) return __builtin_nontemporal_load(p);
    else {
        v4 r;
        asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
        return r;
    }
}

// one-shot: each wave reads R consecutive 1 KiB blocks, writes W
template <int R, int W, int P, int Q>
__global__ __launch_bounds__(256) void mix(const v4 *in, v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    v4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t i = (wave * R + r) * 64 + lane;
        if (i < n) acc ^= ld<Q>(in + i);
    }
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int64_t i = (wave * W + w) * 64 + lane;
        if (i < n / R * W) st<P>(out + i, acc ^ (uint32_t)w);
    }
}

// persistent: the encode's piece streams (block b reads R KiB, writes 1 KiB to each of W streams)
template <int R, int W, int P>
__global__ void pieces(const v4 *in, v4 *out, int64_t nblk) {
    const int lane = threadIdx.x & 63;
    const int64_t G = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nblk; b += G) {
        v4 x[R];
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = __builtin_nontemporal_load(in + (b * R + r) * 64 + lane);
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc ^= x[r];
            st<P>(out + (r * nblk + b) * 64 + lane, x[r]);
        }
#pragma unroll
        for (int w = R; w < W; w++) st<P>(out + (w * nblk + b) * 64 + lane, acc ^ (uint32_t)w);
    }
}

int main() {
    const int64_t RB = (int64_t)1 << 30, WB = (int64_t)3 << 30;
    v4 *A, *B;
    CK(hipMalloc(&A, RB));
    CK(hipMalloc(&B, WB));
    CK(hipMemset(A, 0x5a, RB));
    CK(hipMemset(B, 0x33, WB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
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
    const int64_t n = RB / 16;
    const char *pn[] = {"plain", "nt", "sc1", "sc0 sc1", "sc0 sc1 nt", "sc1 nt", "sc0"};
    const char *qn[] = {"plain", "nt", "sc1"};
#define MIX(R, W, P, Q)                                                                              \
    {                                                                                                \
        const int64_t waves = n / 64 / (R);                                                          \
        char nm[96];                                                                                 \
        snprintf(nm, sizeof nm, "one-shot R=%d W=%d store %s load %s", R, W, pn[P], qn[Q]);          \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                     \
            hipLaunchKernelGGL((mix<R, W, P, Q>), dim3((waves + 3) / 4), dim3(256), 0, 0, A, B, n);  \
        });                                                                                          \
    }
#define PIECES(R, W, P, WPC)                                                                         \
    {                                                                                                \
        const int64_t nblk = n / 64 / (R);                                                           \
        char nm[96];                                                                                 \
        snprintf(nm, sizeof nm, "pieces R=%d W=%d store %s waves/CU=%d", R, W, pn[P], WPC);         \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                     \
            hipLaunchKernelGGL((pieces<R, W, P>), dim3(cus), dim3(64 * (WPC)), 0, 0, A, B, nblk);   \
        });                                                                                          \
    }
    MIX(29, 80, 0, 1) MIX(29, 80, 1, 1) MIX(29, 80, 2, 1) MIX(29, 80, 3, 1) MIX(29, 80, 4, 1) MIX(29, 80, 5, 1)
    MIX(29, 80, 6, 1) MIX(29, 80, 1, 0) MIX(29, 80, 2, 0)
    PIECES(29, 80, 0, 4) PIECES(29, 80, 1, 4) PIECES(29, 80, 2, 4) PIECES(29, 80, 3, 4) PIECES(29, 80, 4, 4)
    PIECES(29, 80, 5, 4) PIECES(29, 80, 6, 4)
    MIX(1, 1, 0, 1) MIX(1, 1, 1, 1) MIX(1, 1, 2, 1) MIX(1, 1, 3, 1)
    MIX(8, 8, 1, 1) MIX(8, 8, 2, 1) MIX(8, 8, 3, 1)
    return 0;
}
