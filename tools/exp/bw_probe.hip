// Developer experiment (not product): what HBM rate does this box give for
// the byte mixes of the encode (1 read : 2.76 write) and rebuild (1 : 1)
// kernels?  Plain streaming kernels, no GF arithmetic.  Bytes are counted as
// read + written; sizes are one encode launch of 8 RS(29,80) 64 MiB segments.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

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

// read-only: xor-reduce to keep loads alive
template <bool NT, int U>
__global__ void rd_kernel(const v4 *in, int64_t n, v4 *sink) {
    v4 acc = {0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
        v4 t[U];
#pragma unroll
        for (int u = 0; u < U; u++) t[u] = (i + u * stride < n) ? ld<NT>(in + i + u * stride) : v4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= t[u];
    }
    if (acc.x == 0x12345678u) sink[0] = acc;
}

template <bool NT, int U>
__global__ void wr_kernel(v4 *out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i + u * stride < n) st<NT>(out + i + u * stride, v4{(uint32_t)i, 1u, 2u, (uint32_t)u});
    }
}

template <bool NT, int U>
__global__ void copy_kernel(const v4 *in, v4 *out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * U) {
        v4 t[U];
#pragma unroll
        for (int u = 0; u < U; u++) t[u] = (i + u * stride < n) ? ld<NT>(in + i + u * stride) : v4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; u++)
            if (i + u * stride < n) st<NT>(out + i + u * stride, t[u]);
    }
}

// 1 read : W writes into W separate output arrays (like encode's pieces)
template <bool NT, int W>
__global__ void fanout_kernel(const v4 *in, v4 *out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const v4 t = ld<NT>(in + i);
#pragma unroll
        for (int w = 0; w < W; w++) st<NT>(out + w * n + i, t ^ (uint32_t)w);
    }
}

// encode-shaped: a workgroup takes a 2048-column tile: reads 29 x 2 KiB
// (8 stripes x 256 B of each share, stripe stride 7424 B), writes 80 x 2 KiB
// runs (one per piece, piece length plen).  No LDS, data just XOR-folded.
template <bool NT>
__global__ __launch_bounds__(256) void encshape_kernel(const uint8_t *seg, uint8_t *pieces, int64_t tiles,
                                                       int64_t tiles_per_seg, int64_t spad, int64_t plen) {
    const int lane = threadIdx.x;  // 256 threads x 16 B = 4 KiB; two tiles' worth per pass? no: 2 KiB = 128 lanes
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t sg = t / tiles_per_seg, tt = t - sg * tiles_per_seg;
        const uint8_t *in = seg + sg * spad;
        uint8_t *out = pieces + sg * plen * 80;
        const int c = lane & 127;   // 16-B chunk within the tile
        const int half = lane >> 7; // two halves split inputs / outputs
        const int64_t q = tt * 128 + c;
        const int64_t s = q / 16, tcol = (q % 16) * 16;
        v4 acc = {0, 0, 0, 0};
        if (s < 9040) {
            for (int j = half; j < 29; j += 2) {
                const v4 x = ld<NT>((const v4 *)(in + s * 7424 + j * 256 + tcol));
                acc ^= x;
                st<NT>((v4 *)(out + j * plen + s * 256 + tcol), x);
            }
            for (int r = half; r < 51; r += 2) st<NT>((v4 *)(out + (29 + r) * plen + s * 256 + tcol), acc ^ (uint32_t)r);
        }
    }
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t spad = 9040LL * 7424, plen = 9040LL * 256;
    const int nseg = 8;
    const double enc_bytes = (double)spad * nseg * (1.0 + 80.0 / 29.0);
    const int64_t big = (int64_t)(enc_bytes / 16) + 1024;  // v4 elements
    v4 *A, *B;
    CK(hipMalloc(&A, big * 16));
    CK(hipMalloc(&B, big * 16 * 2));
    CK(hipMemset(A, 0x5a, big * 16));
    CK(hipMemset(B, 0x33, big * 16 * 2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, double bytes, auto launch) {
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
        printf("%-44s %9.1f us  %6.3f TB/s\n", name, us, bytes / us / 1e6);
        fflush(stdout);
    };
    char nm[96];
    const int64_t n_rw = (int64_t)(enc_bytes / 2 / 16);
    for (int g : {2, 4, 8}) {
        snprintf(nm, 96, "read  U4 grid=%dx plain", g);
        timeit(nm, n_rw * 16.0, [&] { hipLaunchKernelGGL((rd_kernel<false, 4>), dim3(cus * g), dim3(256), 0, 0, A, n_rw, B); });
        snprintf(nm, 96, "read  U4 grid=%dx nt", g);
        timeit(nm, n_rw * 16.0, [&] { hipLaunchKernelGGL((rd_kernel<true, 4>), dim3(cus * g), dim3(256), 0, 0, A, n_rw, B); });
        snprintf(nm, 96, "write U4 grid=%dx plain", g);
        timeit(nm, n_rw * 16.0, [&] { hipLaunchKernelGGL((wr_kernel<false, 4>), dim3(cus * g), dim3(256), 0, 0, B, n_rw); });
        snprintf(nm, 96, "write U4 grid=%dx nt", g);
        timeit(nm, n_rw * 16.0, [&] { hipLaunchKernelGGL((wr_kernel<true, 4>), dim3(cus * g), dim3(256), 0, 0, B, n_rw); });
        snprintf(nm, 96, "copy  U4 grid=%dx plain", g);
        timeit(nm, n_rw * 32.0, [&] { hipLaunchKernelGGL((copy_kernel<false, 4>), dim3(cus * g), dim3(256), 0, 0, A, B, n_rw); });
        snprintf(nm, 96, "copy  U4 grid=%dx nt", g);
        timeit(nm, n_rw * 32.0, [&] { hipLaunchKernelGGL((copy_kernel<true, 4>), dim3(cus * g), dim3(256), 0, 0, A, B, n_rw); });
        const int64_t nf = (int64_t)(enc_bytes / 4 / 16);
        snprintf(nm, 96, "fanout 1r:3w grid=%dx plain", g);
        timeit(nm, nf * 64.0, [&] { hipLaunchKernelGGL((fanout_kernel<false, 3>), dim3(cus * g), dim3(256), 0, 0, A, B, nf); });
        snprintf(nm, 96, "fanout 1r:3w grid=%dx nt", g);
        timeit(nm, nf * 64.0, [&] { hipLaunchKernelGGL((fanout_kernel<true, 3>), dim3(cus * g), dim3(256), 0, 0, A, B, nf); });
        const int64_t tps = (9040LL * 16 + 127) / 128;
        snprintf(nm, 96, "encode-shaped (no LDS) grid=%dx plain", g);
        timeit(nm, enc_bytes, [&] {
            hipLaunchKernelGGL((encshape_kernel<false>), dim3(cus * g), dim3(256), 0, 0, (const uint8_t *)A, (uint8_t *)B,
                               tps * nseg, tps, spad, plen);
        });
        snprintf(nm, 96, "encode-shaped (no LDS) grid=%dx nt", g);
        timeit(nm, enc_bytes, [&] {
            hipLaunchKernelGGL((encshape_kernel<true>), dim3(cus * g), dim3(256), 0, 0, (const uint8_t *)A, (uint8_t *)B,
                               tps * nseg, tps, spad, plen);
        });
    }
    return 0;
}
