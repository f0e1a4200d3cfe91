// Developer experiment (not product): timing variants of the RS(29,80)
// encode kernel to locate its bottleneck.  Build: make -C tools/exp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../uplink_amd/csrc/rs_device.hpp"

using namespace uplink_ec;
using namespace uplink_ec::dev;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// MODE 0 normal, 1 all waves run group 0 code, 2 no XOR compute, 3 copy only (no LDS, no transposes)
template <int K, int N, int NW, int MODE>
__global__ __launch_bounds__(NW * 64, 2) void enc_var(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NW - 1) / NW;
    constexpr int PER = (K + NW - 1) / NW;
    __shared__ uint32_t lds[K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const int64_t tt = tile - seg * a.tiles_per_seg;
        const TileCols c = tile_cols(a, tt, lane);
        if constexpr (MODE == 3) {
            uint4 bufA[PER], bufB[PER];
            const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (j < K) {
                    const uint8_t *p = in_seg + a.in_off[j];
                    bufA[i] = c.vA ? *(const uint4 *)(p + c.inA) : make_uint4(0, 0, 0, 0);
                    bufB[i] = c.vB ? *(const uint4 *)(p + c.inB) : make_uint4(0, 0, 0, 0);
                }
            }
            uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (j < K) {
                    uint8_t *p = out_seg + a.copy_off[j];
                    if (c.vA) *(uint4 *)(p + c.outA) = bufA[i];
                    if (c.vB) *(uint4 *)(p + c.outB) = bufB[i];
                }
            }
            const int rbase = wave * OPW;
            static_for<OPW>([&]<int O>() {
                if (rbase + O < R) {
                    uint8_t *p = out_seg + a.out_off[rbase + O];
                    if (c.vA) *(uint4 *)(p + c.outA) = bufA[O % PER];
                    if (c.vB) *(uint4 *)(p + c.outB) = bufB[O % PER];
                }
            });
            continue;
        } else {
            stage_inputs<NW, PER>(a, seg, c, lds, lane, wave, 0, K, true);
            __syncthreads();
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            if constexpr (MODE == 0) {
                static_for<NW>([&]<int W>() {
                    if (wave == W) compute_special<K, N, OPW, W>(lds, lane, acc);
                });
            } else if constexpr (MODE == 1) {
                compute_special<K, N, OPW, 0>(lds, lane, acc);
            } else {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) acc[o][p] = lds[((o % K) * 8 + p) * 64 + lane];
            }
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            store_rows<OPW>(a, seg, c, rbase, cnt, acc);
            __syncthreads();
        }
    }
}


// warp-specialised: waves 0..3 compute (rows), waves 4..7 load/transpose into a
// double-buffered LDS tile ring; one barrier per tile.
template <int K, int N, bool NT, bool NTL = false, bool RAW = false>
__global__ __launch_bounds__(512, 1) void enc_ws(const RsArgs a) {
    constexpr int NWC = 4;
    constexpr int R = N - K;
    constexpr int OPW = (R + NWC - 1) / NWC;
    constexpr int PER = (K + 3) / 4;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NWC;
    const int lw = wave - NWC;
    int64_t tile = blockIdx.x;
    if (loader && tile < a.total_tiles) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        stage_inputs<4, PER, NTL>(a, seg, c, lds[0], lane, lw, 0, K, true);
    }
    __syncthreads();
    int buf = 0;
    for (; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t next = tile + gridDim.x;
        if (loader) {
            if (next < a.total_tiles) {
                const int64_t seg = next / a.tiles_per_seg;
                const TileCols c = tile_cols(a, next - seg * a.tiles_per_seg, lane);
                stage_inputs<4, PER, NTL>(a, seg, c, lds[buf ^ 1], lane, lw, 0, K, true);
            }
        } else {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            static_for<NWC>([&]<int W>() {
                if (wave == W) compute_special<K, N, OPW, W>(lds[buf], lane, acc);
            });
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            if constexpr (NT) {
                uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
                static_for<OPW>([&]<int O>() {
                    if (O < cnt) {
                        uint32_t w[8];
#pragma unroll
                        for (int p = 0; p < 8; p++) w[p] = acc[O][p];
                        unbitslice8(w);
                        uint8_t *p = out_seg + a.out_off[rbase + O];
                        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                        if (c.vA) __builtin_nontemporal_store((v4){w[0], w[1], w[2], w[3]}, (v4 *)(p + c.outA));
                        if (c.vB) __builtin_nontemporal_store((v4){w[4], w[5], w[6], w[7]}, (v4 *)(p + c.outB));
                    }
                });
            } else {
                store_rows<OPW>(a, seg, c, rbase, cnt, acc);
            }
        }
        if constexpr (RAW) lds_barrier(); else __syncthreads();
        buf ^= 1;
    }
}

__global__ void copy4_kernel(const uint4 *in, uint4 *out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        uint4 a0 = in[i], a1 = in[i + stride], a2 = in[i + 2 * stride], a3 = in[i + 3 * stride];
        out[i] = a0; out[i + stride] = a1; out[i + 2 * stride] = a2; out[i + 3 * stride] = a3;
    }
    for (; i < n; i += stride) out[i] = in[i];
}

__global__ void copy_kernel(const uint4 *in, uint4 *out, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int main(int argc, char **argv) {
    const int k = 29, n = 80, ess = 256, nstripes = 9040, nseg = 8;
    const int64_t spad = (int64_t)nstripes * k * ess, plen = (int64_t)nstripes * ess;
    uint8_t *segs, *pieces;
    CK(hipMalloc(&segs, spad * nseg));
    CK(hipMalloc(&pieces, plen * n * nseg));
    std::vector<uint8_t> h(spad * nseg);
    for (auto &x : h) x = rand();
    CK(hipMemcpy(segs, h.data(), h.size(), hipMemcpyHostToDevice));
    RsArgs a{};
    a.in_base = segs; a.out_base = pieces;
    a.in_stripe_stride = k * ess; a.out_stripe_stride = ess;
    a.in_seg_stride = spad; a.out_seg_stride = plen * n;
    a.nin = k; a.nout = n - k;
    for (int j = 0; j < k; j++) { a.in_off[j] = (int64_t)j * ess; a.copy_off[j] = (int64_t)j * plen; }
    for (int r = 0; r < n - k; r++) a.out_off[r] = (int64_t)(k + r) * plen;
    a.ess = ess; a.cps = ess / 16; a.nstripes = nstripes;
    a.chunks_per_seg = (int64_t)nstripes * (ess / 16);
    a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
    a.total_tiles = a.tiles_per_seg * nseg;
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = (double)spad * nseg * (1.0 + (double)n / k);
    auto timeit = [&](const char *name, auto launch) {
        for (int i = 0; i < 3; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 10;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-34s %9.1f us/8seg  %7.1f us/seg  %6.2f TB/s alg\n", name, us, us / nseg, bytes / us / 1e6);
        fflush(stdout);
    };
    const int grid2 = (int)std::min<int64_t>(a.total_tiles, (int64_t)cus * 2);
    timeit("normal NW4 grid=2x", [&] { hipLaunchKernelGGL((enc_var<29, 80, 4, 0>), dim3(grid2), dim3(256), 0, 0, a); });
    timeit("nocompute NW4 full-grid", [&] { hipLaunchKernelGGL((enc_var<29, 80, 4, 2>), dim3(a.total_tiles), dim3(256), 0, 0, a); });
    {
        const int grid = (int)std::min<int64_t>(a.total_tiles, (int64_t)cus);
        timeit("ws nt-store", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true>), dim3(grid), dim3(512), 0, 0, a); });
        timeit("ws nt-store rawbar", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, false, true>), dim3(grid), dim3(512), 0, 0, a); });
        timeit("ws nt-store nt-load rawbar", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, true, true>), dim3(grid), dim3(512), 0, 0, a); });
        timeit("ws nt-store (data copy nt too) rawbar", [&] { hipLaunchKernelGGL((enc_ws<29, 80, true, true, true>), dim3(grid), dim3(512), 0, 0, a); });
    }
    // plain copy of the same byte count (read spad*(1) write spad*(n/k)) approximated by read+write of equal halves
    const int64_t n16 = (int64_t)(bytes / 2) / 16;
    uint4 *cbuf; CK(hipMalloc(&cbuf, n16 * 16 * 2));
    for (int g : {4, 8, 16})
        for (int u : {1, 4}) {
            char nm[64];
            snprintf(nm, 64, "copy unroll%d grid=%dx (same bytes)", u, g);
            if (u == 1) timeit(nm, [&] { hipLaunchKernelGGL(copy_kernel, dim3(cus * g), dim3(256), 0, 0, cbuf, cbuf + n16, n16); });
            else timeit(nm, [&] { hipLaunchKernelGGL(copy4_kernel, dim3(cus * g), dim3(256), 0, 0, cbuf, cbuf + n16, n16); });
        }
    return 0;
}
