// Developer experiment (not product): the warp-specialised RS(29,80) encoder
// with a variable number of compute waves (NC) and loader waves (NL).  With
// NC = 4 each compute wave is alone on its SIMD and issues VALU at the
// single-wave rate; NC = 8 puts two compute waves on every SIMD.
// Build: make -C tools/exp bin/enc2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../uplink_amd/csrc/rs_device.hpp"

using namespace uplink_ec;
using namespace uplink_ec::dev;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                   \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// MODE 0 normal, 1 memory only (no XOR), 2 compute only (no global traffic)
template <int K, int N, int NC, int NL, int MODE = 0>
__global__ __launch_bounds__((NC + NL) * 64, 1) void enc_ws(const RsArgs a) {
    constexpr int R = N - K;
    constexpr int OPW = (R + NC - 1) / NC;
    constexpr int PER = (K + NL - 1) / NL;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NC;
    const int lw = wave - NC;
    int64_t tile = blockIdx.x;
    if (loader && tile < a.total_tiles && MODE != 2) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        stage_inputs<NL, PER, true>(a, seg, c, lds[0], lane, lw, 0, K, true);
    }
    lds_barrier();
    int buf = 0;
    for (; tile < a.total_tiles; tile += gridDim.x) {
        if (loader) {
            const int64_t next = tile + gridDim.x;
            if (next < a.total_tiles && MODE != 2) {
                const int64_t seg = next / a.tiles_per_seg;
                const TileCols c = tile_cols(a, next - seg * a.tiles_per_seg, lane);
                stage_inputs<NL, PER, true>(a, seg, c, lds[buf ^ 1], lane, lw, 0, K, true);
            }
        } else {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = MODE == 1 ? lds[buf][(o * 8 + p) * 64 + lane] : 0;
            if constexpr (MODE != 1) {
                static_for<NC>([&]<int W>() {
                    if (wave == W) compute_special<K, N, OPW, W>(lds[buf], lane, acc);
                });
            }
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            if constexpr (MODE != 2) {
                store_rows<OPW, true>(a, seg, c, rbase, cnt, acc);
            } else {
#pragma unroll
                for (int o = 0; o < OPW; o++)
#pragma unroll
                    for (int p = 0; p < 8; p++) asm volatile("" ::"v"(acc[o][p]));
            }
        }
        lds_barrier();
        buf ^= 1;
    }
}

// All 8 waves compute parity rows (2 per SIMD: twice the lone-wave VALU
// rate); waves 4..7 also load the next tile: they issue its loads first,
// compute their rows of the current tile while the loads are in flight,
// then write the copies, bit-slice and fill the other LDS slot.
template <int K, int N>
__global__ __launch_bounds__(512, 1) void enc_mix(const RsArgs a) {
    constexpr int NWV = 8, NLD = 4;
    constexpr int R = N - K;
    constexpr int OPW = (R + NWV - 1) / NWV;
    constexpr int PER = (K + NLD - 1) / NLD;
    __shared__ uint32_t lds[2][K * 8 * 64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool loader = wave >= NWV - NLD;
    const int lw = wave - (NWV - NLD);
    int64_t tile = blockIdx.x;
    if (loader && tile < a.total_tiles) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        stage_inputs<NLD, PER, true>(a, seg, c, lds[0], lane, lw, 0, K, true);
    }
    lds_barrier();
    int buf = 0;
    for (; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t next = tile + gridDim.x;
        const bool has_next = loader && next < a.total_tiles;
        uint4 bufA[PER], bufB[PER];
        TileCols cn;
        int64_t segn = 0;
        if (has_next) {  // issue the next tile's loads (consumed after the XOR work)
            segn = next / a.tiles_per_seg;
            cn = tile_cols(a, next - segn * a.tiles_per_seg, lane);
            const uint8_t *in_seg = a.in_base + segn * a.in_seg_stride;
            const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = lw + NLD * i;
                if (j < K) {
                    const uint8_t *p = in_seg + a.in_off[j];
                    bufA[i] = cn.vA ? ld16<true>(p + cn.inA) : z;
                    bufB[i] = cn.vB ? ld16<true>(p + cn.inB) : z;
                }
            }
        }
        {
            const int64_t seg = tile / a.tiles_per_seg;
            const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
            uint32_t acc[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) acc[o][p] = 0;
            static_for<NWV>([&]<int W>() {
                if (wave == W) compute_special<K, N, OPW, W>(lds[buf], lane, acc);
            });
            const int rbase = wave * OPW;
            const int cnt = R - rbase < OPW ? R - rbase : OPW;
            store_rows<OPW, true>(a, seg, c, rbase, cnt, acc);
        }
        if (has_next) {
            uint8_t *out_seg = a.out_base + segn * a.out_seg_stride;
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = lw + NLD * i;
                if (j < K) {
                    uint8_t *p = out_seg + a.copy_off[j];
                    if (cn.vA) st16<true>(p + cn.outA, bufA[i].x, bufA[i].y, bufA[i].z, bufA[i].w);
                    if (cn.vB) st16<true>(p + cn.outB, bufB[i].x, bufB[i].y, bufB[i].z, bufB[i].w);
                    uint32_t w[8] = {bufA[i].x, bufA[i].y, bufA[i].z, bufA[i].w,
                                     bufB[i].x, bufB[i].y, bufB[i].z, bufB[i].w};
                    bitslice8(w);
                    uint32_t *dst = lds[buf ^ 1] + j * 8 * 64 + lane;
#pragma unroll
                    for (int p = 0; p < 8; p++) dst[p * 64] = w[p];
                }
            }
        }
        lds_barrier();
        buf ^= 1;
    }
}

// idles the GPU's memory system for ~`cycles` shader clocks (lets the memory-side
// cache drain the previous kernel's dirty lines, as the rebuild kernel does in bench.py)
__global__ void spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) __builtin_amdgcn_s_sleep(10);
}

int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0;
    constexpr int k = 29, n = 80, ess = 256, nstripes = 9040, nseg = 8;
    const int64_t spad = (int64_t)nstripes * k * ess, plen = (int64_t)nstripes * ess;
    uint8_t *segs, *pieces;
    CK(hipMalloc(&segs, spad * nseg));
    CK(hipMalloc(&pieces, plen * n * nseg));
    std::vector<uint8_t> h(spad * nseg);
    std::mt19937 rng(5);
    for (auto &x : h) x = (uint8_t)rng();
    CK(hipMemcpy(segs, h.data(), h.size(), hipMemcpyHostToDevice));
    RsArgs a{};
    a.in_base = segs;
    a.out_base = pieces;
    a.in_stripe_stride = k * ess;
    a.out_stripe_stride = ess;
    a.in_seg_stride = spad;
    a.out_seg_stride = plen * n;
    a.nin = k;
    a.nout = n - k;
    for (int j = 0; j < k; j++) {
        a.in_off[j] = (int64_t)j * ess;
        a.copy_off[j] = (int64_t)j * plen;
    }
    for (int r = 0; r < n - k; r++) a.out_off[r] = (int64_t)(k + r) * plen;
    a.ess = ess;
    a.cps = ess / 16;
    a.nstripes = nstripes;
    a.chunks_per_seg = (int64_t)nstripes * (ess / 16);
    a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
    a.total_tiles = a.tiles_per_seg * nseg;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)spad * nseg * (1.0 + (double)n / k);
    // reference parity for stripes {0, last} of segment 0 and last
    auto check = [&]() {
        bool ok = true;
        for (int sg : {0, nseg - 1})
            for (int s : {0, 4711, nstripes - 1})
                for (int r = 0; r < n; r++) {
                    std::vector<uint8_t> got(ess);
                    CK(hipMemcpy(got.data(), pieces + sg * plen * n + r * plen + (int64_t)s * ess, ess,
                                 hipMemcpyDeviceToHost));
                    for (int t = 0; t < ess; t++) {
                        uint8_t e = 0;
                        for (int j = 0; j < k; j++)
                            e ^= gf_mul(gen_entry(k, r, j), h[(size_t)sg * spad + (size_t)s * k * ess + j * ess + t]);
                        if (got[t] != e) ok = false;
                    }
                }
        return ok;
    };
    auto timeit = [&](const char *name, auto launch) {
        if (only >= 0 && vidx++ != only) return;
        CK(hipMemset(pieces, 0, plen * n * nseg));
        launch();
        CK(hipDeviceSynchronize());
        const bool ok = check();
        for (int i = 0; i < 150; i++) launch();  // > 50 ms: past the clock ramp under sustained load
        CK(hipDeviceSynchronize());
        const int it = 40;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-34s %6.1f us/seg %6.3f TB/s %s\n", name, us / nseg, bytes / us / 1e6, ok ? "ok" : "WRONG");
        fflush(stdout);
    };
    const int grid = (int)std::min<int64_t>(a.total_tiles, cus);
#define V(NC, NL, M)                                                                               \
    timeit("NC=" #NC " NL=" #NL " mode=" #M,                                                       \
           [&] { hipLaunchKernelGGL((enc_ws<29, 80, NC, NL, M>), dim3(grid), dim3((NC + NL) * 64), 0, 0, a); });
    V(4, 4, 0)
    timeit("mix: 8 computing, 4 of them loading", [&] { hipLaunchKernelGGL((enc_mix<29, 80>), dim3(grid), dim3(512), 0, 0, a); });
    V(4, 4, 1)
    return 0;
}
