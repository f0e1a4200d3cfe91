// Developer experiment (not product): rebuild body that multiplies by a
// runtime coefficient through a jump table of 256 compile-time leaves
// (tools/gen/gen_jump_table.py), the accumulator row chosen by VGPR index
// mode.  RS(29,80), 8 x 64 MiB segments, share sets {51..79} and a random
// 29-subset.  Build: make -C tools/exp bin/dec_jump
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));


typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

// LDS-DMA prefetch: the raw 16-B chunks of the next chunk of inputs land in
// LDS (no VGPRs held across the compute) while this chunk is multiplied.
template <int NW, int PER>
__device__ __forceinline__ void dma_chunk(const RsArgs &a, int64_t seg, const TileCols &c, uint8_t *raw, int wave,
                                          int lane, int j0, int jn) {
    const uint8_t *in_seg = a.in_base + seg * a.in_seg_stride;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const uint8_t *p = in_seg + a.in_off[j0 + j];
            const uint8_t *pa = p + (c.vA ? c.inA : 0);
            const uint8_t *pb = p + (c.vB ? c.inB : 0);
            __builtin_amdgcn_global_load_lds((gbl_void *)pa, (lds_void *)(raw + j * 2048), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gbl_void *)pb, (lds_void *)(raw + j * 2048 + 1024), 16, 0, 0);
        }
    }
}

template <int NW, int PER>
__device__ __forceinline__ void slice_chunk(const RsArgs &a, int64_t seg, const TileCols &c, const uint8_t *raw,
                                            uint32_t *planes, int wave, int lane, int j0, int jn, bool do_copy) {
    uint8_t *out_seg = a.out_base + seg * a.out_seg_stride;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < jn) {
            const uint4 A = *(const uint4 *)(raw + j * 2048 + lane * 16);
            const uint4 B = *(const uint4 *)(raw + j * 2048 + 1024 + lane * 16);
            const int64_t co = a.copy_off[j0 + j];
            if (do_copy && co >= 0) {
                uint8_t *p = out_seg + co;
                if (c.vA) st16<true>(p + c.outA, A.x, A.y, A.z, A.w);
                if (c.vB) st16<true>(p + c.outB, B.x, B.y, B.z, B.w);
            }
            uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
            bitslice8(w);
            uint32_t *dst = planes + j * 8 * 64 + lane;
#pragma unroll
            for (int p = 0; p < 8; p++) dst[p * 64] = w[p];
        }
    }
}

template <int NW, int PER>
__global__ __launch_bounds__(NW * 64, 4) void dec_dma(const RsArgs a) {
    constexpr int JC = PER * NW, OPW = 8;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *planes = smem;                                   // [JC][8][64] words
    uint8_t *raw = (uint8_t *)(smem + JC * 8 * 64);            // [JC][2][1024] B
    uint16_t *lco = (uint16_t *)(raw + JC * 2048);             // leaf offsets
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int group = (wave + (int)(blockIdx.x % NW)) % NW;
    const int npass = a.nout > 0 ? (a.nout + NW * OPW - 1) / (NW * OPW) : 1;
    const int nch = (a.nin + JC - 1) / JC;
    {
        const int per_pass = a.nin * NW * OPW;
        for (int t = threadIdx.x; t < npass * per_pass; t += NW * 64) {
            const int pass = t / per_pass, r = t - pass * per_pass;
            const int j = r / (NW * OPW), g = (r / OPW) % NW, o = r % OPW;
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rb = p0 + g * prow / NW, cn = p0 + (g + 1) * prow / NW - rb;
            lco[t] = o < cn ? (uint16_t)(a.coef[(int64_t)j * a.coef_ld + rb + o] * RS_JT_SLOT) : (uint16_t)0;
        }
    }
    int64_t tile = blockIdx.x;
    if (tile >= a.total_tiles) return;
    int pass = 0, ch = 0;
    int64_t seg = tile / a.tiles_per_seg;
    TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
    dma_chunk<NW, PER>(a, seg, c, raw, wave, lane, 0, a.nin < JC ? a.nin : JC);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    slice_chunk<NW, PER>(a, seg, c, raw, planes, wave, lane, 0, a.nin < JC ? a.nin : JC, true);
    __syncthreads();
    const uint32_t pl_addr = (uint32_t)(uintptr_t)planes + (uint32_t)lane * 4;
    const uint32_t lco_addr = (uint32_t)(uintptr_t)lco;
    u32x8 acc[OPW];
#pragma unroll
    for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
    for (;;) {
        // next step
        int64_t ntile = tile;
        int npas = pass, nc = ch + 1;
        if (nc == nch) {
            nc = 0;
            if (++npas == npass) {
                npas = 0;
                ntile += gridDim.x;
            }
        }
        const bool has_next = ntile < a.total_tiles;
        int64_t nseg = seg;
        TileCols ncols = c;
        if (has_next) {
            if (ntile != tile) {
                nseg = ntile / a.tiles_per_seg;
                ncols = tile_cols(a, ntile - nseg * a.tiles_per_seg, lane);
            }
            const int nj0 = nc * JC, njn = a.nin - nj0 < JC ? a.nin - nj0 : JC;
            dma_chunk<NW, PER>(a, nseg, ncols, raw, wave, lane, nj0, njn);
        }
        const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
        const int rbase = p0 + group * prow / NW;
        const int cnt = p0 + (group + 1) * prow / NW - rbase;
        const int j0 = ch * JC, jn = a.nin - j0 < JC ? a.nin - j0 : JC;
        if (cnt > 0) {
#pragma nounroll
            for (int jj = 0; jj < jn; jj++)
                jt_input(acc, pl_addr + (uint32_t)(jj * 8 * 64 * 4),
                         lco_addr + (uint32_t)((((pass * a.nin + j0 + jj) * NW + group) * OPW) * 2), 0u);
        }
        if (ch == nch - 1) {
            uint32_t rows[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) rows[o][p] = acc[o][p];
            store_rows<OPW, true>(a, seg, c, rbase, cnt, rows);
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
        }
        if (!has_next) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        {
            const int nj0 = nc * JC, njn = a.nin - nj0 < JC ? a.nin - nj0 : JC;
            slice_chunk<NW, PER>(a, nseg, ncols, raw, planes, wave, lane, nj0, njn, npas == 0);
        }
        __syncthreads();
        tile = ntile;
        pass = npas;
        ch = nc;
        seg = nseg;
        c = ncols;
    }
}

template <int NW, int PER>
size_t dma_lds_bytes(const RsArgs &a) {
    const int npass = a.nout > 0 ? (a.nout + NW * 8 - 1) / (NW * 8) : 1;
    return (size_t)PER * NW * (2048 + 2048) + (size_t)npass * a.nin * NW * 8 * 2;
}

constexpr int kJtRows = 8;  // accumulator rows per wave

template <int NW>
__global__ __launch_bounds__(NW * 64, 4) void rs_matmul_jt(const RsArgs a) {
    constexpr int JC = 2 * NW, OPW = kJtRows, PER = 2;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *lds = smem;                                  // 2 x [JC][8 planes][64 lanes]
    uint16_t *lco = (uint16_t *)(smem + 2 * JC * 8 * 64);  // leaf offsets
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int group = (wave + (int)(blockIdx.x % NW)) % NW;
    const int npass = a.nout > 0 ? (a.nout + NW * OPW - 1) / (NW * OPW) : 1;
    {
        const int per_pass = a.nin * NW * OPW;
        for (int t = threadIdx.x; t < npass * per_pass; t += NW * 64) {
            const int pass = t / per_pass, r = t - pass * per_pass;
            const int j = r / (NW * OPW), g = (r / OPW) % NW, o = r % OPW;
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rb = p0 + g * prow / NW, cn = p0 + (g + 1) * prow / NW - rb;
            const int oo = o - (OPW - cn);  // rows right-aligned: jt_input enters at call site OPW - cnt
            lco[t] = oo >= 0 ? (uint16_t)(a.coef[(int64_t)j * a.coef_ld + rb + oo] * RS_JT_SLOT) : (uint16_t)0;
        }
    }
    __syncthreads();
    const uint32_t lds_addr = (uint32_t)(uintptr_t)lds + (uint32_t)lane * 4;
    const uint32_t lco_addr = (uint32_t)(uintptr_t)lco;
    // Plane chunks alternate between two LDS buffers, so one barrier per chunk
    // suffices: a wave staging chunk c+1 has passed barrier c, which every wave
    // reached only after it finished reading chunk c-1 from that buffer.
    int buf = 0;
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        for (int pass = 0; pass < npass; pass++) {
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rbase = p0 + group * prow / NW;
            const int cnt = p0 + (group + 1) * prow / NW - rbase;
            u32x8 acc[OPW];
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
            for (int j0 = 0; j0 < a.nin; j0 += JC) {
                const int jn = a.nin - j0 < JC ? a.nin - j0 : JC;
                stage_inputs<NW, PER, true>(a, seg, c, lds + buf * (JC * 8 * 64), lane, wave, j0, jn, pass == 0);
                lds_barrier();
                if (cnt > 0) {
#pragma nounroll
                    for (int jj = 0; jj < jn; jj++)
                        jt_input(acc, lds_addr + (uint32_t)((buf * JC + jj) * 8 * 64 * 4),
                                 lco_addr + (uint32_t)((((pass * a.nin + j0 + jj) * NW + group) * OPW) * 2),
                                 (uint32_t)(OPW - cnt));
                }
                buf ^= 1;
            }
            uint32_t rows[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) rows[o][p] = acc[o][p];
            store_rows<OPW, true>(a, seg, c, rbase, cnt, rows);
        }
    }
}

template <int NW>
size_t jt_lds_bytes(const RsArgs &a) {
    const int npass = a.nout > 0 ? (a.nout + NW * kJtRows - 1) / (NW * kJtRows) : 1;
    return (size_t)2 * 2 * NW * 8 * 64 * 4 + (size_t)npass * a.nin * NW * kJtRows * 2;
}


int main(int argc, char **argv) {
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    int vidx = 0;
    const int k = 29, n = 80, ess = 256, nstripes = 9040, nseg = 8;
    const int64_t spad = (int64_t)nstripes * k * ess, plen = (int64_t)nstripes * ess;
    uint8_t *pieces, *out;
    CK(hipMalloc(&pieces, plen * n * nseg));
    CK(hipMalloc(&out, spad * nseg));
    std::vector<uint8_t> h(plen * n * nseg);
    std::mt19937 hr(7);
    for (auto &x : h) x = (uint8_t)hr();
    CK(hipMemcpy(pieces, h.data(), h.size(), hipMemcpyHostToDevice));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<int>> sets;
    for (int m : {29, 22, 20, 18, 16}) {
        std::vector<int> st;
        for (int i = 0; i < k - m; i++) st.push_back(i);
        for (int i = 0; i < m; i++) st.push_back(51 + i);
        sets.push_back(st);
    }
    int set_idx = -1;
    for (auto &ids : sets) {
        vidx = 0;
        set_idx++;
        if (getenv("SET") && atoi(getenv("SET")) != set_idx) continue;
        std::vector<uint8_t> m((size_t)k * k, 0);
        for (int i = 0; i < k; i++)
            for (int j = 0; j < k; j++) m[i * k + j] = gen_entry(k, ids[i], j);
        gf_invert(m.data(), k);
        std::vector<int> missing;
        std::vector<bool> present(k, false);
        for (int i : ids)
            if (i < k) present[i] = true;
        for (int i = 0; i < k; i++)
            if (!present[i]) missing.push_back(i);
        const int R = (int)missing.size();
        const int ld = 32;
        std::vector<uint8_t> coef((size_t)k * ld, 0);
        for (int r = 0; r < R; r++)
            for (int c = 0; c < k; c++) coef[c * ld + r] = m[missing[r] * k + c];
        coef.resize(coef.size() + 64, 0);
        uint8_t *dcoef;
        CK(hipMalloc(&dcoef, coef.size()));
        CK(hipMemcpy(dcoef, coef.data(), coef.size(), hipMemcpyHostToDevice));
        RsArgs a{};
        a.in_base = pieces;
        a.out_base = out;
        a.coef = dcoef;
        a.coef_ld = ld;
        a.in_stripe_stride = ess;
        a.out_stripe_stride = (int64_t)k * ess;
        a.in_seg_stride = plen * n;
        a.out_seg_stride = spad;
        a.nin = k;
        a.nout = R;
        for (int c = 0; c < k; c++) {
            a.in_off[c] = (int64_t)ids[c] * plen;
            a.copy_off[c] = ids[c] < k ? (int64_t)ids[c] * ess : -1;
        }
        for (int r = 0; r < R; r++) a.out_off[r] = (int64_t)missing[r] * ess;
        a.ess = ess;
        a.cps = ess / 16;
        a.nstripes = nstripes;
        a.chunks_per_seg = (int64_t)nstripes * (ess / 16);
        a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
        a.total_tiles = a.tiles_per_seg * nseg;
        const double bytes = 2.0 * spad * nseg;
        // host reference: segment 0, stripes 0..1 and the last stripe of the last segment
        auto refstripe = [&](int sg, int s, std::vector<uint8_t> &ref) {
            ref.assign((size_t)k * ess, 0);
            for (int i = 0; i < k; i++)
                for (int t = 0; t < ess; t++) {
                    uint8_t acc = 0;
                    for (int c = 0; c < k; c++)
                        acc ^= gf_mul(m[i * k + c], h[(size_t)sg * plen * n + (size_t)ids[c] * plen + (size_t)s * ess + t]);
                    ref[i * ess + t] = acc;
                }
        };
        std::vector<std::pair<int, int>> checks = {{0, 0}, {0, 1}, {0, 4517}, {nseg - 1, nstripes - 1}};
        std::vector<std::vector<uint8_t>> refs(checks.size());
        for (size_t q = 0; q < checks.size(); q++) refstripe(checks[q].first, checks[q].second, refs[q]);
        auto timeit = [&](const char *name, size_t shmem, auto launch) {
            if (only >= 0 && vidx++ != only) return;
            CK(hipMemset(out, 0, spad * nseg));
            launch(shmem);
            CK(hipDeviceSynchronize());
            bool ok = true;
            for (size_t q = 0; q < checks.size(); q++) {
                std::vector<uint8_t> got((size_t)k * ess);
                CK(hipMemcpy(got.data(), out + checks[q].first * spad + (int64_t)checks[q].second * k * ess, got.size(),
                             hipMemcpyDeviceToHost));
                ok = ok && got == refs[q];
            }
            for (int i = 0; i < 2; i++) launch(shmem);
            CK(hipDeviceSynchronize());
            const int it = 10;
            CK(hipEventRecord(e0));
            for (int i = 0; i < it; i++) launch(shmem);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / it;
            printf("m=%2d %-34s %8.1f us/8seg %7.1f us/seg %6.2f TB/s %s\n", R, name, us, us / nseg, bytes / us / 1e6,
                   ok ? "ok" : "WRONG");
            fflush(stdout);
        };
        for (int rep = 0; rep < 2; rep++) {
            timeit("jt NW2 grid8x", jt_lds_bytes<2>(a), [&](size_t sh) { hipLaunchKernelGGL((rs_matmul_jt<2>), dim3(cus * 8), dim3(128), sh, 0, a); });
            timeit("jt NW3 grid5x", jt_lds_bytes<3>(a), [&](size_t sh) { hipLaunchKernelGGL((rs_matmul_jt<3>), dim3(cus * 5), dim3(192), sh, 0, a); });
            timeit("jt NW4 grid4x", jt_lds_bytes<4>(a), [&](size_t sh) { hipLaunchKernelGGL((rs_matmul_jt<4>), dim3(cus * 4), dim3(256), sh, 0, a); });
        }
    }
    return 0;
}
