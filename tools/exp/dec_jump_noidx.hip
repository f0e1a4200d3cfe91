#define JT_NOJUMP 1
#define JT_NJ_LEAF "v_bitop3_b32 v32, v32, v97, v114 bitop3:0x96\n" "v_bitop3_b32 v33, v33, v98, v115 bitop3:0x96\n" "v_bitop3_b32 v34, v34, v99, v116 bitop3:0x96\n" "v_bitop3_b32 v35, v35, v100, v117 bitop3:0x96\n" "v_bitop3_b32 v36, v36, v101, v118 bitop3:0x96\n" "v_bitop3_b32 v37, v37, v102, v119 bitop3:0x96\n" "v_bitop3_b32 v38, v38, v103, v120 bitop3:0x96\n" "v_bitop3_b32 v39, v39, v104, v121 bitop3:0x96\n"
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
#include "../../uplink_amd/csrc/rs_jump_table.inc"

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

#if defined(JT_NOJUMP)
#define JT_LEAF_P(P) "v_bitop3_b32 v" #P ", v" #P ", v" #P ", v" #P " bitop3:0x96\n"
#define JT_CALL(IDX, EXTRACT)                 \
    "s_nop 0\n" EXTRACT    \
    "s_add_u32 s42, s40, s50\n"               \
    "s_addc_u32 s43, s41, 0\n"                \
    JT_NJ_LEAF
#elif defined(JT_FIXEDTGT)
#define JT_CALL(IDX, EXTRACT)                 \
    "s_nop 0\n"            \
    "s_swappc_b64 s[48:49], s[42:43]\n"
#else
#define JT_CALL(IDX, EXTRACT)                 \
    "s_nop 0\n" EXTRACT    \
    "s_add_u32 s42, s40, s50\n"               \
    "s_addc_u32 s43, s41, 0\n"                \
    "s_swappc_b64 s[48:49], s[42:43]\n"
#endif

// acc rows 0..7 (+= D[row][j] * x_j) for one input whose 8 planes are at LDS
// byte address xa (+256 per plane); ca = LDS address of the 8 16-bit leaf
// offsets (coefficient * RS_JT_SLOT) of this wave's rows.
__device__ __forceinline__ void jt_input_x(u32x8 (&acc)[8], uint32_t xa, uint32_t ca) {
    asm volatile(
        "s_mov_b32 s51, m0\n"
        "ds_read_b32 v96, %[xa]\n"
        "ds_read_b32 v97, %[xa] offset:256\n"
        "ds_read_b32 v99, %[xa] offset:512\n"
        "ds_read_b32 v103, %[xa] offset:768\n"
        "ds_read_b32 v111, %[xa] offset:1024\n"
        "ds_read_b32 v112, %[xa] offset:1280\n"
        "ds_read_b32 v114, %[xa] offset:1536\n"
        "ds_read_b32 v118, %[xa] offset:1792\n"
        "ds_read_b128 v[104:107], %[ca]\n"
        "s_waitcnt lgkmcnt(0)\n"
        "v_readfirstlane_b32 s44, v104\n"
        "v_readfirstlane_b32 s45, v105\n"
        "v_readfirstlane_b32 s46, v106\n"
        "v_readfirstlane_b32 s47, v107\n"
        "v_xor_b32 v98, v96, v97\n"
        "v_xor_b32 v100, v96, v99\n"
        "v_xor_b32 v101, v97, v99\n"
        "v_xor_b32 v102, v98, v99\n"
        "v_xor_b32 v104, v96, v103\n"
        "v_xor_b32 v105, v97, v103\n"
        "v_xor_b32 v106, v98, v103\n"
        "v_xor_b32 v107, v99, v103\n"
        "v_xor_b32 v108, v100, v103\n"
        "v_xor_b32 v109, v101, v103\n"
        "v_xor_b32 v110, v102, v103\n"
        "v_xor_b32 v113, v111, v112\n"
        "v_xor_b32 v115, v111, v114\n"
        "v_xor_b32 v116, v112, v114\n"
        "v_xor_b32 v117, v113, v114\n"
        "v_xor_b32 v119, v111, v118\n"
        "v_xor_b32 v120, v112, v118\n"
        "v_xor_b32 v121, v113, v118\n"
        "v_xor_b32 v122, v114, v118\n"
        "v_xor_b32 v123, v115, v118\n"
        "v_xor_b32 v124, v116, v118\n"
        "v_xor_b32 v125, v117, v118\n"
        "s_getpc_b64 s[40:41]\n"
        ".Lgp%=:\n"
        "s_add_u32 s40, s40, .Ltab%=-.Lgp%=\n"
        "s_addc_u32 s41, s41, 0\n"
#ifdef JT_FIXEDTGT
        "s_and_b32 s50, s44, 0xffff\n"
        "s_add_u32 s42, s40, s50\n"
        "s_addc_u32 s43, s41, 0\n"
#endif
        "s_nop 0\n"
        JT_CALL(0, "s_and_b32 s50, s44, 0xffff\n")
        JT_CALL(8, "s_lshr_b32 s50, s44, 16\n")
        JT_CALL(16, "s_and_b32 s50, s45, 0xffff\n")
        JT_CALL(24, "s_lshr_b32 s50, s45, 16\n")
        JT_CALL(32, "s_and_b32 s50, s46, 0xffff\n")
        JT_CALL(40, "s_lshr_b32 s50, s46, 16\n")
        JT_CALL(48, "s_and_b32 s50, s47, 0xffff\n")
        JT_CALL(56, "s_lshr_b32 s50, s47, 16\n")
        "s_nop 0\n"
        "s_mov_b32 m0, s51\n"
        "s_branch .Lend%=\n"
        ".Ltab%=:\n"
        RS_JUMP_TABLE_ASM
        ".Lend%=:\n"
        : "+{v[32:39]}"(acc[0]), "+{v[40:47]}"(acc[1]), "+{v[48:55]}"(acc[2]), "+{v[56:63]}"(acc[3]),
          "+{v[64:71]}"(acc[4]), "+{v[72:79]}"(acc[5]), "+{v[80:87]}"(acc[6]), "+{v[88:95]}"(acc[7])
        : [xa] "v"(xa), [ca] "v"(ca)
        : "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108",
          "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
          "v122", "v123", "v124", "v125", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49",
          "s50", "s51", "scc", "memory");
}

constexpr int JC = 8;

// MODE 0 normal; 1 no compute (memory only); 2 no global loads/stores (compute + LDS only)
template <int NW, int MINW, int MODE = 0>
__global__ __launch_bounds__(NW * 64, MINW) void dec_jt(const RsArgs a) {
    constexpr int OPW = 8;
    constexpr int PER = (JC + NW - 1) / NW;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *lds = smem;                                      // JC * 8 * 64 words
    uint16_t *lco = (uint16_t *)(smem + JC * 8 * 64);          // [pass][j][group][8]
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
            lco[t] = o < cn ? (uint16_t)(a.coef[(int64_t)j * a.coef_ld + rb + o] * RS_JT_SLOT) : 0;
        }
    }
    __syncthreads();
    const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
    const uint32_t lco_base = (uint32_t)(uintptr_t)lco;
    for (int64_t tile = blockIdx.x; tile < a.total_tiles; tile += gridDim.x) {
        const int64_t seg = tile / a.tiles_per_seg;
        const TileCols c = tile_cols(a, tile - seg * a.tiles_per_seg, lane);
        for (int pass = 0; pass < npass; pass++) {
            const int p0 = pass * a.nout / npass, prow = (pass + 1) * a.nout / npass - p0;
            const int rbase = p0 + group * prow / NW;
            const int cnt = p0 + (group + 1) * prow / NW - rbase;
            u32x8 acc[8];
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
            for (int j0 = 0; j0 < a.nin; j0 += JC) {
                const int jn = a.nin - j0 < JC ? a.nin - j0 : JC;
                if (MODE != 2) stage_inputs<NW, PER, true>(a, seg, c, lds, lane, wave, j0, jn, pass == 0);
                else for (int q = threadIdx.x; q < jn * 8 * 64; q += NW * 64) lds[q] = q * 0x9E3779B9u + (uint32_t)tile;
                __syncthreads();
                if (MODE != 1 && cnt > 0) {
#pragma nounroll
                    for (int jj = 0; jj < jn; jj++) {
                        const uint32_t xa = lds_base + (uint32_t)((jj * 8 * 64 + lane) * 4);
                        const uint32_t ca = lco_base + (uint32_t)((((pass * a.nin + j0 + jj) * NW + group) * OPW) * 2);
                        jt_input_x(acc, xa, ca);
                    }
                }
                __syncthreads();
            }
            uint32_t accs[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) accs[o][p] = acc[o][p];
            if (MODE != 2) store_rows<OPW, true>(a, seg, c, rbase, cnt, accs);
            else if (accs[0][0] == 0x12345u && accs[cnt & 7][3] == 0x777u) a.out_base[lane] = 1;
        }
    }
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
    {
        std::vector<int> s;
        for (int i = 51; i < 80; i++) s.push_back(i);
        sets.push_back(s);
    }
    {
        std::mt19937 rng(29);
        std::vector<int> all(n);
        for (int i = 0; i < n; i++) all[i] = i;
        std::shuffle(all.begin(), all.end(), rng);
        std::vector<int> s(all.begin(), all.begin() + k);
        std::sort(s.begin(), s.end());
        sets.push_back(s);
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
        const size_t sh4 = JC * 8 * 64 * 4 + (size_t)k * 4 * 8 * 2 + 64;
        const size_t sh8 = JC * 8 * 64 * 4 + (size_t)k * 8 * 8 * 2 + 64;
        for (int rep = 0; rep < 1; rep++) {
            timeit("PROBE memory only grid8x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2, 1>), dim3(cus * 8), dim3(256), sh, 0, a); });
            timeit("PROBE compute only grid8x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2, 2>), dim3(cus * 8), dim3(256), sh, 0, a); });
            timeit("PROBE compute only grid4x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2, 2>), dim3(cus * 4), dim3(256), sh, 0, a); });
            timeit("jt NW4 grid4x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2>), dim3(cus * 4), dim3(256), sh, 0, a); });
            timeit("jt NW4 grid3x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2>), dim3(cus * 3), dim3(256), sh, 0, a); });
            timeit("jt NW4 grid8x", sh4, [&](size_t sh) { hipLaunchKernelGGL((dec_jt<4, 2>), dim3(cus * 8), dim3(256), sh, 0, a); });
        }
    }
    return 0;
}
