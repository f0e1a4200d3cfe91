// Developer experiment (not product): issue rate of the rebuild body's
// instruction mix on one CU-full of waves.  Each wave runs ITER iterations of
// 64 v_bitop3 (8 planes x 8 rows), optionally with 4 SALU per 8 VALU (the
// call-site bookkeeping) and/or VGPR index mode on around them.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "rowtabs_probe.inc"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

#define B8(a0, l0, h0)                                        \
    "v_bitop3_b32 v" #a0 ", v" #a0 ", v" #l0 ", v" #h0 " bitop3:0x96\n"
#define ROW(A)                                                                                         \
    "v_bitop3_b32 v" #A "0, v" #A "0, v97, v114 bitop3:0x96\n"                                         \
    "v_bitop3_b32 v" #A "1, v" #A "1, v98, v115 bitop3:0x96\n"                                         \
    "v_bitop3_b32 v" #A "2, v" #A "2, v99, v116 bitop3:0x96\n"                                         \
    "v_bitop3_b32 v" #A "3, v" #A "3, v100, v117 bitop3:0x96\n"                                        \
    "v_bitop3_b32 v" #A "4, v" #A "4, v101, v118 bitop3:0x96\n"                                        \
    "v_bitop3_b32 v" #A "5, v" #A "5, v102, v119 bitop3:0x96\n"                                        \
    "v_bitop3_b32 v" #A "6, v" #A "6, v103, v120 bitop3:0x96\n"                                        \
    "v_bitop3_b32 v" #A "7, v" #A "7, v104, v121 bitop3:0x96\n"
#define SAL "s_and_b32 s50, s44, 0xffff\n s_add_u32 s42, s40, s50\n s_addc_u32 s43, s41, 0\n s_add_u32 m0, m0, 8\n"

template <int MODE>
__global__ __launch_bounds__(256) void probe(int iters, uint32_t *out, const uint32_t *offs = nullptr) {
    uint32_t r = threadIdx.x;
    for (int i = 0; i < iters; i++) {
        if constexpr (MODE == 0) {
            asm volatile(ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10)
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121");
        } else if constexpr (MODE == 1) {
            asm volatile(SAL ROW(3) SAL ROW(4) SAL ROW(5) SAL ROW(6) SAL ROW(7) SAL ROW(8) SAL ROW(9) SAL ROW(10)
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121", "s40", "s41", "s42", "s43", "s44", "s50", "m0", "scc");
        } else if constexpr (MODE == 2) {
            asm volatile("s_mov_b32 s51, m0\n"
                         "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
                         ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10)
                         "s_set_gpr_idx_off\n s_mov_b32 m0, s51\n"
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121", "s51", "m0");
        } else if constexpr (MODE == 4) {
            asm volatile("s_mov_b32 s51, m0\n"
                         "s_set_gpr_idx_on 0, gpr_idx(DST)\n"
                         ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10)
                         "s_set_gpr_idx_off\n s_mov_b32 m0, s51\n"
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121", "s51", "m0");
        } else if constexpr (MODE == 5) {
            asm volatile("s_mov_b32 s51, m0\n"
                         "s_set_gpr_idx_on 0, gpr_idx(SRC0)\n"
                         ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10)
                         "s_set_gpr_idx_off\n s_mov_b32 m0, s51\n"
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121", "s51", "m0");
        } else if constexpr (MODE == 6) {
            asm volatile("s_mov_b32 s51, m0\n"
                         "s_set_gpr_idx_on 0, gpr_idx(SRC1)\n"
                         ROW(3) ROW(4) ROW(5) ROW(6) ROW(7) ROW(8) ROW(9) ROW(10)
                         "s_set_gpr_idx_off\n s_mov_b32 m0, s51\n"
                         ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "v120", "v121", "s51", "m0");
        } else if constexpr (MODE == 7) {
            // per-row leaf tables (no index mode): 8 calls with per-wave coefficient pattern [wave][29][8]
            const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const uint32_t *o = offs + (w * 29 + (i % 29)) * 8;
            asm volatile("s_load_dwordx8 s[52:59], %[o], 0\n s_waitcnt lgkmcnt(0)\n" JT_ROWCALLS
                         :: [o] "s"(o)
                         : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                         "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55",
                         "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68",
                         "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81",
                         "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94",
                         "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106",
                         "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",
                         "v119", "s40", "s41", "s42", "s43", "s48", "s49", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "scc");
        } else {
            // call/return: 8 calls of an 8-bitop3 leaf per iteration
            asm volatile(
                "s_getpc_b64 s[40:41]\n.Lp%=:\n s_add_u32 s40, s40, .Lleaf%=-.Lp%=\n s_addc_u32 s41, s41, 0\n"
                "s_swappc_b64 s[48:49], s[40:41]\n s_swappc_b64 s[48:49], s[40:41]\n"
                "s_swappc_b64 s[48:49], s[40:41]\n s_swappc_b64 s[48:49], s[40:41]\n"
                "s_swappc_b64 s[48:49], s[40:41]\n s_swappc_b64 s[48:49], s[40:41]\n"
                "s_swappc_b64 s[48:49], s[40:41]\n s_swappc_b64 s[48:49], s[40:41]\n"
                "s_branch .Le%=\n.Lleaf%=:\n" ROW(3) "s_setpc_b64 s[48:49]\n.Le%=:\n"
                ::: "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v97", "v98", "v99", "v100",
                "v101", "v102", "v103", "v104", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121",
                "s40", "s41", "s48", "s49", "scc");
        }
    }
    if (r == 0xFFFFFFFFu) out[0] = r;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 20000;
    std::vector<uint32_t> hoffs(4 * 29 * 8);
    std::mt19937 rng(1);
    for (auto &x : hoffs) x = (rng() % 255 + 1) * 72;
    uint32_t *doffs;
    CK(hipMalloc(&doffs, hoffs.size() * 4));
    CK(hipMemcpy(doffs, hoffs.data(), hoffs.size() * 4, hipMemcpyHostToDevice));
    auto run = [&](const char *name, int mode, int wpc) {
        // wpc waves per CU: blocks of 256 threads (4 waves, one per SIMD)
        dim3 grid(cus * (wpc / 4));
        auto L = [&] {
            if (mode == 0) hipLaunchKernelGGL(probe<0>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 1) hipLaunchKernelGGL(probe<1>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 2) hipLaunchKernelGGL(probe<2>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 3) hipLaunchKernelGGL(probe<3>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 4) hipLaunchKernelGGL(probe<4>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 5) hipLaunchKernelGGL(probe<5>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 6) hipLaunchKernelGGL(probe<6>, grid, dim3(256), 0, 0, iters, out);
            if (mode == 7) hipLaunchKernelGGL(probe<7>, grid, dim3(256), 0, 0, iters, out, doffs);
        };
        L();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        L();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double valu = (double)iters * 64 * (wpc / 4);  // per SIMD
        const double cyc = ms * 1e-3 * 2.1e9;
        printf("%-28s waves/SIMD=%d  %8.3f ms  %.2f cycles/VALU per SIMD (at 2.1 GHz)\n", name, wpc / 4, ms,
               cyc / valu);
        fflush(stdout);
    };
    for (int w : {8, 16}) {
        run("pure bitop3", 0, w);
        run("bitop3 + 4 SALU / 8", 1, w);
        run("bitop3 idx SRC0,DST", 2, w);

        run("per-row tables, 928 hot leaves", 7, w);
        run("8 x call(8 bitop3 leaf)", 3, w);
    }
    return 0;
}
