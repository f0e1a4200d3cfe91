// Experiment: VALU issue cost per SIMD of single integer ops on gfx950,
// 8 waves per SIMD, 8 independent destinations per block (so no dependent
// stalls).  Feeds the BLAKE3 G-function design.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

#define X8(OP)                                                                                                     \
    OP(40) OP(41) OP(42) OP(43) OP(44) OP(45) OP(46) OP(47)
#define XOR(d) "v_xor_b32 v" #d ", v" #d ", v60\n"
#define XOR3(d) "v_xor3_b32 v" #d ", v" #d ", v60, v61\n"
#define BOP3(d) "v_bitop3_b32 v" #d ", v" #d ", v60, v61 bitop3:0x96\n"
#define ADD(d) "v_add_u32 v" #d ", v" #d ", v60\n"
#define ADD3(d) "v_add3_u32 v" #d ", v" #d ", v60, v61\n"
#define ALIGN(d) "v_alignbit_b32 v" #d ", v" #d ", v" #d ", 12\n"
#define PERM(d) "v_perm_b32 v" #d ", v" #d ", v" #d ", v62\n"
#define LSHL(d) "v_lshlrev_b32 v" #d ", 7, v" #d "\n"
#define PKADD(d) "v_pk_add_u16 v" #d ", v" #d ", v60\n"
#define XAD(d) "v_xad_u32 v" #d ", v" #d ", v60, v61\n"
#define MOV(d) "v_mov_b32 v" #d ", v60\n"
#define SDWA(d) "v_xor_b32_sdwa v" #d ", v" #d ", v60 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n"
#define ABYTE(d) "v_alignbyte_b32 v" #d ", v" #d ", v" #d ", 1\n"
#define LSHR(d) "v_lshrrev_b32 v" #d ", 7, v" #d "\n"
#define OR3(d) "v_or3_b32 v" #d ", v" #d ", v60, v61\n"
#define LSHLOR(d) "v_lshl_or_b32 v" #d ", v" #d ", 7, v60\n"
#define CLOB                                                                                                          \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v60", "v61", "v62"

#define KERNEL(NAME, OP)                                                                            \
    __global__ __launch_bounds__(256) void NAME(int iters) {                                      \
        asm volatile("v_mov_b32 v60, 3\n v_mov_b32 v61, 5\n v_mov_b32 v62, 0x03020100\n" ::: CLOB); \
        for (int i = 0; i < iters; i++)                                                            \
            asm volatile(X8(OP) X8(OP) X8(OP) X8(OP) X8(OP) X8(OP) X8(OP) X8(OP) ::: CLOB);        \
    }

KERNEL(k_xor, XOR)
KERNEL(k_bop3, BOP3)
KERNEL(k_add, ADD)
KERNEL(k_add3, ADD3)
KERNEL(k_align, ALIGN)
KERNEL(k_perm, PERM)
KERNEL(k_lshl, LSHL)
KERNEL(k_pkadd, PKADD)
KERNEL(k_xad, XAD)
KERNEL(k_mov, MOV)
KERNEL(k_sdwa, SDWA)
KERNEL(k_abyte, ABYTE)
KERNEL(k_lshr, LSHR)
KERNEL(k_or3, OR3)
KERNEL(k_lshlor, LSHLOR)

int main() {
    int dev;
    CK(hipGetDevice(&dev));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, dev));
    const int cus = p.multiProcessorCount;
    const int iters = 4000;
    const dim3 grid(cus * 8);  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
    struct K {
        const char *n;
        void (*f)(int);
    } ks[] = {{"v_xor_b32", k_xor},   {"v_bitop3_b32", k_bop3}, {"v_add_u32", k_add},
              {"v_add3_u32", k_add3}, {"v_alignbit_b32", k_align}, {"v_perm_b32", k_perm}, {"v_lshlrev_b32", k_lshl},
              {"v_pk_add_u16", k_pkadd}, {"v_xad_u32", k_xad}, {"v_mov_b32", k_mov}, {"v_xor_b32_sdwa", k_sdwa}, {"v_alignbyte_b32", k_abyte},
              {"v_lshrrev_b32", k_lshr}, {"v_or3_b32", k_or3}, {"v_lshl_or_b32", k_lshlor}};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto &k : ks) {
        for (int w = 0; w < 3; w++) k.f<<<grid, 256>>>(iters);
        CK(hipEventRecord(a));
        k.f<<<grid, 256>>>(iters);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double instr_per_simd = 8.0 * iters * 64;  // 8 waves x iters x 64 instructions
        printf("%-16s %8.3f ms  %5.2f ns/instr/SIMD  (= %.2f cycles at 2.4 GHz)\n", k.n, ms,
               ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    }
    return 0;
}
