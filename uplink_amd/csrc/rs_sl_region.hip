// Template code object of the straight-line rebuild bodies (rs_sl_codegen.cpp).
//
// Built on its own (hipcc --genco) and embedded in the library
// (tools/gen/embed_sl_image.py -> <build dir>/obj/rs_sl_image.inc).  Its one kernel,
// rs_sl_where, writes the absolute address of `region`: a block of code
// space inside its own text that the library fills, per decode matrix, with
// generated straight-line multiply-accumulate code before it loads the image
// as a module (hipModuleLoadData).  The runtime-matrix kernel in the library
// (rs_matmul_jt<NW, true>, rs_kernels.hip) then calls into that code.
//
// Built twice, with 256 KiB and 2 MiB regions (UPLINK_SL_REGION_WORDS).
// The kernel jumps over the region, so none of its bytes run here.  The
// region starts with four marker words (found and overwritten by the
// library) and is filled with s_endpgm; the embedding script strips the fill
// and the library restores it, so the embedded image stays small.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_sl.hpp"

#ifndef UPLINK_SL_REGION_WORDS  // the Makefile builds one image per region size
#define UPLINK_SL_REGION_WORDS UPLINK_SL_REGION_WORDS_SMALL
#endif
#define SL_STR2(x) #x
#define SL_STR(x) SL_STR2(x)

extern "C" __global__ __launch_bounds__(64) void rs_sl_where(uint64_t *out) {
    uint32_t lo, hi;
    asm volatile(
        "s_getpc_b64 s[40:41]\n"
        ".Lsl_pc%=:\n"
        "s_add_u32 s40, s40, .Lsl_region%=-.Lsl_pc%=\n"
        "s_addc_u32 s41, s41, 0\n"
        "s_mov_b32 %0, s40\n"
        "s_mov_b32 %1, s41\n"
        "s_getpc_b64 s[42:43]\n"
        ".Lsl_pc2%=:\n"
        "s_add_u32 s42, s42, .Lsl_end%=-.Lsl_pc2%=\n"
        "s_addc_u32 s43, s43, 0\n"
        "s_setpc_b64 s[42:43]\n"
        ".p2align 8\n"
        ".Lsl_region%=:\n"
        ".long " SL_STR(UPLINK_SL_MAGIC0) ", " SL_STR(UPLINK_SL_MAGIC1) ", " SL_STR(UPLINK_SL_MAGIC2) ", "
        SL_STR(UPLINK_SL_MAGIC3) "\n"
        ".fill " SL_STR(UPLINK_SL_REGION_WORDS) " - 4, 4, 0xbf810000\n"
        ".Lsl_end%=:\n"
        : "=s"(lo), "=s"(hi)
        :
        : "s40", "s41", "s42", "s43", "scc");
    // every lane stores the same word: no branch around the store
    out[0] = ((uint64_t)hi << 32) | lo;
}
