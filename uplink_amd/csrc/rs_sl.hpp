// Straight-line rebuild bodies: generated GF(2^8) multiply-accumulate code for
// one runtime matrix (host side; rs_sl_codegen.cpp).
//
// The jump-table body (rs_device.hpp jt_inputs) multiplies a runtime
// coefficient in with a call per (row, input) into a leaf, the accumulator row
// chosen by VGPR index mode; both cost VALU issue (index mode
// ~8 us, the calls ~4 us of an all-parity RS(29,80) rebuild).  For a matrix
// that is used over many stripes (a decode plan) the library instead writes
// the whole product as straight-line code: for each (pass, chunk of inputs,
// wave row group) one code segment that reads the chunk's bit planes from
// LDS, forms only the 4-plane combinations its coefficients use and applies
// one v_bitop3 (or v_xor) per (row, plane, input) on fixed registers, i.e.
// the compile-time encoder's body with the coefficients of this matrix.  The
// segments go into the code region of a template code object
// (rs_sl_region.hip), which is loaded as a module per plan; the
// runtime-matrix kernel calls segment (pass, chunk, group) through a table
// of absolute addresses, once per chunk.
//
// Register contract (shared with rs_matmul_jt<NW, true> in rs_kernels.hip;
// the same registers as the jump table's): accumulators v[32:95] (row o,
// plane p at v[32 + 8o + p]); v[96:125] scratch -- the input's planes 0-3 in
// v[96:99] and 4-7 in v[100:103], then the 4-plane combinations; v126 = LDS
// byte address of the chunk's first input for this lane, in the wide layout of
// rs_device.hpp slice_inputs (input jj at +2048 jj, planes 0-3 of the lane as
// one 16-byte word at +0, planes 4-7 at +1024; the lane's 16 bytes are folded
// into v126); return address s[48:49].  A chunk is at most chunk_inputs(nw)
// inputs; the inputs are dealt evenly over ceil(nin / chunk_inputs(nw)) chunks.
// Generated code touches nothing else: no memory but LDS reads, no scalar
// registers, no M0.
#pragma once
#include <stdint.h>

#include <vector>

// marker words at the start of the template's region, and its size
#define UPLINK_SL_MAGIC0 0x5ec7a11e
#define UPLINK_SL_MAGIC1 0x0b0d1e50
#define UPLINK_SL_MAGIC2 0x2981e4c0
#define UPLINK_SL_MAGIC3 0x7e91a7e5
// code space per plan: two templates, 256 KiB and 2 MiB; a plan takes the
// smaller one its code fits (rs_sl_region.hip is built once per size)
#define UPLINK_SL_REGION_WORDS_SMALL 65536
#define UPLINK_SL_REGION_WORDS_LARGE 524288

namespace uplink_ec {
namespace sl {

constexpr int kRegionWordsSmall = UPLINK_SL_REGION_WORDS_SMALL;
constexpr int kRegionWords = UPLINK_SL_REGION_WORDS_LARGE;  // the most any plan may use
constexpr uint32_t kNoSegment = 0xffffffffu;

// Row split of the runtime-matrix kernel (rs_kernels.hip) with a
// straight-line body: `rows` rows in npass passes of at most nw * 8, each
// pass's rows dealt to the nw groups (waves).
struct Split {
    int nw, npass;
    int rbase(int pass, int g, int rows) const;
    int count(int pass, int g, int rows) const;
};
Split split_for(int rows);  // the kernel launch (launch_matmul_sl) uses the same split

// Inputs per chunk (the most; the inputs are dealt evenly over
// ceil(nin / chunk_inputs) chunks): 2 per wave.  -DUPLINK_SL_CHUNK2 sets the
// 2-wave figure for A/B builds: 4, 6 or 8 inputs (RS(29,80) in 8, 5 or 4
// chunks, each a barrier and a round trip to memory) rebuild within 0.2 %
// of each other (profiles/r04/exp/ab_chunk.log).
#ifndef UPLINK_SL_CHUNK2
#define UPLINK_SL_CHUNK2 4
#endif
constexpr int chunk_inputs(int nw) { return nw == 2 ? UPLINK_SL_CHUNK2 : 2 * nw; }

// Generate the segments of M (rows x nin, row-major) into `code` (cap words,
// pre-filled by the caller).  seg_off receives, for [pass][chunk][group], the
// byte offset of that segment in the region (kNoSegment when the group has no
// rows in that pass).  Returns the number of words used, or 0 when the code
// does not fit in cap words.  Any plan of up to 128 rows and 128 inputs fits
// kRegionWords.
size_t generate(const uint8_t *M, int rows, int nin, uint32_t *code, size_t cap, std::vector<uint32_t> &seg_off);

// The template code object (an ELF) with room for `words` words of code
// (the small template if they fit it, else the large one), its region
// restored (marker words + s_endpgm fill); region_off receives the byte
// offset of the region in it and region_words its size.
std::vector<uint8_t> template_image(size_t words, size_t *region_off, size_t *region_words);

}  // namespace sl
}  // namespace uplink_ec
