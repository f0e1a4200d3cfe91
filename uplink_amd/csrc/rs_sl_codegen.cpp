// Straight-line rebuild bodies: code generation (see rs_sl.hpp for the design
// and the register contract).
//
// Five gfx950 instruction forms are emitted, encoded here directly (each
// encoding is checked against the LLVM disassembler and a CPU emulation of
// the generated code in tests/test_sl_codegen.py):
//   ds_read_b128   v[D:D+3], v126 offset:O  planes 0-3 / 4-7 of input jj: O = 2048 jj (+ 1024)
//   s_waitcnt      lgkmcnt(N)
//   v_xor_b32_e32  vD, vA, vB            4-plane combinations; single-combination rows
//   v_bitop3_b32   vD, vD, vL, vH 0x96   acc ^= lo[L] ^ hi[H]
//   s_setpc_b64    s[48:49]              return to the calling kernel
#include <stdlib.h>
#include <string.h>

#include "gf256_field.hpp"
#include "rs_sl.hpp"
#include "rs_sl_image.inc"

namespace uplink_ec {
namespace sl {

namespace {

constexpr int kAcc = 32, kXa = 126;
constexpr int kRows = 8;  // accumulator rows per wave (rs_kernels.hip kJtRows)

// The input's planes land by two ds_read_b128: planes 0-3 (lo[1], lo[2],
// lo[4], lo[8]) in v[96:99], planes 4-7 (hi[...]) in v[100:103]; the other
// combinations follow, lo in v[104:114], hi in v[115:125].
constexpr int combo_slot(int m) {  // index of m among the 11 multi-bit nibbles
    int i = 0;
    for (int x = 1; x < m; x++) i += (x & (x - 1)) != 0;
    return i;
}
uint32_t lo_reg(int L) {
    return (uint32_t)((L & (L - 1)) == 0 ? 96 + (L == 1 ? 0 : L == 2 ? 1 : L == 4 ? 2 : 3) : 104 + combo_slot(L));
}
uint32_t hi_reg(int H) {
    return (uint32_t)((H & (H - 1)) == 0 ? 100 + (H == 1 ? 0 : H == 2 ? 1 : H == 4 ? 2 : 3) : 115 + combo_slot(H));
}

struct Emitter {
    uint32_t *code;
    size_t cap, n = 0;
    bool overflow = false;
    void word(uint32_t w) {
        if (n < cap) code[n] = w;
        else overflow = true;
        n++;
    }
    void ds_read_b128(uint32_t vdst, uint32_t vaddr, uint32_t offset) {
        word(0xd9fe0000u | (offset & 0xffffu));
        word((vdst << 24) | vaddr);
    }
    void waitcnt_lgkm(uint32_t cnt) { word(0xbf8cc07fu | ((cnt & 15u) << 8)); }
    void v_xor(uint32_t vdst, uint32_t va, uint32_t vb) { word((0x15u << 25) | (vdst << 17) | (vb << 9) | (256u + va)); }
    void v_bitop3_xor3(uint32_t vdst, uint32_t va, uint32_t vb, uint32_t vc) {
        word(0xd2340200u | vdst);
        word(0xd0000000u | ((256u + vc) << 18) | ((256u + vb) << 9) | (256u + va));
    }
    void s_setpc_ret() { word(0xbe801d30u); }
};

int low_bit(int m) { return m & -m; }

// One segment: inputs j0 .. j0+jn-1 of the chunk into rows rbase .. rbase+cnt-1.
void emit_segment(Emitter &e, const uint8_t *M, int nin, int rbase, int cnt, int j0, int jn) {
    for (int jj = 0; jj < jn; jj++) {
        const int j = j0 + jj;
        bool need_lo[16] = {}, need_hi[16] = {};
        bool any = false;
        for (int o = 0; o < cnt; o++) {
            const uint8_t c = M[(size_t)(rbase + o) * nin + j];
            if (!c) continue;
            for (int p = 0; p < 8; p++) {
                const uint8_t row = mul_bitrow(c, p);
                need_lo[row & 15] = true;
                need_hi[row >> 4] = true;
                any = true;
            }
        }
        if (!any) continue;
        // closure: lo[m] = lo[m ^ low(m)] ^ x[bit(low(m))]
        for (int m = 15; m >= 1; m--) {
            if (need_lo[m]) need_lo[m ^ low_bit(m)] = need_lo[low_bit(m)] = true;
            if (need_hi[m]) need_hi[m ^ low_bit(m)] = need_hi[low_bit(m)] = true;
        }
        need_lo[0] = need_hi[0] = false;
        // input jj at 2048 jj: planes 0-3 of the lane at +16 lane, planes 4-7 at +1024 +16 lane
        const uint32_t base = (uint32_t)jj * 2048u;
        bool any_lo = false, any_hi = false;
        for (int q = 0; q < 4; q++) any_lo |= need_lo[1 << q], any_hi |= need_hi[1 << q];
        const int nhi = any_hi ? 1 : 0;
        if (any_lo) e.ds_read_b128(96, kXa, base);
        if (any_hi) e.ds_read_b128(100, kXa, base + 1024u);
        bool lo_combo = false, hi_combo = false;
        for (int m = 1; m < 16; m++) {
            if (m != low_bit(m)) lo_combo |= need_lo[m], hi_combo |= need_hi[m];
        }
        // the low planes land first (LDS returns in order): combine them while the high ones arrive
        if (lo_combo) {
            e.waitcnt_lgkm((uint32_t)nhi);
            for (int m = 1; m < 16; m++)
                if (need_lo[m] && m != low_bit(m)) e.v_xor(lo_reg(m), lo_reg(m ^ low_bit(m)), lo_reg(low_bit(m)));
        }
        e.waitcnt_lgkm(0);
        if (hi_combo)
            for (int m = 1; m < 16; m++)
                if (need_hi[m] && m != low_bit(m)) e.v_xor(hi_reg(m), hi_reg(m ^ low_bit(m)), hi_reg(low_bit(m)));
        for (int o = 0; o < cnt; o++) {
            const uint8_t c = M[(size_t)(rbase + o) * nin + j];
            if (!c) continue;
            for (int p = 0; p < 8; p++) {
                const uint8_t row = mul_bitrow(c, p);
                const int L = row & 15, H = row >> 4;
                const uint32_t acc = (uint32_t)(kAcc + kRows * o + p);
                if (L && H) e.v_bitop3_xor3(acc, acc, lo_reg(L), hi_reg(H));
                else if (L) e.v_xor(acc, acc, lo_reg(L));
                else if (H) e.v_xor(acc, acc, hi_reg(H));
            }
        }
    }
    e.s_setpc_ret();
}

}  // namespace

int Split::rbase(int pass, int g, int rows) const {
    const int p0 = pass * rows / npass, prow = (pass + 1) * rows / npass - p0;
    return p0 + g * prow / nw;
}

int Split::count(int pass, int g, int rows) const {
    const int p0 = pass * rows / npass, prow = (pass + 1) * rows / npass - p0;
    return p0 + (g + 1) * prow / nw - rbase(pass, g, rows);
}

Split split_for(int rows) {
    Split s;
    // 2-4 waves up to 32 rows, 8 past them (2 workgroups per CU), so up to 64
    // rows take one pass over the inputs.  15-16 rows on 3 waves (5-6 rows
    // each), not 2 (8 each): RS(29,80) m = 16 394 vs 401-405 us per 16 segments
    // (profiles/r04/exp/ab_rows_per_wave.log).  Not 5-7 waves: a 127-VGPR wave
    // leaves a CU 16 wave slots, which 5-wave workgroups fill to about 10 (SQ
    // wave cycles), so m = 29 on 5 waves took 590-614 against 412 us on 4, and
    // Decode at k+20 (33-40 rows) 48 against 43 us per segment on 8
    // (profiles/r04/exp/nw8_decode.log).  -D overrides for A/B builds.
#ifndef UPLINK_SL_TWO_WAVE_ROWS
#define UPLINK_SL_TWO_WAVE_ROWS 14
#endif
#ifndef UPLINK_SL_WIDE_ROWS_PER_WAVE  // rows per wave past 32 rows (at most kRows)
#define UPLINK_SL_WIDE_ROWS_PER_WAVE 4
#endif
    // (the env var of the same name overrides it for A/B runs; read once, so the
    // generated code and the launches of a process always agree)
    static const int RW = [] {
        const char *e = getenv("UPLINK_SL_WIDE_ROWS_PER_WAVE");
        const int v = e ? atoi(e) : UPLINK_SL_WIDE_ROWS_PER_WAVE;
        return v >= 4 && v <= kRows ? v : UPLINK_SL_WIDE_ROWS_PER_WAVE;
    }();
    s.nw = rows <= UPLINK_SL_TWO_WAVE_ROWS ? 2
           : rows <= 3 * kRows                ? 3
           : rows <= 4 * kRows                ? 4
           : rows >= 8 * RW                   ? 8
                                              : (rows + RW - 1) / RW;
    s.npass = rows > 0 ? (rows + s.nw * kRows - 1) / (s.nw * kRows) : 1;
    return s;
}

size_t generate(const uint8_t *M, int rows, int nin, uint32_t *code, size_t cap, std::vector<uint32_t> &seg_off) {
    const Split sp = split_for(rows);
    const int jc = chunk_inputs(sp.nw), nchunks = (nin + jc - 1) / jc, ch_size = (nin + nchunks - 1) / nchunks;
    seg_off.assign((size_t)sp.npass * nchunks * sp.nw, kNoSegment);
    Emitter e{code, cap};
    // the region's first 64 words stay s_endpgm: no segment starts at offset 0
    e.n = 64;
    for (int pass = 0; pass < sp.npass; pass++)
        for (int ch = 0; ch < nchunks; ch++)
            for (int g = 0; g < sp.nw; g++) {
                const int cnt = sp.count(pass, g, rows);
                if (cnt <= 0) continue;
                // segments start on 64-byte instruction-cache lines
                while (e.n & 15) e.word(0xbf810000u);
                seg_off[((size_t)pass * nchunks + ch) * sp.nw + g] = (uint32_t)(e.n * 4);
                const int j0 = ch * ch_size, jn = nin - j0 < ch_size ? nin - j0 : ch_size;
                emit_segment(e, M, nin, sp.rbase(pass, g, rows), cnt, j0, jn);
            }
    if (e.overflow) return 0;
    return e.n;
}

std::vector<uint8_t> template_image(size_t words, size_t *region_off, size_t *region_words) {
    const bool small = words <= (size_t)kRegionWordsSmall;
    const unsigned char *head = small ? kSlHead : kSlHeadLarge, *tail = small ? kSlTail : kSlTailLarge;
    const size_t nhead = small ? sizeof(kSlHead) : sizeof(kSlHeadLarge);
    const size_t ntail = small ? sizeof(kSlTail) : sizeof(kSlTailLarge);
    const size_t nw = small ? (size_t)kRegionWordsSmall : (size_t)kRegionWords;
    std::vector<uint8_t> img(nhead + nw * 4 + ntail);
    memcpy(img.data(), head, nhead);
    uint8_t *r = img.data() + nhead;
    const uint32_t magic[4] = {UPLINK_SL_MAGIC0, UPLINK_SL_MAGIC1, UPLINK_SL_MAGIC2, UPLINK_SL_MAGIC3};
    for (size_t i = 0; i < nw; i++) {
        const uint32_t w = i < 4 ? magic[i] : 0xbf810000u;
        memcpy(r + 4 * i, &w, 4);
    }
    memcpy(img.data() + nhead + nw * 4, tail, ntail);
    *region_off = nhead;
    *region_words = nw;
    return img;
}

}  // namespace sl
}  // namespace uplink_ec
