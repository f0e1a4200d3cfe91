// GF(2^8) arithmetic and the systematic generator matrix of the Reed-Solomon
// code that storj/uplink's eestream uses (storj.io/infectious v0.0.2, reached
// through private/eestream/fec.go:15-17 and rs.go:11-61).
//
// Field: x^8+x^4+x^3+x^2+1 (0x11d), alpha = 2 (the zfec field infectious ports).
// Generator: G[i][j] = L_j(x_i), the Lagrange basis over the points
// x_0 = 0, x_r = alpha^(r-1).  This equals infectious' inverted-Vandermonde
// construction; tests/test_oracle.py pins it against
// the oracle's zfec construction.
//
// Everything here is constexpr and self-contained (no library headers), so
// the compile-time-G encoders can take G as a constant both in the library
// build and when hiprtc compiles an encoder for a new (k, n) at run time
// (rs_encoder_jit.cpp).
#pragma once
#include "rs_types.hpp"

namespace uplink_ec {

struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
    uint8_t inv[256];
};

constexpr GfTables make_gf_tables() {
    GfTables t{};
    int x = 1;
    for (int i = 0; i < 255; i++) {
        t.exp[i] = (uint8_t)x;
        t.exp[i + 255] = (uint8_t)x;
        t.log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11d;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    t.log[0] = 0;  // unused: callers test for zero first
    t.inv[0] = 0;
    for (int a = 1; a < 256; a++) t.inv[a] = t.exp[255 - t.log[a]];
    return t;
}

inline constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kGf.exp[kGf.log[a] + kGf.log[b]];
}
constexpr uint8_t gf_inv(uint8_t a) { return kGf.inv[a]; }
constexpr uint8_t gf_point(int r) { return r == 0 ? 0 : kGf.exp[(r - 1) % 255]; }

// G[i][j] for 0 <= i < n, 0 <= j < k
constexpr uint8_t gen_entry(int k, int i, int j) {
    uint8_t num = 1, den = 1;
    const uint8_t xi = gf_point(i), xj = gf_point(j);
    for (int m = 0; m < k; m++) {
        if (m == j) continue;
        const uint8_t xm = gf_point(m);
        num = gf_mul(num, (uint8_t)(xi ^ xm));
        den = gf_mul(den, (uint8_t)(xj ^ xm));
    }
    return gf_mul(num, gf_inv(den));
}

// Row p of the 8x8 GF(2) matrix of "multiply by c": bit q set when bit p of
// c * 2^q is set.  In bit-sliced form, output plane p = XOR of input planes q
// with bit q set.
constexpr uint8_t mul_bitrow(uint8_t c, int p) {
    uint8_t row = 0;
    for (int q = 0; q < 8; q++)
        if ((gf_mul(c, (uint8_t)(1u << q)) >> p) & 1) row |= (uint8_t)(1u << q);
    return row;
}

}  // namespace uplink_ec
