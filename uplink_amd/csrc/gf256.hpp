// Host-side GF(2^8) helpers on top of gf256_field.hpp: the k x k inversion of
// a decode matrix.
#pragma once
#include <vector>

#include "gf256_field.hpp"

namespace uplink_ec {

// Gauss-Jordan inverse over GF(2^8) (row pivoting); returns false if singular.
// Host-side setup for the decode matrix, never on the data path.
inline bool gf_invert(uint8_t *m, int k) {
    std::vector<uint8_t> aug((size_t)k * 2 * k);
    const int w = 2 * k;
    for (int r = 0; r < k; r++) {
        for (int c = 0; c < k; c++) aug[r * w + c] = m[r * k + c];
        for (int c = 0; c < k; c++) aug[r * w + k + c] = (uint8_t)(r == c);
    }
    for (int c = 0; c < k; c++) {
        int p = -1;
        for (int r = c; r < k; r++)
            if (aug[r * w + c]) { p = r; break; }
        if (p < 0) return false;
        if (p != c)
            for (int j = 0; j < w; j++) {
                uint8_t t = aug[p * w + j];
                aug[p * w + j] = aug[c * w + j];
                aug[c * w + j] = t;
            }
        const uint8_t iv = gf_inv(aug[c * w + c]);
        for (int j = 0; j < w; j++) aug[c * w + j] = gf_mul(iv, aug[c * w + j]);
        for (int r = 0; r < k; r++) {
            if (r == c) continue;
            const uint8_t f = aug[r * w + c];
            if (!f) continue;
            for (int j = 0; j < w; j++) aug[r * w + j] ^= gf_mul(f, aug[c * w + j]);
        }
    }
    for (int r = 0; r < k; r++)
        for (int c = 0; c < k; c++) m[r * k + c] = aug[r * w + k + c];
    return true;
}

}  // namespace uplink_ec
