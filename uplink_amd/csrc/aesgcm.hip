// AES-256-GCM segment encryption and decryption on the GPU (SURVEY.md §8f
// row 4).
//
// Replaces, for whole segments, what the upload's splitter does through
// encryption.TransformWriterPadded(buf, NewEncrypter(EncAESGCM, &contentKey,
// &nonce, BlockSize)) (private/storage/streams/splitter/splitter.go:156,170)
// and what the download does through decryptRanger (streams/store.go:347-382):
// AES-256-GCM over blocks of InBlockSize = BlockSize - 16 plaintext bytes,
// block b sealed under nonce + b (12 bytes, little-endian increment),
// written as ciphertext || tag.  BlockSize is 29*256 (project.go:84), so an
// encrypted block is exactly one RS(29,80) stripe.  The cipher code is
// storj.io/common/encryption (go.mod:14); the CPU oracle is
// oracle/aesgcm_oracle.c, pinned by the GCM specification's test cases.
//
// One wave per GCM block.  The block's GHASH inputs (ciphertext sub-blocks
// then the length block, m of them) are padded at the front with zeros to
// 64*J slots; lane l takes slots l, l+64, ..., so loads and stores of
// consecutive lanes are consecutive 16-byte words.  Each lane runs AES-CTR on
// its sub-blocks and a Horner GHASH with multiplier H^64,
//     acc_l = sum_j Y[l+64j] * (H^64)^(J-1-j),
// then multiplies by H^(64-l); the XOR over lanes is the GHASH
//     sum_t Y[t] * H^(64J - t)
// (leading zero slots do not change it).  Lanes whose first slot is padding
// compute AES(K, J0) instead, which masks the tag.
//
// AES: T-tables in LDS, round keys in SGPRs.  GHASH: the Horner steps on an
// 8-bit table of H^64 (16 lookups per product), the final products by
// H^(64-l) on Shoup's 4-bit tables of H^1..H^64, all in LDS (20 KB per key,
// built on the host by gcm_prepare).  36.6 KB of LDS and 128 VGPRs per
// workgroup of 4 waves: four workgroups per CU.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "aesgcm.hpp"

namespace uplink_ec {
namespace {

// ---- tables (host and device) ----

constexpr uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
constexpr uint8_t gmul8(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

struct AesTables {
    uint8_t sbox[256];
    uint32_t t0[256];
    constexpr AesTables() : sbox{}, t0{} {
        uint8_t ex[256] = {}, lg[256] = {};  // powers of the generator 3
        uint8_t p = 1;
        for (int i = 0; i < 255; i++) {
            ex[i] = p;
            lg[p] = (uint8_t)i;
            p = (uint8_t)(p ^ xtime(p));
        }
        for (int x = 0; x < 256; x++) {
            const uint8_t inv = x ? ex[(255 - lg[x]) % 255] : 0;  // multiplicative inverse mod 0x11b
            uint8_t s = inv, r = inv;
            for (int i = 0; i < 4; i++) {  // affine map
                r = (uint8_t)((r << 1) | (r >> 7));
                s ^= r;
            }
            sbox[x] = (uint8_t)(s ^ 0x63);
        }
        for (int x = 0; x < 256; x++) {
            const uint8_t s = sbox[x];
            t0[x] = (uint32_t)xtime(s) << 24 | (uint32_t)s << 16 | (uint32_t)s << 8 | (uint8_t)(xtime(s) ^ s);
        }
    }
};
constexpr AesTables kAes{};
__device__ constexpr AesTables kAesDev{};

constexpr uint32_t ror32(uint32_t x, int n) { return n ? (x >> n) | (x << (32 - n)) : x; }

// Shoup's reduction constants for a 4-bit shift, placed at the top of word 0
__device__ constexpr uint32_t kRem4[16] = {0x0000u << 16, 0x1C20u << 16, 0x3840u << 16, 0x2460u << 16,
                                           0x7080u << 16, 0x6CA0u << 16, 0x48C0u << 16, 0x54E0u << 16,
                                           0xE100u << 16, 0xFD20u << 16, 0xD940u << 16, 0xC560u << 16,
                                           0x9180u << 16, 0x8DA0u << 16, 0xA9C0u << 16, 0xB5E0u << 16};

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

// Reduction constants for an 8-bit shift (the bits of the shifted-out byte
// folded back through x^128 = x^7 + x^2 + x + 1, reflected): the top 16 bits of word 0
struct Rem8 {
    uint16_t r[256];
    constexpr Rem8() : r{} {
        for (int b = 0; b < 256; b++) {
            uint64_t hi = 0, lo = (uint64_t)b;
            for (int i = 0; i < 8; i++) {
                const uint64_t carry = lo & 1;
                lo = (lo >> 1) | (hi << 63);
                hi = (hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
            }
            r[b] = (uint16_t)(hi >> 48);
        }
    }
};
__device__ constexpr Rem8 kRem8{};

// T-table layout: T0 alone, replicated kCopies times with copy c of entry x
// at word x*kCopies + c; lane l reads copy l % kCopies; T1..T3 are rotations
// of T0.  16 copies (16 KB) with four workgroups per CU beat 32 copies with
// three (DESIGN.md §4c has the measured alternatives).
#ifndef UPLINK_GCM_COPIES  // (-D for A/B builds)
#define UPLINK_GCM_COPIES 16
#endif
constexpr int kCopies = UPLINK_GCM_COPIES;

struct Lds {
    uint32_t t[256 * kCopies];
    uint32_t rem[16];
    uint32_t htab[64][16][4];    // H^1..H^64
    uint32_t h8[256][4];         // byte * H^64
    uint16_t rem8[256];          // (16 bits each: with three workgroups' tables the CU's LDS is full)
};

// Tk[x] for this lane
template <int k>
__device__ __forceinline__ uint32_t T(const Lds &L, uint32_t x, uint32_t copy) {
    const uint32_t v = L.t[x * kCopies + copy];
    return k ? __builtin_amdgcn_alignbit(v, v, 8 * k) : v;
}

// AES-256 of the big-endian words s[4] with round keys rk (SGPRs), T-tables in LDS
__device__ __forceinline__ void aes_encrypt(uint32_t (&s)[4], const uint32_t *__restrict__ rk, const Lds &L) {
    const uint32_t cp = threadIdx.x % kCopies;
    uint32_t a = s[0] ^ rk[0], b = s[1] ^ rk[1], c = s[2] ^ rk[2], d = s[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < 14; r++) {
        const uint32_t e = T<0>(L, a >> 24, cp) ^ T<1>(L, (b >> 16) & 255, cp) ^ T<2>(L, (c >> 8) & 255, cp) ^ T<3>(L, d & 255, cp) ^ rk[4 * r];
        const uint32_t f = T<0>(L, b >> 24, cp) ^ T<1>(L, (c >> 16) & 255, cp) ^ T<2>(L, (d >> 8) & 255, cp) ^ T<3>(L, a & 255, cp) ^ rk[4 * r + 1];
        const uint32_t g = T<0>(L, c >> 24, cp) ^ T<1>(L, (d >> 16) & 255, cp) ^ T<2>(L, (a >> 8) & 255, cp) ^ T<3>(L, b & 255, cp) ^ rk[4 * r + 2];
        const uint32_t h = T<0>(L, d >> 24, cp) ^ T<1>(L, (a >> 16) & 255, cp) ^ T<2>(L, (b >> 8) & 255, cp) ^ T<3>(L, c & 255, cp) ^ rk[4 * r + 3];
        a = e, b = f, c = g, d = h;
    }
    // last round: S-box bytes, picked out of the T-tables (T2 MSB, T3 byte 2, T0 byte 1, T1 LSB = S[x])
    s[0] = ((T<2>(L, a >> 24, cp) & 0xff000000u) | (T<3>(L, (b >> 16) & 255, cp) & 0x00ff0000u) |
            (T<0>(L, (c >> 8) & 255, cp) & 0x0000ff00u) | (T<1>(L, d & 255, cp) & 0xffu)) ^ rk[56];
    s[1] = ((T<2>(L, b >> 24, cp) & 0xff000000u) | (T<3>(L, (c >> 16) & 255, cp) & 0x00ff0000u) |
            (T<0>(L, (d >> 8) & 255, cp) & 0x0000ff00u) | (T<1>(L, a & 255, cp) & 0xffu)) ^ rk[57];
    s[2] = ((T<2>(L, c >> 24, cp) & 0xff000000u) | (T<3>(L, (d >> 16) & 255, cp) & 0x00ff0000u) |
            (T<0>(L, (a >> 8) & 255, cp) & 0x0000ff00u) | (T<1>(L, b & 255, cp) & 0xffu)) ^ rk[58];
    s[3] = ((T<2>(L, d >> 24, cp) & 0xff000000u) | (T<3>(L, (a >> 16) & 255, cp) & 0x00ff0000u) |
            (T<0>(L, (b >> 8) & 255, cp) & 0x0000ff00u) | (T<1>(L, c & 255, cp) & 0xffu)) ^ rk[59];
}

// z = x * E in GF(2^128) (GCM bit order), E given by its 4-bit table; words big-endian
__device__ __forceinline__ void gf_mul(uint32_t (&z)[4], const uint32_t (&x)[4], const uint32_t (*tab)[4],
                                       const uint32_t *rem) {
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        const uint32_t byte = (x[i >> 2] >> ((3 - (i & 3)) * 8)) & 0xff;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint32_t nib = h ? byte >> 4 : byte & 15;
            if (i != 15 || h) {
                const uint32_t r = rem[z3 & 15];
                z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
                z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
                z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
                z0 = (z0 >> 4) ^ r;
            }
            z0 ^= tab[nib][0], z1 ^= tab[nib][1], z2 ^= tab[nib][2], z3 ^= tab[nib][3];
        }
    }
    z[0] = z0, z[1] = z1, z[2] = z2, z[3] = z3;
}

// z = x * E with E's 8-bit table (one lookup and one reduction per byte: half
// the steps of gf_mul's 4-bit table)
__device__ __forceinline__ void gf_mul8(uint32_t (&z)[4], const uint32_t (&x)[4], const uint32_t (*tab)[4],
                                        const uint16_t *rem8) {
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        const uint32_t byte = (x[i >> 2] >> ((3 - (i & 3)) * 8)) & 0xff;
        if (i != 15) {
            const uint32_t r = (uint32_t)rem8[z3 & 0xff] << 16;
            z3 = __builtin_amdgcn_alignbit(z2, z3, 8);
            z2 = __builtin_amdgcn_alignbit(z1, z2, 8);
            z1 = __builtin_amdgcn_alignbit(z0, z1, 8);
            z0 = (z0 >> 8) ^ r;
        }
        const uint4 t = *reinterpret_cast<const uint4 *>(tab[byte]);
        z0 ^= t.x, z1 ^= t.y, z2 ^= t.z, z3 ^= t.w;
    }
    z[0] = z0, z[1] = z1, z[2] = z2, z[3] = z3;
}

// bytes [0, n) of the 16-byte word at p (n < 16), big-endian words, zero padded
__device__ __forceinline__ void load_tail(const uint8_t *p, uint32_t n, uint32_t (&w)[4]) {
    w[0] = w[1] = w[2] = w[3] = 0;
    for (uint32_t i = 0; i < n; i++) w[i >> 2] |= (uint32_t)p[i] << (24 - 8 * (i & 3));
}

#ifndef UPLINK_GCM_WAVES_PER_EU  // (-D for A/B builds: a register budget of 512 / this per lane)
#define UPLINK_GCM_WAVES_PER_EU 4
#endif
template <bool kOpen>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(UPLINK_GCM_WAVES_PER_EU))) void gcm_blocks(
    GcmBatch a, uint32_t wgs_per_seg) {
    __shared__ Lds L;
    const uint32_t seg = blockIdx.x / wgs_per_seg;
    const uint32_t wg = blockIdx.x % wgs_per_seg;
    const GcmSched *ks = a.sched + seg;
    for (int i = threadIdx.x; i < 256 * kCopies; i += blockDim.x) L.t[i] = kAesDev.t0[i / kCopies];
    if (threadIdx.x < 16) L.rem[threadIdx.x] = kRem4[threadIdx.x];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(&ks->htab[0][0][0]);
        uint4 *dst = reinterpret_cast<uint4 *>(&L.htab[0][0][0]);
        for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) dst[i] = src[i];
        const uint4 *s8 = reinterpret_cast<const uint4 *>(&ks->h64_8[0][0]);
        uint4 *d8 = reinterpret_cast<uint4 *>(&L.h8[0][0]);
        for (int i = threadIdx.x; i < 256; i += blockDim.x) {
            d8[i] = s8[i];
            L.rem8[i] = kRem8.r[i];
        }
    }
    __syncthreads();
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; i++) rk[i] = ks->rk[i];  // uniform: scalar loads

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t ib = a.in_block;
    const uint32_t nsub = (ib + 15) / 16, tail = ib & 15;
    const uint32_t slots = nsub + 1;  // + the length block
    const uint32_t steps = (slots + 63) / 64, pad = steps * 64 - slots;
    const uint8_t *nonce = a.nonces + 12ull * seg;
    uint32_t nw[3];
#pragma unroll
    for (int i = 0; i < 3; i++)
        nw[i] = (uint32_t)nonce[4 * i] | (uint32_t)nonce[4 * i + 1] << 8 | (uint32_t)nonce[4 * i + 2] << 16 |
                (uint32_t)nonce[4 * i + 3] << 24;  // little-endian 96-bit integer
    const uint64_t clen_bits = (uint64_t)ib * 8;

    for (uint32_t b = wg * 4 + wave; b < a.nblocks; b += wgs_per_seg * 4) {
        // nonce + b, little-endian with carry across the 12 bytes; then big-endian words for AES
        uint32_t n0 = nw[0], n1 = nw[1], n2 = nw[2];
        {
            const uint64_t lo = (uint64_t)n0 + (uint32_t)b;
            n0 = (uint32_t)lo;
            const uint64_t mid = (uint64_t)n1 + (lo >> 32);
            n1 = (uint32_t)mid;
            n2 += (uint32_t)(mid >> 32);
        }
        const uint32_t j0w0 = bswap(n0), j0w1 = bswap(n1), j0w2 = bswap(n2);
        const uint8_t *src = a.in + (int64_t)seg * a.in_seg_stride + (int64_t)b * a.in_blk_stride;
        uint8_t *dst = a.out + (int64_t)seg * a.out_seg_stride + (int64_t)b * a.out_blk_stride;
        uint32_t acc[4] = {0, 0, 0, 0}, ekj0[4] = {0, 0, 0, 0};
        for (uint32_t j = 0; j < steps; j++) {
            const uint32_t t = (uint32_t)lane + 64 * j;
            const bool is_data = t >= pad && t + 1 < pad + slots;
            const bool is_len = t + 1 == pad + slots;
            const uint32_t sidx = t - pad;
            // every lane runs the AES (no divergent second pass): data lanes on their counter block,
            // padding lanes on J0 (the tag mask), the length-block lane on a value it ignores
            uint32_t ks4[4] = {j0w0, j0w1, j0w2, is_data ? 2 + sidx : 1};
            aes_encrypt(ks4, rk, L);
            uint32_t y[4] = {0, 0, 0, 0};
            if (is_data) {
                const uint32_t n = (sidx + 1 == nsub && tail) ? tail : 16;
                uint32_t in4[4];
                if (n == 16) {
                    const uint4 w = *reinterpret_cast<const uint4 *>(src + 16ull * sidx);
                    in4[0] = bswap(w.x), in4[1] = bswap(w.y), in4[2] = bswap(w.z), in4[3] = bswap(w.w);
                } else {
                    load_tail(src + 16ull * sidx, n, in4);
                }
                uint32_t o4[4];
#pragma unroll
                for (int q = 0; q < 4; q++) o4[q] = in4[q] ^ ks4[q];
                if (n == 16) {
                    *reinterpret_cast<uint4 *>(dst + 16ull * sidx) =
                        make_uint4(bswap(o4[0]), bswap(o4[1]), bswap(o4[2]), bswap(o4[3]));
                } else {
                    for (uint32_t i = 0; i < n; i++) dst[16ull * sidx + i] = (uint8_t)(o4[i >> 2] >> (24 - 8 * (i & 3)));
                    // GHASH sees the zero-padded ciphertext
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t lo = 4 * q;
                        const uint32_t keep = n >= lo + 4 ? 0xffffffffu : n <= lo ? 0u : ~(0xffffffffu >> (8 * (n - lo)));
                        o4[q] &= keep;
                        in4[q] &= keep;
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) y[q] = kOpen ? in4[q] : o4[q];
            } else if (is_len) {  // len(A) = 0 || len(C) in bits
                y[2] = (uint32_t)(clen_bits >> 32);
                y[3] = (uint32_t)clen_bits;
            } else if (j == 0) {
#pragma unroll
                for (int q = 0; q < 4; q++) ekj0[q] = ks4[q];
            }
            // Horner step with H^64
            if (j) {
                uint32_t m[4];
                gf_mul8(m, acc, L.h8, L.rem8);
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] = m[q] ^ y[q];
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] = y[q];
            }
        }
        {
            uint32_t m[4];
            gf_mul(m, acc, L.htab[63 - lane], L.rem);
#pragma unroll
            for (int q = 0; q < 4; q++) acc[q] = m[q];
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
            for (int q = 0; q < 4; q++) acc[q] ^= __shfl_xor(acc[q], off);
        if (pad == 0) {  // no padding lane computed AES(K, J0): lane 0 does it now
            if (lane == 0) {
                uint32_t k4[4] = {j0w0, j0w1, j0w2, 1};
                aes_encrypt(k4, rk, L);
#pragma unroll
                for (int q = 0; q < 4; q++) ekj0[q] = k4[q];
            }
        }
        if (lane == 0) {
            uint32_t tag[4];
#pragma unroll
            for (int q = 0; q < 4; q++) tag[q] = acc[q] ^ ekj0[q];
            if (kOpen) {
                const uint8_t *given = src + ib;
                bool ok = true;
                for (int i = 0; i < 16; i++) ok &= given[i] == (uint8_t)(tag[i >> 2] >> (24 - 8 * (i & 3)));
                if (!ok) atomicMin(a.status + seg, (int32_t)b);
            } else {
                for (int i = 0; i < 16; i++) dst[ib + i] = (uint8_t)(tag[i >> 2] >> (24 - 8 * (i & 3)));
            }
        }
    }
}

// ---- host helpers ----

uint32_t sub_word(uint32_t w) {
    return (uint32_t)kAes.sbox[w >> 24] << 24 | (uint32_t)kAes.sbox[(w >> 16) & 255] << 16 |
           (uint32_t)kAes.sbox[(w >> 8) & 255] << 8 | kAes.sbox[w & 255];
}

void key_expand(const uint8_t key[32], uint32_t rk[60]) {
    for (int i = 0; i < 8; i++)
        rk[i] = (uint32_t)key[4 * i] << 24 | (uint32_t)key[4 * i + 1] << 16 | (uint32_t)key[4 * i + 2] << 8 | key[4 * i + 3];
    uint8_t rcon = 1;
    for (int i = 8; i < 60; i++) {
        uint32_t t = rk[i - 1];
        if (i % 8 == 0) {
            t = sub_word(ror32(t, 24)) ^ ((uint32_t)rcon << 24);
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            t = sub_word(t);
        }
        rk[i] = rk[i - 8] ^ t;
    }
}

// 128-bit GCM field element as (hi, lo) big-endian halves
struct U128 {
    uint64_t hi, lo;
};
U128 gf_mul_bits(U128 x, U128 y) {  // GCM spec Algorithm 1
    U128 z{0, 0}, v = y;
    for (int i = 0; i < 128; i++) {
        const uint64_t bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        if (bit) z.hi ^= v.hi, z.lo ^= v.lo;
        const uint64_t carry = v.lo & 1;
        v.lo = (v.lo >> 1) | (v.hi << 63);
        v.hi = (v.hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
    }
    return z;
}

// tab[b] = b * e for every byte b (bit 7 of b the coefficient of x^0)
void shoup_table8(U128 e, uint32_t tab[256][4]) {
    U128 t[256] = {};
    t[128] = e;
    U128 v = e;
    for (int i = 64; i > 0; i >>= 1) {
        const uint64_t carry = v.lo & 1;
        v.lo = (v.lo >> 1) | (v.hi << 63);
        v.hi = (v.hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
        t[i] = v;
    }
    for (int i = 2; i < 256; i <<= 1)
        for (int j = 1; j < i; j++) t[i + j] = U128{t[i].hi ^ t[j].hi, t[i].lo ^ t[j].lo};
    for (int i = 0; i < 256; i++) {
        tab[i][0] = (uint32_t)(t[i].hi >> 32), tab[i][1] = (uint32_t)t[i].hi;
        tab[i][2] = (uint32_t)(t[i].lo >> 32), tab[i][3] = (uint32_t)t[i].lo;
    }
}

void shoup_table(U128 e, uint32_t tab[16][4]) {
    U128 t[16] = {};
    t[8] = e;
    U128 v = e;
    for (int i = 4; i > 0; i >>= 1) {  // t[i] = e * x^(3 - log2 i): one right shift with reduction each
        const uint64_t carry = v.lo & 1;
        v.lo = (v.lo >> 1) | (v.hi << 63);
        v.hi = (v.hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
        t[i] = v;
    }
    for (int i = 2; i < 16; i <<= 1)
        for (int j = 1; j < i; j++) t[i + j] = U128{t[i].hi ^ t[j].hi, t[i].lo ^ t[j].lo};
    for (int i = 0; i < 16; i++) {
        tab[i][0] = (uint32_t)(t[i].hi >> 32), tab[i][1] = (uint32_t)t[i].hi;
        tab[i][2] = (uint32_t)(t[i].lo >> 32), tab[i][3] = (uint32_t)t[i].lo;
    }
}

}  // namespace

void aes256_encrypt_block(const uint32_t rk[60], const uint8_t in[16], uint8_t out[16]) {
    uint32_t s[4];
    for (int i = 0; i < 4; i++)
        s[i] = ((uint32_t)in[4 * i] << 24 | (uint32_t)in[4 * i + 1] << 16 | (uint32_t)in[4 * i + 2] << 8 | in[4 * i + 3]) ^
               rk[i];
    for (int r = 1; r <= 14; r++) {
        uint8_t b[16];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) b[4 * i + j] = kAes.sbox[(s[(i + j) % 4] >> (24 - 8 * j)) & 255];  // SubBytes+ShiftRows
        for (int i = 0; i < 4; i++) {
            uint8_t *c = b + 4 * i;
            uint8_t m[4] = {c[0], c[1], c[2], c[3]};
            if (r != 14) {  // MixColumns
                m[0] = (uint8_t)(gmul8(c[0], 2) ^ gmul8(c[1], 3) ^ c[2] ^ c[3]);
                m[1] = (uint8_t)(c[0] ^ gmul8(c[1], 2) ^ gmul8(c[2], 3) ^ c[3]);
                m[2] = (uint8_t)(c[0] ^ c[1] ^ gmul8(c[2], 2) ^ gmul8(c[3], 3));
                m[3] = (uint8_t)(gmul8(c[0], 3) ^ c[1] ^ c[2] ^ gmul8(c[3], 2));
            }
            s[i] = ((uint32_t)m[0] << 24 | (uint32_t)m[1] << 16 | (uint32_t)m[2] << 8 | m[3]) ^ rk[4 * r + i];
        }
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(s[i] >> (24 - 8 * j));
}

void gcm_prepare(const uint8_t key[32], GcmSched *out) {
    std::memset(out, 0, sizeof *out);
    key_expand(key, out->rk);
    uint8_t zero[16] = {0}, h[16];
    aes256_encrypt_block(out->rk, zero, h);
    U128 H{0, 0};
    for (int i = 0; i < 8; i++) H.hi = H.hi << 8 | h[i], H.lo = H.lo << 8 | h[8 + i];
    U128 p = H;
    for (int k = 0; k < 64; k++) {  // htab[k] = table of H^(k+1)
        shoup_table(p, out->htab[k]);
        if (k == 63) shoup_table8(p, out->h64_8);
        p = gf_mul_bits(p, H);
    }
}

hipError_t gcm_launch(const GcmBatch &b, bool open, hipStream_t stream) {
    if (b.nseg == 0 || b.nblocks == 0) return hipSuccess;
    if (b.in_block == 0 || b.in_block > (1u << 24)) return hipErrorInvalidValue;
    // enough workgroups to fill the chip many times over, each looping over blocks of one segment:
    // 32 per CU (8 segments: seal 167.3 us per segment, against 168.3 at 16, 174.7 at 8, 184.0 at
    // 4; profiles/r05/gcm/ab_grid*.json; UPLINK_GCM_GRID_PER_CU for A/B)
    static const uint64_t per_cu = [] {
        const char *e = getenv("UPLINK_GCM_GRID_PER_CU");
        const int v = e ? atoi(e) : 32;
        return (uint64_t)(v > 0 && v <= 64 ? v : 32);
    }();
    uint32_t wgs = (b.nblocks + 3) / 4;
    const uint32_t cap = (uint32_t)((256ull * per_cu + b.nseg - 1) / b.nseg);
    if (wgs > cap) wgs = cap < 1 ? 1 : cap;
    const dim3 grid(b.nseg * wgs);
    if (open)
        gcm_blocks<true><<<grid, 256, 0, stream>>>(b, wgs);
    else
        gcm_blocks<false><<<grid, 256, 0, stream>>>(b, wgs);
    return hipGetLastError();
}

}  // namespace uplink_ec

// ---- C-ABI (include/uplink_ec.h) ----
#include "../../include/uplink_ec.h"

namespace uplink_ec {
namespace {

__global__ void gcm_status_init(int32_t *s, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) s[i] = 0x7fffffff;
}
__global__ void gcm_status_fini(int32_t *s, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && s[i] == 0x7fffffff) s[i] = -1;
}

// PadReader padding written in place after `len` bytes of each segment
__global__ void pad_segments(uint8_t *segs, int64_t stride, uint64_t len, uint32_t p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p) return;
    uint8_t v = (uint8_t)p;
    if (i + 4 >= p) v = (uint8_t)(p >> (8 * (p - 1 - i)));  // last 4 bytes: big-endian p
    segs[(int64_t)blockIdx.y * stride + len + i] = v;
}

int gcm_fail(hipError_t e) { return e == hipSuccess ? EC_OK : (e == hipErrorInvalidValue ? EC_ERR_INVALID_ARG : EC_ERR_DEVICE); }

int gcm_run(const uint8_t *in, size_t nseg, size_t nblocks, size_t in_block, const void *keys, const uint8_t *nonces,
            uint8_t *out, int32_t *status, bool open, hipStream_t st, int64_t in_seg = 0, int64_t out_seg = 0) {
    if (nseg == 0 || nblocks == 0) return EC_OK;
    if (!in || !out || !keys || !nonces || (open && !status)) return EC_ERR_INVALID_ARG;
    if (in_block == 0 || in_block > (1u << 24) || nseg > 0xFFFFFFu || nblocks > 0x7FFFFFFFu) return EC_ERR_UNSUPPORTED;
    const int64_t ob = (int64_t)in_block + 16;
    GcmBatch b{};
    b.in = in;
    b.out = out;
    b.in_blk_stride = open ? ob : (int64_t)in_block;
    b.out_blk_stride = open ? (int64_t)in_block : ob;
    b.in_seg_stride = in_seg ? in_seg : b.in_blk_stride * (int64_t)nblocks;
    b.out_seg_stride = out_seg ? out_seg : b.out_blk_stride * (int64_t)nblocks;
    if (b.in_seg_stride < b.in_blk_stride * (int64_t)nblocks || b.out_seg_stride < b.out_blk_stride * (int64_t)nblocks ||
        ((b.in_seg_stride | b.out_seg_stride) & 15))
        return EC_ERR_INVALID_ARG;
    b.sched = static_cast<const GcmSched *>(keys);
    b.nonces = nonces;
    b.status = status;
    b.nseg = (uint32_t)nseg;
    b.nblocks = (uint32_t)nblocks;
    b.in_block = (uint32_t)in_block;
    const bool aligned = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0 &&
                         in_block % 16 == 0;
    if (!aligned) return EC_ERR_UNSUPPORTED;  // 16-byte words throughout (storj's 7408-byte blocks qualify)
    const unsigned g = (unsigned)((nseg + 255) / 256);
    if (open) {
        gcm_status_init<<<g, 256, 0, st>>>(status, (uint32_t)nseg);
        if (hipGetLastError() != hipSuccess) return EC_ERR_DEVICE;
    }
    int rc = gcm_fail(gcm_launch(b, open, st));
    if (rc == EC_OK && open) {
        gcm_status_fini<<<g, 256, 0, st>>>(status, (uint32_t)nseg);
        rc = gcm_fail(hipGetLastError());
    }
    return rc;
}

}  // namespace
}  // namespace uplink_ec

using namespace uplink_ec;

extern "C" {

size_t ec_gcm_key_bytes(void) { return sizeof(GcmSched); }

int ec_gcm_prepare_keys(const uint8_t *keys, size_t nkeys, void *dev_keys, ec_stream stream) {
    if (nkeys == 0) return EC_OK;
    if (!keys || !dev_keys) return EC_ERR_INVALID_ARG;
    // pageable staging (a pinned allocation per call costs more than the 16 KB copy)
    std::vector<GcmSched> host(nkeys);
    for (size_t i = 0; i < nkeys; i++) gcm_prepare(keys + 32 * i, &host[i]);
    hipStream_t st = (hipStream_t)stream;
    int rc = hipMemcpyAsync(dev_keys, host.data(), nkeys * sizeof(GcmSched), hipMemcpyHostToDevice, st) == hipSuccess
                 ? EC_OK
                 : EC_ERR_DEVICE;
    if (hipStreamSynchronize(st) != hipSuccess) rc = EC_ERR_DEVICE;  // before the staging buffer goes
    return rc;
}

int ec_gcm_seal_segments(const uint8_t *plain, size_t nseg, size_t nblocks, size_t in_block, const void *dev_keys,
                         const uint8_t *dev_nonces, uint8_t *out, ec_stream stream) {
    return gcm_run(plain, nseg, nblocks, in_block, dev_keys, dev_nonces, out, nullptr, false, (hipStream_t)stream);
}

int ec_gcm_seal_segments_strided(const uint8_t *plain, long long plain_seg_stride, size_t nseg, size_t nblocks,
                                 size_t in_block, const void *dev_keys, const uint8_t *dev_nonces, uint8_t *out,
                                 long long out_seg_stride, ec_stream stream) {
    return gcm_run(plain, nseg, nblocks, in_block, dev_keys, dev_nonces, out, nullptr, false, (hipStream_t)stream,
                   plain_seg_stride, out_seg_stride);
}

int ec_gcm_open_segments_strided(const uint8_t *cipher, long long cipher_seg_stride, size_t nseg, size_t nblocks,
                                 size_t in_block, const void *dev_keys, const uint8_t *dev_nonces, uint8_t *out,
                                 long long out_seg_stride, int32_t *dev_status, ec_stream stream) {
    return gcm_run(cipher, nseg, nblocks, in_block, dev_keys, dev_nonces, out, dev_status, true, (hipStream_t)stream,
                   cipher_seg_stride, out_seg_stride);
}

int ec_gcm_open_segments(const uint8_t *cipher, size_t nseg, size_t nblocks, size_t in_block, const void *dev_keys,
                         const uint8_t *dev_nonces, uint8_t *out, int32_t *dev_status, ec_stream stream) {
    return gcm_run(cipher, nseg, nblocks, in_block, dev_keys, dev_nonces, out, dev_status, true, (hipStream_t)stream);
}

static int gcm_host(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *in, size_t nblocks,
                    size_t in_block, uint8_t *out, long long *bad_block, bool open) {
    if (!key || !nonce || (nblocks && (!in || !out))) return EC_ERR_INVALID_ARG;
    if (bad_block) *bad_block = -1;
    if (nblocks == 0) return EC_OK;
    const size_t ob = in_block + 16;
    const size_t in_bytes = nblocks * (open ? ob : in_block), out_bytes = nblocks * (open ? in_block : ob);
    hipStream_t st = nullptr;
    uint8_t *d = nullptr;
    int rc = EC_OK;
    const size_t a_in = (in_bytes + 255) & ~(size_t)255, a_out = (out_bytes + 255) & ~(size_t)255;
    do {
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { rc = EC_ERR_DEVICE; st = nullptr; break; }
        if (hipMalloc(&d, a_in + a_out + sizeof(GcmSched) + 256) != hipSuccess) { rc = EC_ERR_DEVICE; d = nullptr; break; }
        uint8_t *d_in = d, *d_out = d + a_in, *d_key = d_out + a_out, *d_misc = d_key + sizeof(GcmSched);
        rc = ec_gcm_prepare_keys(key, 1, d_key, st);
        if (rc) break;
        if (hipMemcpyAsync(d_misc, nonce, 12, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(d_in, in, in_bytes, hipMemcpyHostToDevice, st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        int32_t *d_status = reinterpret_cast<int32_t *>(d_misc + 16);
        rc = gcm_run(d_in, 1, nblocks, in_block, d_key, d_misc, d_out, d_status, open, st);
        if (rc) break;
        int32_t status = -1;
        if (hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
            (open && hipMemcpyAsync(&status, d_status, 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess) { rc = EC_ERR_DEVICE; break; }
        if (open && status >= 0) {
            if (bad_block) *bad_block = status;
            rc = EC_ERR_AUTH;
        }
    } while (0);
    if (st) (void)hipStreamSynchronize(st);
    if (d) (void)hipFree(d);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}

int ec_pad_segments(uint8_t *segs, size_t nseg, long long seg_stride, size_t data_len, size_t block, ec_stream stream) {
    if (nseg == 0) return EC_OK;
    if (!segs || block == 0 || nseg > 65535) return EC_ERR_INVALID_ARG;
    const uint64_t p = 4 + (block - (data_len + 4) % block) % block;
    if ((long long)(data_len + p) > seg_stride && nseg > 1) return EC_ERR_INVALID_ARG;
    pad_segments<<<dim3((unsigned)((p + 255) / 256), (unsigned)nseg), 256, 0, (hipStream_t)stream>>>(
        segs, seg_stride, data_len, (uint32_t)p);
    return gcm_fail(hipGetLastError());
}

int ec_gcm_seal_host(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *plain, size_t nblocks,
                     size_t in_block, uint8_t *out) {
    return gcm_host(key, nonce, plain, nblocks, in_block, out, nullptr, false);
}

int ec_gcm_open_host(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *cipher, size_t nblocks,
                     size_t in_block, uint8_t *out, long long *bad_block) {
    return gcm_host(key, nonce, cipher, nblocks, in_block, out, bad_block, true);
}

}  // extern "C"
