/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Nothing in the product path
 * (uplink_amd/, include/) may link, load or call this file.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as
 * the checker / the reported CPU baseline.
 *
 * CPU restatement of the Reed-Solomon arithmetic that storj/uplink's
 * private/eestream path delegates to `storj.io/infectious v0.0.2`
 * (go.mod:17, go.sum:104-105).  That module is NOT vendored in the reference
 * tree and is absent from this container, so this file restates its published
 * algorithm (a Go port of Rizzo/zfec) from the description in SURVEY.md
 * Appendix A.  Each function names the eestream call site it serves:
 *
 *   or_new_fec          <- eestream.NewFEC            private/eestream/fec.go:15-17
 *                          (callers encode.go:69-87)
 *   or_encode_single    <- rsScheme.EncodeSingle      private/eestream/rs.go:21-23
 *                          (driven by segmentupload/encode.go:39-75, encode.go:173-202)
 *   or_encode           <- rsScheme.Encode            private/eestream/rs.go:25-30
 *   or_rebuild          <- rsScheme.Rebuild           private/eestream/rs.go:40-45
 *                          (driven by stripe.go:382-428)
 *   or_decode           <- rsScheme.Decode            private/eestream/rs.go:32-38
 *                          (Correct + Rebuild; layout as unsafe_rs.go:32-52)
 *
 * Parity pinning: the reference's own tests pin round trips, piece sizes and
 * two error strings (rs_test.go, segmentupload/encode_test.go:53,63) but no
 * parity byte, and no Go toolchain / infectious copy exists here to run.  The
 * generator matrix is therefore built two independent ways here (the zfec
 * inverted-Vandermonde construction and the closed-form Lagrange basis) and
 * the two must agree, plus the SURVEY Appendix A fingerprints; see
 * tests/test_oracle.py.  Exact parity bytes are therefore "parity unpinned"
 * with respect to an execution of the reference.
 *
 * Reference-shaped CPU baseline helpers (or_baseline_*) reproduce the
 * per-piece, per-stripe EncodeSingle loop of segmentupload/encode.go:39-75 and
 * the per-stripe Rebuild (with a per-stripe k x k inversion) of
 * stripe.go:382-428, using a PSHUFB nibble-table addmul the way infectious
 * does on amd64.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>
#include <immintrin.h>

/* ---------------------------------------------------------------- GF(2^8) */
/* zfec/infectious field: x^8+x^4+x^3+x^2+1 (0x11d), generator alpha = 2. */
static uint8_t gf_exp[510];
static int gf_log[256];
static uint8_t gf_inv[256];
static uint8_t gf_mul_table[256][256];
/* nibble tables for the PSHUFB addmul (infectious amd64 addmul) */
static uint8_t nib_lo[256][16], nib_hi[256][16];
static int gf_ready = 0;
static pthread_once_t gf_once = PTHREAD_ONCE_INIT;

static void gf_init_once(void) {
    int x = 1;
    for (int i = 0; i < 255; i++) {
        gf_exp[i] = (uint8_t)x;
        gf_exp[i + 255] = (uint8_t)x;
        gf_log[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11d;
    }
    gf_log[0] = 255; /* zfec: log(0) = A0 = 255 */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++)
            gf_mul_table[a][b] = (a == 0 || b == 0) ? 0 : gf_exp[gf_log[a] + gf_log[b]];
    gf_inv[0] = 0;
    for (int a = 1; a < 256; a++) gf_inv[a] = gf_exp[255 - gf_log[a]];
    for (int c = 0; c < 256; c++)
        for (int v = 0; v < 16; v++) {
            nib_lo[c][v] = gf_mul_table[c][v];
            nib_hi[c][v] = gf_mul_table[c][v << 4];
        }
    gf_ready = 1;
}
void or_init(void) { pthread_once(&gf_once, gf_init_once); }

uint8_t or_gf_mul(uint8_t a, uint8_t b) { or_init(); return gf_mul_table[a][b]; }
uint8_t or_gf_exp(int i) { or_init(); return gf_exp[i % 255]; }
uint8_t or_gf_inv(uint8_t a) { or_init(); return gf_inv[a]; }

/* ------------------------------------------------------------------ addmul */
/* z[i] ^= c * x[i]  (c == 0 is a no-op), infectious addmul. */
static void addmul_scalar(uint8_t *z, const uint8_t *x, uint8_t c, size_t n) {
    if (c == 0) return;
    const uint8_t *row = gf_mul_table[c];
    for (size_t i = 0; i < n; i++) z[i] ^= row[x[i]];
}

__attribute__((target("avx2")))
static void addmul_avx2(uint8_t *z, const uint8_t *x, uint8_t c, size_t n) {
    if (c == 0) return;
    __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib_lo[c]));
    __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)nib_hi[c]));
    __m256i m = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i v = _mm256_loadu_si256((const __m256i *)(x + i));
        __m256i a = _mm256_shuffle_epi8(lo, _mm256_and_si256(v, m));
        __m256i b = _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi64(v, 4), m));
        __m256i r = _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(z + i)), _mm256_xor_si256(a, b));
        _mm256_storeu_si256((__m256i *)(z + i), r);
    }
    if (i < n) addmul_scalar(z + i, x + i, c, n - i);
}

__attribute__((target("ssse3")))
static void addmul_ssse3(uint8_t *z, const uint8_t *x, uint8_t c, size_t n) {
    if (c == 0) return;
    __m128i lo = _mm_loadu_si128((const __m128i *)nib_lo[c]);
    __m128i hi = _mm_loadu_si128((const __m128i *)nib_hi[c]);
    __m128i m = _mm_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 16 <= n; i += 16) {
        __m128i v = _mm_loadu_si128((const __m128i *)(x + i));
        __m128i a = _mm_shuffle_epi8(lo, _mm_and_si128(v, m));
        __m128i b = _mm_shuffle_epi8(hi, _mm_and_si128(_mm_srli_epi64(v, 4), m));
        _mm_storeu_si128((__m128i *)(z + i), _mm_xor_si128(_mm_loadu_si128((const __m128i *)(z + i)), _mm_xor_si128(a, b)));
    }
    if (i < n) addmul_scalar(z + i, x + i, c, n - i);
}

static int simd_level = -1; /* 0 scalar, 1 ssse3, 2 avx2; or_set_simd overrides */
static void addmul(uint8_t *z, const uint8_t *x, uint8_t c, size_t n) {
    if (simd_level < 0) {
        __builtin_cpu_init();
        simd_level = __builtin_cpu_supports("avx2") ? 2 : (__builtin_cpu_supports("ssse3") ? 1 : 0);
    }
    if (simd_level == 2) addmul_avx2(z, x, c, n);
    else if (simd_level == 1) addmul_ssse3(z, x, c, n);
    else addmul_scalar(z, x, c, n);
}
void or_set_simd(int level) { simd_level = level; }
int or_get_simd(void) { addmul(NULL, NULL, 0, 0); return simd_level; }

/* --------------------------------------------------------- matrix helpers */
/* zfec _invert_mat: Gauss-Jordan inversion over GF(2^8) with row pivoting.
 * Returns 0 on success, -1 for a singular matrix.  Rebuild uses it on the
 * k x k decode matrix (inside infectious.FEC.Rebuild). */
int or_invert_matrix(uint8_t *m, int k) {
    or_init();
    uint8_t *aug = (uint8_t *)calloc((size_t)k * 2 * k, 1);
    for (int r = 0; r < k; r++) {
        memcpy(aug + (size_t)r * 2 * k, m + (size_t)r * k, k);
        aug[(size_t)r * 2 * k + k + r] = 1;
    }
    int w = 2 * k;
    for (int c = 0; c < k; c++) {
        int p = -1;
        for (int r = c; r < k; r++) if (aug[(size_t)r * w + c]) { p = r; break; }
        if (p < 0) { free(aug); return -1; }
        if (p != c)
            for (int j = 0; j < w; j++) {
                uint8_t t = aug[(size_t)p * w + j];
                aug[(size_t)p * w + j] = aug[(size_t)c * w + j];
                aug[(size_t)c * w + j] = t;
            }
        uint8_t iv = gf_inv[aug[(size_t)c * w + c]];
        for (int j = 0; j < w; j++) aug[(size_t)c * w + j] = gf_mul_table[iv][aug[(size_t)c * w + j]];
        for (int r = 0; r < k; r++) {
            if (r == c) continue;
            uint8_t f = aug[(size_t)r * w + c];
            if (!f) continue;
            for (int j = 0; j < w; j++) aug[(size_t)r * w + j] ^= gf_mul_table[f][aug[(size_t)c * w + j]];
        }
    }
    for (int r = 0; r < k; r++) memcpy(m + (size_t)r * k, aug + (size_t)r * w + k, k);
    free(aug);
    return 0;
}

/* ------------------------------------------------------------------ NewFEC */
/* infectious NewFEC (zfec fec_new), SURVEY.md Appendix A item 2:
 *   temp rows 0..k-1  = inverse of the k x k Vandermonde on points
 *                       {0, a^1, ..., a^(k-1)}   (createInvertedVdm)
 *   temp rows r >= k  = [a^(r*c)]_c              (point a^r)
 *   enc rows r >= k   = temp_row_r * inverse     (systematic parity rows)
 *   enc rows 0..k-1   = identity
 * vand_matrix (k x n, used by Correct's syndrome matrix) has column j =
 * [x_j^0 .. x_j^(k-1)] with x_0 = 0, x_j = a^(j-1).
 * Errors: "requires 1 <= k <= n <= 256" (returned as -1). */
int or_new_fec(int k, int n, uint8_t *enc_matrix, uint8_t *vand_matrix) {
    or_init();
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return -1;
    /* top: Vandermonde V_top[r][c] = x_r^c, x_0 = 0, x_r = a^r; invert it */
    uint8_t *vtop = (uint8_t *)calloc((size_t)k * k, 1);
    for (int r = 0; r < k; r++)
        for (int c = 0; c < k; c++) {
            if (r == 0) vtop[c] = (c == 0) ? 1 : 0;
            else vtop[(size_t)r * k + c] = gf_exp[(r * c) % 255];
        }
    if (or_invert_matrix(vtop, k) != 0) { free(vtop); return -2; }
    memset(enc_matrix, 0, (size_t)n * k);
    for (int i = 0; i < k; i++) enc_matrix[(size_t)i * k + i] = 1;
    for (int r = k; r < n; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++)
                acc ^= gf_mul_table[gf_exp[(r * i) % 255]][vtop[(size_t)i * k + c]];
            enc_matrix[(size_t)r * k + c] = acc;
        }
    free(vtop);
    if (vand_matrix) {
        memset(vand_matrix, 0, (size_t)k * n);
        vand_matrix[0] = 1;
        uint8_t g = 1;
        for (int row = 0; row < k; row++) {
            uint8_t a = 1;
            for (int col = 1; col < n; col++) {
                vand_matrix[(size_t)row * n + col] = a;
                a = gf_mul_table[g][a];
            }
            g = gf_mul_table[2][g];
        }
    }
    return 0;
}

/* Closed-form cross-check: G[i][j] = L_j(x_i) over points x_0 = 0,
 * x_r = a^(r-1) (zfec indexing).  Independent of or_new_fec's inversion. */
int or_lagrange_fec(int k, int n, uint8_t *enc_matrix) {
    or_init();
    if (k <= 0 || n <= 0 || k > 256 || n > 256 || k > n) return -1;
    uint8_t xs[256];
    xs[0] = 0;
    for (int r = 1; r < n; r++) xs[r] = gf_exp[(r - 1) % 255];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < k; j++) {
            uint8_t num = 1, den = 1;
            for (int m = 0; m < k; m++) {
                if (m == j) continue;
                num = gf_mul_table[num][xs[i] ^ xs[m]];
                den = gf_mul_table[den][xs[j] ^ xs[m]];
            }
            enc_matrix[(size_t)i * k + j] = gf_mul_table[num][gf_inv[den]];
        }
    return 0;
}

/* ----------------------------------------------------------- EncodeSingle */
/* error codes mirror infectious' messages:
 *  -1 "num must be non-negative"     (pinned segmentupload/encode_test.go:53)
 *  -2 "num must be less than %d"     (pinned segmentupload/encode_test.go:63)
 *  -3 "input length must be a multiple of %d"
 *  -4 "output length must be %d"                                          */
int or_encode_single(int k, int n, const uint8_t *enc, const uint8_t *in, size_t in_len,
                     uint8_t *out, size_t out_len, int num) {
    or_init();
    if (num < 0) return -1;
    if (num >= n) return -2;
    if (in_len % (size_t)k) return -3;
    size_t bs = in_len / (size_t)k;
    if (out_len != bs) return -4;
    if (num < k) { memcpy(out, in + (size_t)num * bs, bs); return 0; }
    memset(out, 0, bs);
    for (int i = 0; i < k; i++) addmul(out, in + (size_t)i * bs, enc[(size_t)num * k + i], bs);
    return 0;
}

/* Encode: all n shares of `in`, share i written to out + i*bs. */
int or_encode(int k, int n, const uint8_t *enc, const uint8_t *in, size_t in_len, uint8_t *out) {
    or_init();
    if (in_len % (size_t)k) return -3;
    size_t bs = in_len / (size_t)k;
    for (int i = 0; i < n; i++) {
        int r = or_encode_single(k, n, enc, in, in_len, out + (size_t)i * bs, bs, i);
        if (r) return r;
    }
    return 0;
}

/* ----------------------------------------------------------------- Rebuild */
/* infectious FEC.Rebuild:
 *  - fewer than k shares -> NotEnoughShares (-10)
 *  - shares sorted by Number in place (numbers[] and data[] are permuted)
 *  - for i in 0..k-1: take the front share if its Number == i, else take from
 *    the back of the sorted list
 *  - Number >= n -> "invalid share id" (-11)
 *  - present data shares pass through, missing data shares are rebuilt via
 *    the inverse of the chosen rows of enc_matrix (singular -> -12)
 * Output: the k data shares, share i at out + i*len (the layout of
 * unsafeRSScheme.Decode, unsafe_rs.go:38-46, and of the copy in
 * stripe.go:410-412). */
static void sort_shares(int ns, int *numbers, const uint8_t **data) {
    for (int a = 1; a < ns; a++) {           /* stable insertion sort */
        int kn = numbers[a]; const uint8_t *kd = data[a]; int b = a - 1;
        while (b >= 0 && numbers[b] > kn) { numbers[b + 1] = numbers[b]; data[b + 1] = data[b]; b--; }
        numbers[b + 1] = kn; data[b + 1] = kd;
    }
}

int or_rebuild(int k, int n, const uint8_t *enc, int ns, int *numbers, const uint8_t **data,
               size_t len, uint8_t *out) {
    or_init();
    if (ns < k) return -10;
    sort_shares(ns, numbers, data);
    uint8_t *m = (uint8_t *)calloc((size_t)k * k, 1);
    int *idx = (int *)malloc(sizeof(int) * k);
    const uint8_t **sv = (const uint8_t **)malloc(sizeof(void *) * k);
    int b = 0, e = ns - 1;
    for (int i = 0; i < k; i++) {
        int id; const uint8_t *d;
        if (numbers[b] == i) { id = numbers[b]; d = data[b]; b++; }
        else { id = numbers[e]; d = data[e]; e--; }
        if (id >= n || id < 0) { free(m); free(idx); free(sv); return -11; }
        if (id < k) {
            m[(size_t)i * (k + 1)] = 1;
            memcpy(out + (size_t)id * len, d, len);
        } else {
            memcpy(m + (size_t)i * k, enc + (size_t)id * k, k);
        }
        sv[i] = d; idx[i] = id;
    }
    if (or_invert_matrix(m, k) != 0) { free(m); free(idx); free(sv); return -12; }
    for (int i = 0; i < k; i++) {
        if (idx[i] >= k) {
            uint8_t *dst = out + (size_t)i * len;
            memset(dst, 0, len);
            for (int c = 0; c < k; c++) addmul(dst, sv[c], m[(size_t)i * k + c], len);
        }
    }
    free(m); free(idx); free(sv);
    return 0;
}

/* -------------------------------------------------- Correct (Berlekamp-Welch) */
/* infectious FEC.Correct/Decode.  A byte column is
 * checked against the code (the syndrome test is equivalent to "the received
 * values are one codeword"); a column that is not a codeword is corrected by
 * Berlekamp-Welch on the points x_0 = 0, x_r = a^(r-1) with e = (r-k)/2:
 * e <= 0 -> NotEnoughShares (-10); a non-zero remainder -> TooManyErrors (-13).
 * PARITY NOTE: infectious' own linear solver is not available here; this
 * restatement solves the BW system by Gauss-Jordan with free variables set to
 * zero, which returns the unique decoding whenever one exists.  Columns with
 * more than e errors are "parity unpinned" (documented in DESIGN.md). */
static int poly_eval_pts(const uint8_t *coef, int deg, uint8_t x) { /* coef[0] = const */
    uint8_t acc = 0;
    for (int i = deg; i >= 0; i--) acc = gf_mul_table[acc][x] ^ coef[i];
    return acc;
}

static uint8_t gf_pow(uint8_t x, int e) {
    uint8_t r = 1;
    for (int i = 0; i < e; i++) r = gf_mul_table[r][x];
    return r;
}

/* solve A (dim x dim) u = f ; returns 0 ok (free vars = 0), -1 inconsistent */
static int solve_system(uint8_t *A, uint8_t *f, int dim, uint8_t *u) {
    int row = 0;
    int *pivcol = (int *)malloc(sizeof(int) * dim);
    for (int c = 0; c < dim && row < dim; c++) {
        int p = -1;
        for (int r = row; r < dim; r++) if (A[r * dim + c]) { p = r; break; }
        if (p < 0) continue;
        if (p != row) {
            for (int j = 0; j < dim; j++) { uint8_t t = A[p * dim + j]; A[p * dim + j] = A[row * dim + j]; A[row * dim + j] = t; }
            uint8_t t = f[p]; f[p] = f[row]; f[row] = t;
        }
        uint8_t iv = gf_inv[A[row * dim + c]];
        for (int j = 0; j < dim; j++) A[row * dim + j] = gf_mul_table[iv][A[row * dim + j]];
        f[row] = gf_mul_table[iv][f[row]];
        for (int r = 0; r < dim; r++) {
            if (r == row || !A[r * dim + c]) continue;
            uint8_t fac = A[r * dim + c];
            for (int j = 0; j < dim; j++) A[r * dim + j] ^= gf_mul_table[fac][A[row * dim + j]];
            f[r] ^= gf_mul_table[fac][f[row]];
        }
        pivcol[row] = c;
        row++;
    }
    for (int r = row; r < dim; r++) if (f[r]) { free(pivcol); return -1; }
    memset(u, 0, dim);
    for (int r = 0; r < row; r++) u[pivcol[r]] = f[r];
    free(pivcol);
    return 0;
}

/* Berlekamp-Welch on one byte column: vals[i] at share numbers nums[i]
 * (r values).  On success writes the corrected codeword value for every
 * share number 0..n-1 into out_cw. */
static int bw_column(int k, int n, int r, const int *nums, const uint8_t *vals, uint8_t *out_cw) {
    int e = (r - k) / 2;
    if (e <= 0) return -10;
    int q = e + k;               /* Q has q coefficients (deg < q) */
    int dim = q + e;             /* unknowns: Q (q) and E's low e coeffs */
    if (dim > r) dim = r;        /* use the first dim equations (r >= dim by construction) */
    uint8_t *A = (uint8_t *)calloc((size_t)dim * dim, 1);
    uint8_t *f = (uint8_t *)calloc(dim, 1);
    uint8_t *u = (uint8_t *)calloc(dim, 1);
    for (int i = 0; i < dim; i++) {
        uint8_t x = nums[i] == 0 ? 0 : gf_exp[(nums[i] - 1) % 255];
        uint8_t ri = vals[i];
        f[i] = gf_mul_table[gf_pow(x, e)][ri];
        for (int j = 0; j < q; j++) A[i * dim + j] = gf_pow(x, j);
        for (int t = 0; t < e; t++) A[i * dim + q + t] = gf_mul_table[gf_pow(x, t)][ri];
    }
    /* Q(x) - E'(x) r = x^e r   where E = x^e + E' */
    int rc = solve_system(A, f, dim, u);
    if (rc) { free(A); free(f); free(u); return -13; }
    uint8_t Q[512], E[512];
    memset(Q, 0, sizeof Q); memset(E, 0, sizeof E);
    for (int j = 0; j < q; j++) Q[j] = u[j];
    for (int t = 0; t < e; t++) E[t] = u[q + t];
    E[e] = 1;
    /* polynomial long division Q / E (E monic) */
    uint8_t rem[512]; memcpy(rem, Q, sizeof rem);
    uint8_t P[512]; memset(P, 0, sizeof P);
    for (int d = q - 1; d >= e; d--) {
        uint8_t co = rem[d];
        if (!co) continue;
        P[d - e] = co;
        for (int t = 0; t <= e; t++) rem[d - e + t] ^= gf_mul_table[co][E[t]];
    }
    for (int d = 0; d < e; d++) if (rem[d]) { free(A); free(f); free(u); return -13; }
    for (int i = 0; i < n; i++) {
        uint8_t x = i == 0 ? 0 : gf_exp[(i - 1) % 255];
        out_cw[i] = (uint8_t)poly_eval_pts(P, k - 1, x);
    }
    free(A); free(f); free(u);
    return 0;
}

/* Correct: shares sorted in place; data[] buffers are modified in place (the
 * caller passes writable buffers: infectious corrects share.Data in place). */
int or_correct(int k, int n, const uint8_t *enc, int ns, int *numbers, uint8_t **data, size_t len) {
    or_init();
    if (ns < k) return -10;
    sort_shares(ns, numbers, (const uint8_t **)data);
    if (ns == k) return 0;  /* no redundancy: every column is trivially a codeword */
    /* codeword test per column: re-encode from the first k shares (rebuild)
     * and compare the remaining ones */
    uint8_t *vals = (uint8_t *)malloc(ns);
    uint8_t *cw = (uint8_t *)malloc(n);
    int *nums = (int *)malloc(sizeof(int) * ns);
    uint8_t *dm = (uint8_t *)calloc((size_t)k * k, 1);
    /* interpolation matrix from the first k shares to all n points:
     * all shares are evaluations of one degree<k polynomial at x_num.  Build
     * W = G_rows(first k)^-1 and R = G * W so cw = R * vals[0..k) */
    for (int i = 0; i < k; i++) memcpy(dm + (size_t)i * k, enc + (size_t)numbers[i] * k, k);
    if (or_invert_matrix(dm, k) != 0) { free(vals); free(cw); free(nums); free(dm); return -12; }
    for (int i = 0; i < ns; i++) nums[i] = numbers[i];
    int rc = 0;
    for (size_t col = 0; col < len && rc == 0; col++) {
        for (int i = 0; i < ns; i++) vals[i] = data[i][col];
        /* data vector d = dm * vals[0..k) ; check shares k..ns-1 */
        int ok = 1;
        uint8_t dvec[256];
        for (int a = 0; a < k; a++) {
            uint8_t acc = 0;
            for (int c = 0; c < k; c++) acc ^= gf_mul_table[dm[(size_t)a * k + c]][vals[c]];
            dvec[a] = acc;
        }
        for (int i = k; i < ns && ok; i++) {
            uint8_t acc = 0;
            for (int c = 0; c < k; c++) acc ^= gf_mul_table[enc[(size_t)nums[i] * k + c]][dvec[c]];
            if (acc != vals[i]) ok = 0;
        }
        if (ok) continue;
        rc = bw_column(k, n, ns, nums, vals, cw);
        if (rc == 0)
            for (int i = 0; i < ns; i++) data[i][col] = cw[nums[i]];
    }
    free(vals); free(cw); free(nums); free(dm);
    return rc;
}

/* Decode = Correct + Rebuild into out (k*len), rsScheme.Decode rs.go:32-38 */
int or_decode(int k, int n, const uint8_t *enc, int ns, int *numbers, uint8_t **data, size_t len, uint8_t *out) {
    int rc = or_correct(k, n, enc, ns, numbers, data, len);
    if (rc) return rc;
    if (ns == 0) return -14;
    return or_rebuild(k, n, enc, ns, numbers, (const uint8_t **)data, len, out);
}

/* Decode as infectious runs it over whole share buffers (FEC.Correct: one
 * syndrome row per share beyond k, accumulated with addmul over the whole
 * buffer, Berlekamp-Welch only on the columns where a syndrome is non-zero;
 * then Rebuild).  Same results as or_decode, whose per-column check is the
 * plain restatement; this one is the CPU baseline of the reference benchmark's
 * Decode (rs_test.go:616-631), not a checker of anything.
 * Syndrome rows: with B the first k sorted shares and R the rest,
 * H = [G_R G_B^-1 | I] annihilates every codeword restricted to B u R. */
int or_decode_fast(int k, int n, const uint8_t *enc, int ns, int *numbers, uint8_t **data, size_t len, uint8_t *out) {
    or_init();
    if (ns < k) return -10;
    sort_shares(ns, numbers, (const uint8_t **)data);
    if (ns > k) {
        uint8_t *gb = (uint8_t *)calloc((size_t)k * k, 1);
        for (int i = 0; i < k; i++) memcpy(gb + (size_t)i * k, enc + (size_t)numbers[i] * k, k);
        if (or_invert_matrix(gb, k) != 0) { free(gb); return -12; }
        uint8_t *syn = (uint8_t *)malloc(len), *h = (uint8_t *)malloc(k), *cw = (uint8_t *)malloc(n),
                *vals = (uint8_t *)malloc(ns);
        int rc = 0;
        for (int r = k; r < ns && rc == 0; r++) {
            for (int b = 0; b < k; b++) {  /* h = G_r G_B^-1 */
                uint8_t acc = 0;
                for (int c = 0; c < k; c++) acc ^= gf_mul_table[enc[(size_t)numbers[r] * k + c]][gb[(size_t)c * k + b]];
                h[b] = acc;
            }
            memcpy(syn, data[r], len);
            for (int b = 0; b < k; b++) addmul(syn, data[b], h[b], len);
            for (size_t col = 0; col < len && rc == 0; col++) {
                if (!syn[col]) continue;
                for (int i = 0; i < ns; i++) vals[i] = data[i][col];
                rc = bw_column(k, n, ns, numbers, vals, cw);
                if (rc == 0) {
                    for (int i = 0; i < ns; i++) data[i][col] = cw[numbers[i]];
                    /* later syndrome rows see the corrected column */
                }
            }
        }
        free(gb); free(syn); free(h); free(cw); free(vals);
        if (rc) return rc;
    }
    return or_rebuild(k, n, enc, ns, numbers, (const uint8_t **)data, len, out);
}

/* ------------------------------------------------ reference-shaped baseline */
/* Segment layout [stripe][k][ess]; pieces [n][nstripes*ess].
 * Per piece, per stripe EncodeSingle (segmentupload/encode.go:39-75): the
 * exact per-call work infectious does (zero + k addmuls for a parity share,
 * a copy for a data share).  Work is split over `threads` pthreads by piece
 * number, as uplink runs one goroutine per piece (single.go:149-210). */
typedef struct {
    int k, n, ess; const uint8_t *enc; const uint8_t *seg; size_t nstripes;
    uint8_t *pieces; int p0, p1;
} enc_job;

static void *enc_worker(void *arg) {
    enc_job *j = (enc_job *)arg;
    size_t stripe = (size_t)j->k * j->ess, plen = j->nstripes * j->ess;
    for (int num = j->p0; num < j->p1; num++)
        for (size_t s = 0; s < j->nstripes; s++)
            or_encode_single(j->k, j->n, j->enc, j->seg + s * stripe, stripe,
                             j->pieces + (size_t)num * plen + s * j->ess, j->ess, num);
    return NULL;
}

int or_baseline_encode_segment(int k, int n, int ess, const uint8_t *enc, const uint8_t *seg,
                               size_t nstripes, uint8_t *pieces, int threads) {
    or_init();
    if (threads < 1) threads = 1;
    if (threads > n) threads = n;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    enc_job *jobs = (enc_job *)malloc(sizeof(enc_job) * threads);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (enc_job){k, n, ess, enc, seg, nstripes, pieces, n * t / threads, n * (t + 1) / threads};
        pthread_create(&th[t], NULL, enc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

/* Per-stripe Rebuild (stripe.go:382-428): every stripe re-sorts, re-inverts
 * and rebuilds, writing stripe-major output [stripe][k][ess].  Threads split
 * the stripe range (many concurrent downloads in uplink). */
typedef struct {
    int k, n, ess; const uint8_t *enc; int ns; const int *nums; const uint8_t *const *pieces;
    uint8_t *out; size_t s0, s1; int rc;
} dec_job;

static void *dec_worker(void *arg) {
    dec_job *j = (dec_job *)arg;
    int nums[256]; const uint8_t *ptr[256];
    size_t stripe = (size_t)j->k * j->ess;
    for (size_t s = j->s0; s < j->s1; s++) {
        for (int i = 0; i < j->ns; i++) { nums[i] = j->nums[i]; ptr[i] = j->pieces[i] + s * j->ess; }
        int rc = or_rebuild(j->k, j->n, j->enc, j->ns, nums, ptr, j->ess, j->out + s * stripe);
        if (rc) { j->rc = rc; return NULL; }
    }
    return NULL;
}

int or_baseline_rebuild_segment(int k, int n, int ess, const uint8_t *enc, int ns, const int *nums,
                                const uint8_t *const *pieces, size_t nstripes, uint8_t *out, int threads) {
    or_init();
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    dec_job *jobs = (dec_job *)malloc(sizeof(dec_job) * threads);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (dec_job){k, n, ess, enc, ns, nums, pieces, out,
                            nstripes * t / threads, nstripes * (t + 1) / threads, 0};
        pthread_create(&th[t], NULL, dec_worker, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
    free(th); free(jobs);
    return rc;
}

/* The optimised CPU variant of the same two loops (SURVEY §8d "all rows per
 * stripe"), reported next to the reference-shaped baseline: threads split the
 * stripes; each thread walks blocks of 32 stripes (~230 KB of input, L2-resident)
 * and produces every piece's share of them, so each input byte is read from
 * memory once instead of once per piece; the rebuild inverts once per share
 * set instead of once per stripe.  Same results as the reference-shaped
 * loops (tests/test_oracle.py). */
typedef struct {
    int k, n, ess; const uint8_t *enc; const uint8_t *seg; size_t nstripes; uint8_t *pieces;
    size_t s0, s1;
    const uint8_t *dmat; const int *ids; const uint8_t *const *src; uint8_t *out;  /* rebuild */
} fast_job;

static void *fast_enc_worker(void *arg) {
    fast_job *j = (fast_job *)arg;
    const size_t stripe = (size_t)j->k * j->ess, plen = j->nstripes * j->ess, blk = 32;
    for (size_t b0 = j->s0; b0 < j->s1; b0 += blk) {
        const size_t b1 = b0 + blk < j->s1 ? b0 + blk : j->s1;
        for (int num = 0; num < j->n; num++) {
            for (size_t s = b0; s < b1; s++) {
                const uint8_t *in = j->seg + s * stripe;
                uint8_t *o = j->pieces + (size_t)num * plen + s * j->ess;
                if (num < j->k) { memcpy(o, in + (size_t)num * j->ess, j->ess); continue; }
                memset(o, 0, j->ess);
                for (int i = 0; i < j->k; i++) addmul(o, in + (size_t)i * j->ess, j->enc[(size_t)num * j->k + i], j->ess);
            }
        }
    }
    return NULL;
}

int or_fast_encode_segment(int k, int n, int ess, const uint8_t *enc, const uint8_t *seg, size_t nstripes,
                           uint8_t *pieces, int threads) {
    or_init();
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    fast_job *jobs = (fast_job *)calloc(threads, sizeof(fast_job));
    for (int t = 0; t < threads; t++) {
        jobs[t] = (fast_job){k, n, ess, enc, seg, nstripes, pieces, nstripes * t / threads, nstripes * (t + 1) / threads,
                             NULL, NULL, NULL, NULL};
        pthread_create(&th[t], NULL, fast_enc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs);
    return 0;
}

static void *fast_dec_worker(void *arg) {
    fast_job *j = (fast_job *)arg;
    const size_t stripe = (size_t)j->k * j->ess;
    for (size_t s = j->s0; s < j->s1; s++) {
        uint8_t *o = j->out + s * stripe;
        for (int i = 0; i < j->k; i++) {
            uint8_t *dst = o + (size_t)i * j->ess;
            if (j->ids[i] < j->k) { memcpy(o + (size_t)j->ids[i] * j->ess, j->src[i] + s * j->ess, j->ess); continue; }
            memset(dst, 0, j->ess);
            for (int c = 0; c < j->k; c++) addmul(dst, j->src[c] + s * j->ess, j->dmat[(size_t)i * j->k + c], j->ess);
        }
    }
    return NULL;
}

/* Rebuild from exactly k pieces (numbers `nums`, any order): one share choice
 * and one inversion, then every stripe. */
int or_fast_rebuild_segment(int k, int n, int ess, const uint8_t *enc, const int *nums, const uint8_t *const *pieces,
                            size_t nstripes, uint8_t *out, int threads) {
    or_init();
    int numbers[256]; const uint8_t *data[256]; int ids[256]; const uint8_t *src[256];
    for (int i = 0; i < k; i++) { numbers[i] = nums[i]; data[i] = pieces[i]; }
    sort_shares(k, numbers, data);
    uint8_t *m = (uint8_t *)calloc((size_t)k * k, 1);
    int b = 0, e = k - 1;
    for (int i = 0; i < k; i++) {
        if (numbers[b] == i) { ids[i] = numbers[b]; src[i] = data[b]; b++; }
        else { ids[i] = numbers[e]; src[i] = data[e]; e--; }
        if (ids[i] >= n || ids[i] < 0) { free(m); return -11; }
        if (ids[i] < k) m[(size_t)i * (k + 1)] = 1;
        else memcpy(m + (size_t)i * k, enc + (size_t)ids[i] * k, k);
    }
    if (or_invert_matrix(m, k) != 0) { free(m); return -12; }
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    fast_job *jobs = (fast_job *)calloc(threads, sizeof(fast_job));
    for (int t = 0; t < threads; t++) {
        jobs[t] = (fast_job){k, n, ess, enc, NULL, nstripes, NULL, nstripes * t / threads, nstripes * (t + 1) / threads,
                             m, ids, src, out};
        pthread_create(&th[t], NULL, fast_dec_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th); free(jobs); free(m);
    return 0;
}

/* ------------------------------------------------------------- padding */
/* storj.io/common encryption.PadReader: p = 4 +
 * (bs - (len+4) % bs) % bs pad bytes, every pad byte = byte(p), the last 4
 * bytes big-endian uint32(p).  Returns the padded length; writes the pad
 * after `len` bytes of buf (buf must hold the padded length). */
size_t or_pad(uint8_t *buf, size_t len, size_t bs) {
    size_t p = 4 + (bs - (len + 4) % bs) % bs;
    for (size_t i = 0; i < p; i++) buf[len + i] = (uint8_t)p;
    uint32_t pv = (uint32_t)p;
    buf[len + p - 4] = (uint8_t)(pv >> 24);
    buf[len + p - 3] = (uint8_t)(pv >> 16);
    buf[len + p - 2] = (uint8_t)(pv >> 8);
    buf[len + p - 1] = (uint8_t)pv;
    return len + p;
}
