/* C-ABI test from plain C -- the view a cgo binding has of the engine
 * (INTEGRATION.md §2): include/uplink_ec.h + libuplink_ec.so, host buffers,
 * no Python or torch in the process.  Checks every ErasureScheme export and
 * the host-memory batch pipeline against the CPU oracle (test
 * infrastructure: oracle/infectious_oracle.c), plus the pinned error codes
 * and strings, and the BLAKE3 / AES-256-GCM entry points against
 * oracle/blake3_oracle.c and oracle/aesgcm_oracle.c.  Built by `make -C tests/c`, run by tests/test_c_abi.py on a
 * GPU box.  Exit status 0 = all checks passed. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uplink_ec.h"

/* oracle (CPU restatement of storj.io/infectious) */
int or_new_fec(int k, int n, uint8_t *enc_matrix, uint8_t *vand_matrix);
int or_encode(int k, int n, const uint8_t *enc, const uint8_t *in, size_t in_len, uint8_t *out);
int or_decode(int k, int n, const uint8_t *enc, int ns, int *numbers, uint8_t **data, size_t len, uint8_t *out);
int or_baseline_encode_segment(int k, int n, int ess, const uint8_t *enc, const uint8_t *seg, size_t stripes,
                               uint8_t *pieces, int threads);

/* oracles of the adjacent stages */
void b3_hash(const uint8_t *in, size_t len, uint8_t out[32]);
int64_t ag_encrypt_blocks(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *plain, size_t nblocks,
                          size_t in_block, uint8_t *out, int threads);

/* milliseconds since the start of main: every progress line is stamped, so a
 * run stopped by a timeout names the phase it was in */
static struct timespec t_start;
static double ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (t.tv_sec - t_start.tv_sec) * 1e3 + (t.tv_nsec - t_start.tv_nsec) * 1e-6;
}

static int failures = 0;
#define CHECK(cond, ...)                                                                                \
    do {                                                                                                \
        if (!(cond)) {                                                                                  \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                                        \
            fprintf(stderr, __VA_ARGS__);                                                               \
            fprintf(stderr, "\n");                                                                      \
            failures++;                                                                                 \
        }                                                                                               \
    } while (0)

static uint64_t rng_state = 0x5EED0000ull;
static uint8_t rnd8(void) {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(rng_state >> 56);
}
static void fill(uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) p[i] = rnd8();
}

/* body: EC_BODY_AUTO (per-stripe calls on the jump table) or
 * EC_BODY_STRAIGHT_LINE (every runtime-matrix launch on generated code) */
static void scheme_surface(int k, int n, int ess, int body) {
    ec_ctx *ctx = NULL;
    int rc = ec_create(k, n, ess, &ctx);
    CHECK(rc == EC_OK, "ec_create(%d,%d,%d) = %d (%s)", k, n, ess, rc, ec_strerror(rc));
    if (rc) return;
    CHECK(ec_set_body(ctx, body) == EC_OK, "ec_set_body(%d)", body);
    CHECK(ec_required(ctx) == k && ec_total(ctx) == n && ec_share_size(ctx) == ess &&
              ec_stripe_size(ctx) == k * ess,
          "sizes");
    uint8_t *enc = malloc((size_t)n * k), *vand = malloc((size_t)n * k);
    or_new_fec(k, n, enc, vand);
    uint8_t *g = malloc((size_t)n * k);
    ec_generator(ctx, g);
    CHECK(memcmp(g, enc, (size_t)n * k) == 0, "generator != oracle enc_matrix (%d,%d)", k, n);

    const size_t stripe = (size_t)k * ess;
    uint8_t *in = malloc(stripe), *all = malloc((size_t)n * ess), *ref = malloc((size_t)n * ess);
    uint8_t *one = malloc(ess);
    fill(in, stripe);
    printf("[%9.1f ms]   per-stripe encode\n", ms());
    CHECK(ec_encode(ctx, in, stripe, all) == EC_OK, "ec_encode");
    or_encode(k, n, enc, in, stripe, ref);
    CHECK(memcmp(all, ref, (size_t)n * ess) == 0, "ec_encode != oracle (%d,%d,%d)", k, n, ess);
    for (int num = 0; num < n; num += (n > 8 ? n / 8 : 1)) {
        CHECK(ec_encode_single(ctx, in, stripe, one, ess, num) == EC_OK, "ec_encode_single");
        CHECK(memcmp(one, ref + (size_t)num * ess, ess) == 0, "ec_encode_single num=%d", num);
    }
    /* pinned error strings (segmentupload/encode_test.go:53,63) */
    char msg[128];
    rc = ec_encode_single(ctx, in, stripe, one, ess, -1);
    CHECK(rc == EC_ERR_NUM_NEGATIVE, "num -1 -> %d", rc);
    ec_format_error(ctx, rc, 0, msg, sizeof msg);
    CHECK(strcmp(msg, "num must be non-negative") == 0, "msg '%s'", msg);
    rc = ec_encode_single(ctx, in, stripe, one, ess, n);
    CHECK(rc == EC_ERR_NUM_RANGE, "num n -> %d", rc);
    ec_format_error(ctx, rc, 0, msg, sizeof msg);
    char want[64];
    snprintf(want, sizeof want, "num must be less than %d", n);
    CHECK(strcmp(msg, want) == 0, "msg '%s' want '%s'", msg, want);

    /* Rebuild / Decode from the last k shares (all parity when n >= 2k) */
    printf("[%9.1f ms]   per-stripe rebuild / decode\n", ms());
    int nums[256];
    const uint8_t *shp[256];
    uint8_t *shw[256];
    uint8_t *out = malloc(stripe), *out2 = malloc(stripe);
    for (int i = 0; i < k; i++) {
        nums[i] = n - k + i;
        shp[i] = all + (size_t)(n - k + i) * ess;
    }
    CHECK(ec_rebuild(ctx, k, nums, shp, ess, out) == EC_OK, "ec_rebuild");
    CHECK(memcmp(out, in, stripe) == 0, "ec_rebuild != input (%d,%d,%d)", k, n, ess);
    if (ess % 16 == 0)
        CHECK(ec_last_body(ctx) == (body == EC_BODY_STRAIGHT_LINE ? EC_BODY_STRAIGHT_LINE : EC_BODY_JUMP_TABLE),
              "body of a per-stripe rebuild: %d", ec_last_body(ctx));
    if (n - k >= 2) {
        /* Decode with 2 extra shares, one of them corrupted: Berlekamp-Welch */
        int ns = k + 2;
        for (int i = 0; i < ns; i++) {
            nums[i] = n - ns + i;
            shw[i] = malloc(ess);
            memcpy(shw[i], all + (size_t)(n - ns + i) * ess, ess);
        }
        shw[1][ess / 2] ^= 0x5a;
        uint8_t *cp[256];
        int cn[256];
        for (int i = 0; i < ns; i++) {
            cp[i] = malloc(ess);
            memcpy(cp[i], shw[i], ess);
            cn[i] = nums[i];
        }
        rc = ec_decode(ctx, ns, nums, shw, ess, out);
        CHECK(rc == EC_OK, "ec_decode rc %d", rc);
        CHECK(memcmp(out, in, stripe) == 0, "ec_decode did not correct (%d,%d)", k, n);
        rc = or_decode(k, n, enc, ns, cn, cp, ess, out2);
        CHECK(rc == 0 && memcmp(out2, in, stripe) == 0, "oracle decode");
        for (int i = 0; i < ns; i++) {
            free(shw[i]);
            free(cp[i]);
        }
    }
    /* NotEnoughShares */
    rc = ec_rebuild(ctx, k - 1, nums, shp, ess, out);
    CHECK(rc == EC_ERR_NOT_ENOUGH_SHARES, "k-1 shares -> %d", rc);

    /* host-memory batch pipeline: 3 segments of 5 stripes */
    printf("[%9.1f ms]   host pipeline\n", ms());
    const size_t nseg = 3, stripes = 5, spad = stripes * stripe, plen = stripes * (size_t)ess;
    uint8_t *segs = malloc(nseg * spad), *pieces = malloc(nseg * (size_t)n * plen), *pref = malloc((size_t)n * plen);
    uint8_t *back = malloc(nseg * spad);
    fill(segs, nseg * spad);
    CHECK(ec_encode_segments_host(ctx, segs, nseg, stripes, pieces, 0) == EC_OK, "ec_encode_segments_host");
    for (size_t s = 0; s < nseg; s++) {
        or_baseline_encode_segment(k, n, ess, enc, segs + s * spad, stripes, pref, 1);
        CHECK(memcmp(pieces + s * (size_t)n * plen, pref, (size_t)n * plen) == 0, "segment %zu pieces", s);
    }
    const uint8_t *pp[256];
    for (int i = 0; i < k; i++) {
        nums[i] = n - 1 - i; /* any order */
        pp[i] = pieces + (size_t)(n - 1 - i) * plen;
    }
    CHECK(ec_rebuild_segments_host(ctx, k, nums, pp, stripes, nseg, (long long)n * plen, back) == EC_OK,
          "ec_rebuild_segments_host");
    CHECK(memcmp(back, segs, nseg * spad) == 0, "rebuilt segments != input (%d,%d,%d)", k, n, ess);

    free(segs), free(pieces), free(pref), free(back);
    free(in), free(all), free(ref), free(one), free(out), free(out2), free(enc), free(vand), free(g);
    printf("[%9.1f ms]   ec_destroy\n", ms());
    ec_destroy(ctx);
}

/* A share set per segment (the cgo entry for concurrent downloads,
 * INTEGRATION.md "Many downloads at once"): nseg segments in device memory,
 * each rebuilt from its own set by ec_rebuild_segments_sets, then decoded with
 * error detection by ec_decode_segments_sets from k + 2 shares with one piece
 * corrupted -- outputs against the input, pieces against the oracle's. */
static void share_sets_surface(int k, int n, int ess) {
    ec_ctx *ctx = NULL;
    int rc = ec_create(k, n, ess, &ctx);
    CHECK(rc == EC_OK, "ec_create(%d,%d,%d) = %d", k, n, ess, rc);
    if (rc) return;
    uint8_t *enc = malloc((size_t)n * k), *vand = malloc((size_t)n * k);
    or_new_fec(k, n, enc, vand);
    enum { NSEG = 3 };
    const size_t stripes = 37, stripe = (size_t)k * ess, spad = stripes * stripe, plen = stripes * (size_t)ess;
    uint8_t *segs = malloc(NSEG * spad), *pieces = malloc(NSEG * (size_t)n * plen), *back = malloc(NSEG * spad);
    fill(segs, NSEG * spad);
    for (size_t g = 0; g < NSEG; g++)
        or_baseline_encode_segment(k, n, ess, enc, segs + g * spad, stripes, pieces + g * (size_t)n * plen, 1);
    uint8_t *d_pieces = ec_device_alloc(NSEG * (size_t)n * plen), *d_out = ec_device_alloc(NSEG * spad);
    CHECK(d_pieces && d_out, "ec_device_alloc");
    if (!d_pieces || !d_out) goto done;
    CHECK(ec_copy(d_pieces, pieces, NSEG * (size_t)n * plen) == EC_OK, "ec_copy H2D");
    /* segment 0: the last k shares (all parity when n >= 2k); 1: every other share from the top,
     * shuffled; 2: the data shares but one, plus share n-1 */
    int ns[NSEG], nums[NSEG * 256];
    const uint8_t *ptrs[NSEG * 256];
    uint8_t *outs[NSEG];
    int at = 0;
    for (int g = 0; g < NSEG; g++) {
        ns[g] = k;
        for (int i = 0; i < k; i++) {
            int num = g == 0 ? n - k + i : g == 1 ? (n - 1 - 2 * i + n) % n : (i < k - 1 ? i : n - 1);
            if (g == 1 && 2 * k > n) num = n - 1 - i;
            nums[at + i] = num;
        }
        if (g == 1)
            for (int i = k - 1; i > 0; i--) { /* any order */
                const int j = rnd8() % (i + 1), t = nums[at + i];
                nums[at + i] = nums[at + j], nums[at + j] = t;
            }
        for (int i = 0; i < k; i++) ptrs[at + i] = d_pieces + ((size_t)g * n + nums[at + i]) * plen;
        outs[g] = d_out + g * spad;
        at += k;
    }
    printf("[%9.1f ms]   ec_rebuild_segments_sets RS(%d,%d)\n", ms(), k, n);
    rc = ec_rebuild_segments_sets(ctx, NSEG, ns, nums, ptrs, stripes, outs, NULL);
    CHECK(rc == EC_OK, "ec_rebuild_segments_sets rc %d (%s)", rc, ec_strerror(rc));
    CHECK(ec_copy(back, d_out, NSEG * spad) == EC_OK, "ec_copy D2H");
    for (int g = 0; g < NSEG; g++)
        CHECK(memcmp(back + g * spad, segs + g * spad, spad) == 0, "sets rebuild: segment %d != input (%d,%d)", g, k, n);
    /* the same sets one segment per call (a lone download's segment: one launch, rows solved on the host) */
    {
        uint8_t *zero = calloc(NSEG * spad, 1);
        CHECK(ec_copy(d_out, zero, NSEG * spad) == EC_OK, "clear outputs");
        free(zero);
        for (int g = 0, off = 0; g < NSEG; off += ns[g], g++) {
            rc = ec_rebuild_segments_sets(ctx, 1, ns + g, nums + off, ptrs + off, stripes, outs + g, NULL);
            CHECK(rc == EC_OK, "ec_rebuild_segments_sets (one segment) rc %d (%s)", rc, ec_strerror(rc));
        }
        CHECK(ec_copy(back, d_out, NSEG * spad) == EC_OK, "ec_copy D2H");
        for (int g = 0; g < NSEG; g++)
            CHECK(memcmp(back + g * spad, segs + g * spad, spad) == 0, "sets rebuild, one per call: segment %d (%d,%d)", g,
                  k, n);
    }
    if (n - k >= 2) {
        /* Decode: k + 2 shares per segment, segment 1's second share corrupted in one byte */
        uint8_t *dptr[NSEG * 256];
        at = 0;
        for (int g = 0; g < NSEG; g++) {
            ns[g] = k + 2;
            for (int i = 0; i < k + 2; i++) {
                nums[at + i] = (g + 7 * i) % n; /* (7 is prime to every n here) */
                dptr[at + i] = d_pieces + ((size_t)g * n + nums[at + i]) * plen;
            }
            at += k + 2;
        }
        uint8_t *bad = dptr[(k + 2) + 1] + plen / 2 + 5, flip;
        CHECK(ec_copy(&flip, bad, 1) == EC_OK, "read a byte");
        flip ^= 0xA5;
        CHECK(ec_copy(bad, &flip, 1) == EC_OK, "corrupt a byte");
        uint8_t *zero = calloc(NSEG * spad, 1);
        CHECK(ec_copy(d_out, zero, NSEG * spad) == EC_OK, "clear outputs");
        free(zero);
        printf("[%9.1f ms]   ec_decode_segments_sets RS(%d,%d)\n", ms(), k, n);
        rc = ec_decode_segments_sets(ctx, NSEG, ns, nums, dptr, stripes, outs, NULL);
        CHECK(rc == EC_OK, "ec_decode_segments_sets rc %d (%s)", rc, ec_strerror(rc));
        CHECK(ec_copy(back, d_out, NSEG * spad) == EC_OK, "ec_copy D2H");
        for (int g = 0; g < NSEG; g++)
            CHECK(memcmp(back + g * spad, segs + g * spad, spad) == 0, "sets decode: segment %d != input (%d,%d)", g, k,
                  n);
        /* the corrupted share is corrected in place, as infectious corrects share.Data */
        uint8_t *fixed = malloc(plen);
        CHECK(ec_copy(fixed, dptr[(k + 2) + 1], plen) == EC_OK, "ec_copy D2H");
        CHECK(memcmp(fixed, pieces + ((size_t)n + nums[(k + 2) + 1]) * plen, plen) == 0,
              "sets decode: corrupted piece not corrected (%d,%d)", k, n);
        free(fixed);
    }
done:
    ec_device_free(d_pieces);
    ec_device_free(d_out);
    free(segs), free(pieces), free(back), free(enc), free(vand);
    ec_destroy(ctx);
}

/* BLAKE3 piece hashes and AES-256-GCM blocks through the host entry points */
static void adjacent_stages(void) {
    const size_t lens[] = {0, 1, 1024, 1025, 300000};
    for (size_t t = 0; t < sizeof lens / sizeof lens[0]; t++) {
        const size_t len = lens[t], np = 3;
        uint8_t *buf = malloc(np * len + 1), h[3 * 32], want[32];
        fill(buf, np * len + 1);
        CHECK(ec_blake3_host(buf, np, (long long)len, len, h) == EC_OK, "ec_blake3_host len %zu", len);
        for (size_t j = 0; j < np; j++) {
            b3_hash(buf + j * len, len, want);
            CHECK(memcmp(h + 32 * j, want, 32) == 0, "BLAKE3 piece %zu of length %zu", j, len);
        }
        free(buf);
    }
    uint8_t key[32], nonce[12];
    fill(key, 32);
    fill(nonce, 12);
    nonce[0] = 0xfe; /* the block counter carries into byte 1 */
    const size_t nb = 40, ib = 7408, ob = ib + 16;
    uint8_t *plain = malloc(nb * ib), *ct = malloc(nb * ob), *ref = malloc(nb * ob), *back = malloc(nb * ib);
    fill(plain, nb * ib);
    CHECK(ec_gcm_seal_host(key, nonce, plain, nb, ib, ct) == EC_OK, "ec_gcm_seal_host");
    CHECK(ag_encrypt_blocks(key, nonce, plain, nb, ib, ref, 4) == -1, "oracle seal");
    CHECK(memcmp(ct, ref, nb * ob) == 0, "GCM ciphertext || tag != oracle");
    long long bad = 0;
    CHECK(ec_gcm_open_host(key, nonce, ct, nb, ib, back, &bad) == EC_OK && bad == -1, "ec_gcm_open_host");
    CHECK(memcmp(back, plain, nb * ib) == 0, "GCM round trip");
    ct[17 * ob + ib + 3] ^= 1; /* a tag byte of block 17 */
    int rc = ec_gcm_open_host(key, nonce, ct, nb, ib, back, &bad);
    CHECK(rc == EC_ERR_AUTH && bad == 17, "tampered tag -> rc %d block %lld", rc, bad);
    CHECK(strcmp(ec_strerror(EC_ERR_AUTH), "cipher: message authentication failed") == 0, "auth error text");
    free(plain), free(ct), free(ref), free(back);
}

int main(int argc, char **argv) {
    setvbuf(stdout, NULL, _IONBF, 0); /* progress survives an abort */
    clock_gettime(CLOCK_MONOTONIC, &t_start);
    /* --build-id: which library this binary runs against, before any GPU work */
    if (argc > 1 && strcmp(argv[1], "--build-id") == 0) {
        printf("%s\n", ec_build_id());
        return 0;
    }
    printf("[%9.1f ms] library build %s\n", ms(), ec_build_id());
    ec_ctx *bad = NULL;
    CHECK(ec_create(0, 4, 256, &bad) == EC_ERR_PARAMS, "k = 0");
    CHECK(ec_create(5, 4, 256, &bad) == EC_ERR_PARAMS, "k > n");
    CHECK(ec_device_count() >= 1, "no device");
    const int cfg[][3] = {{2, 4, 1024}, {4, 10, 256}, {29, 80, 256}, {20, 60, 4096}, {3, 7, 100}, {10, 20, 64}};
    for (size_t i = 0; i < sizeof cfg / sizeof cfg[0]; i++) {
        for (int body = EC_BODY_AUTO; body <= EC_BODY_STRAIGHT_LINE; body += EC_BODY_STRAIGHT_LINE) {
            printf("[%9.1f ms] RS(%d,%d) ess %d body %d\n", ms(), cfg[i][0], cfg[i][1], cfg[i][2], body);
            scheme_surface(cfg[i][0], cfg[i][1], cfg[i][2], body);
        }
    }
    const int scfg[][3] = {{29, 80, 256}, {4, 10, 256}, {20, 60, 4096}};
    for (size_t i = 0; i < sizeof scfg / sizeof scfg[0]; i++) {
        printf("[%9.1f ms] share sets RS(%d,%d) ess %d\n", ms(), scfg[i][0], scfg[i][1], scfg[i][2]);
        share_sets_surface(scfg[i][0], scfg[i][1], scfg[i][2]);
    }
    printf("[%9.1f ms] adjacent stages\n", ms());
    adjacent_stages();
    printf("[%9.1f ms] returning from main (process exit follows)\n", ms());
    printf("%s: %d failures\n", failures ? "FAIL" : "ok", failures);
    return failures ? 1 : 0;
}
