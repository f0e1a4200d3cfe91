/* Per-stripe ErasureScheme calls through the C-ABI from many OS threads, as an
 * unchanged Go caller makes them (no Python, no GIL):
 *   segmentupload's EncodedReader calls EncodeSingle once per (piece, stripe)
 *   (private/storage/streams/segmentupload/encode.go:58) from up to 300 piece
 *   goroutines (private/testuplink/uplink.go:83); StripeReader calls Rebuild
 *   once per stripe (private/eestream/stripe.go:407-413).
 * For RS(29,80), ess 256 (7424-byte stripes): aggregate calls/s and mean
 * latency of ec_encode_single (parity pieces) and ec_rebuild (all-parity share
 * set) from T threads, next to the CPU oracle's or_encode_single / or_rebuild
 * (infectious' per-call work) on the same threads.  One JSON line.
 *   gcc -O2 -std=gnu11 -Iinclude tools/per_stripe_bench.c -o per_stripe_bench \
 *       -Luplink_amd/lib -luplink_ec -Loracle/build -linfectious_oracle -lpthread
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uplink_ec.h"

int or_lagrange_fec(int k, int n, uint8_t *enc_matrix);
int or_encode(int k, int n, const uint8_t *enc, const uint8_t *in, size_t in_len, uint8_t *out);
int or_encode_single(int k, int n, const uint8_t *enc, const uint8_t *in, size_t in_len, uint8_t *out,
                     size_t out_len, int num);
int or_rebuild(int k, int n, const uint8_t *enc, int ns, int *numbers, const uint8_t **data, size_t len,
               uint8_t *out);

enum { K = 29, N = 80, ESS = 256, STRIPE = K * ESS, NSTRIPE = 64 };

static ec_ctx *g_ctx;
static uint8_t g_enc[N * K];
static uint8_t *g_stripes;  /* NSTRIPE x STRIPE */
static uint8_t *g_shares;   /* NSTRIPE x N x ESS */
static double g_seconds = 1.0;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

typedef struct {
    int id, mode; /* 0 gpu encode_single, 1 gpu rebuild, 2 cpu encode_single, 3 cpu rebuild */
    double stop;
    long calls;
    double busy;
    int err;
} Worker;

static void *run(void *p) {
    Worker *w = (Worker *)p;
    uint8_t out[STRIPE];
    long i = 0;
    const double t0 = now();
    while (now() < w->stop) {
        const int s = (int)((w->id * 7 + i) % NSTRIPE);
        const uint8_t *stripe = g_stripes + (size_t)s * STRIPE;
        int rc = 0;
        if (w->mode == 0 || w->mode == 2) {
            const int num = K + (int)(i % (N - K));
            rc = w->mode == 0 ? ec_encode_single(g_ctx, stripe, STRIPE, out, ESS, num)
                              : or_encode_single(K, N, g_enc, stripe, STRIPE, out, ESS, num);
        } else {
            int nums[K];
            const uint8_t *sh[K];
            for (int j = 0; j < K; j++) {
                nums[j] = N - K + j;
                sh[j] = g_shares + ((size_t)s * N + (size_t)nums[j]) * ESS;
            }
            rc = w->mode == 1 ? ec_rebuild(g_ctx, K, nums, sh, ESS, out) : or_rebuild(K, N, g_enc, K, nums, sh, ESS, out);
            if (!rc && memcmp(out, stripe, STRIPE)) rc = -99;
        }
        if (rc) {
            w->err = rc;
            break;
        }
        i++;
    }
    w->calls = i;
    w->busy = now() - t0;
    return NULL;
}

static void measure(const char *name, int mode, int threads, int first) {
    Worker *w = calloc((size_t)threads, sizeof(Worker));
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    const double t0 = now(), stop = t0 + g_seconds;
    for (int t = 0; t < threads; t++) {
        w[t].id = t;
        w[t].mode = mode;
        w[t].stop = stop;
        pthread_create(&th[t], NULL, run, &w[t]);
    }
    long calls = 0;
    double lat = 0;
    int err = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        calls += w[t].calls;
        lat += w[t].busy / (w[t].calls ? w[t].calls : 1);
        if (w[t].err) err = w[t].err;
    }
    const double wall = now() - t0;
    printf("%s{\"op\": \"%s\", \"threads\": %d, \"calls_per_s\": %.0f, \"mean_latency_us\": %.2f, "
           "\"MB_per_s_of_stripes\": %.1f, \"error\": %d}",
           first ? "" : ", ", name, threads, calls / wall, lat / threads * 1e6, calls * (double)STRIPE / wall / 1e6, err);
    fflush(stdout);
    free(w);
    free(th);
}

int main(int argc, char **argv) {
    if (argc > 1) g_seconds = atof(argv[1]);
    if (ec_create(K, N, ESS, &g_ctx) != EC_OK) {
        fprintf(stderr, "ec_create failed\n");
        return 1;
    }
    or_lagrange_fec(K, N, g_enc);
    g_stripes = malloc((size_t)NSTRIPE * STRIPE);
    g_shares = malloc((size_t)NSTRIPE * N * ESS);
    srand(1);
    for (size_t i = 0; i < (size_t)NSTRIPE * STRIPE; i++) g_stripes[i] = (uint8_t)rand();
    for (int s = 0; s < NSTRIPE; s++)
        or_encode(K, N, g_enc, g_stripes + (size_t)s * STRIPE, STRIPE, g_shares + (size_t)s * N * ESS);
    const int threads[] = {1, 4, 16, 64, 300};
    printf("{\"config\": \"RS(29,80), ess 256, one 7424-byte stripe per call, C threads\", \"results\": [");
    int first = 1;
    for (int t = 0; t < 5; t++) {
        measure("ec_encode_single", 0, threads[t], first);
        first = 0;
        measure("ec_rebuild", 1, threads[t], 0);
        measure("oracle_encode_single", 2, threads[t], 0);
        measure("oracle_rebuild", 3, threads[t], 0);
    }
    printf("]}\n");
    ec_destroy(g_ctx);
    return 0;
}
