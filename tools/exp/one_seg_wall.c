/* Developer experiment (GPU box): configs[2] as a C client (a cgo caller) sees
 * it -- one RS(29,80) 64 MiB segment rebuilt from a fresh seeded 29-subset per
 * call through ec_rebuild_segments_sets, wall clock from the call to the
 * stream synchronised, median of 200 calls; beside it the same clock around a
 * 4-byte hipMemsetAsync (this box's floor for one stream operation and a
 * synchronisation from C).  The pieces are not a codeword (timing only).
 *   gcc -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/exp/one_seg_wall.c \
 *       -Luplink_amd/lib -luplink_ec -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/uplink_amd/lib \
 *       -Wl,-rpath,/opt/rocm/lib -o tools/exp/bin/one_seg_wall */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uplink_ec.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static uint64_t rng = 20261018;
static uint32_t rnd(void) {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(rng >> 33);
}

int main(void) {
    enum { K = 29, N = 80, ESS = 256, REPS = 200 };
    const size_t stripes = 9040, plen = stripes * ESS, spad = stripes * (size_t)K * ESS;
    ec_ctx *ctx = NULL;
    if (ec_create(K, N, ESS, &ctx) != EC_OK) return 1;
    uint8_t *pieces = ec_device_alloc((size_t)N * plen), *out = ec_device_alloc(spad);
    if (!pieces || !out) return 1;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    double call[REPS], wall[REPS], floor_[REPS];
    for (int r = -5; r < REPS; r++) {
        int perm[N];
        for (int i = 0; i < N; i++) perm[i] = i;
        for (int i = N - 1; i > 0; i--) {
            const int j = (int)(rnd() % (uint32_t)(i + 1)), t = perm[i];
            perm[i] = perm[j], perm[j] = t;
        }
        int ns = K;
        const uint8_t *ptrs[K];
        for (int i = 0; i < K; i++) ptrs[i] = pieces + (size_t)perm[i] * plen;
        uint8_t *outs[1] = {out};
        (void)hipStreamSynchronize(s);
        const double t0 = now_us();
        if (ec_rebuild_segments_sets(ctx, 1, &ns, perm, ptrs, stripes, outs, (ec_stream)s) != EC_OK) return 2;
        const double t1 = now_us();
        (void)hipStreamSynchronize(s);
        const double t2 = now_us();
        (void)hipMemsetAsync(out, 0, 4, s);
        (void)hipStreamSynchronize(s);
        const double t3 = now_us();
        if (r >= 0) call[r] = t1 - t0, wall[r] = t2 - t0, floor_[r] = t3 - t2;
    }
    qsort(call, REPS, sizeof(double), cmp);
    qsort(wall, REPS, sizeof(double), cmp);
    qsort(floor_, REPS, sizeof(double), cmp);
    printf("{\"one_segment_wall_us_median\": %.1f, \"wall_us_min\": %.1f, \"call_returns_us_median\": %.1f, "
           "\"memset4_wall_us_median\": %.1f, \"calls\": %d}\n",
           wall[REPS / 2], wall[0], call[REPS / 2], floor_[REPS / 2], REPS);
    ec_device_free(pieces);
    ec_device_free(out);
    (void)hipStreamDestroy(s);
    ec_destroy(ctx);
    return 0;
}
