/* Process exit while the library compiles a run-time encoder.
 * A caller that asks for an RS(k, n) with no compiled encoder gets the
 * runtime-matrix kernel at once while hiprtc compiles the encoder in a
 * background thread.  This client returns from main with that compile still
 * running, with no ec_destroy: exit() must wait for the compile before the
 * compiler library's static destructors run (round 2 aborted here with
 * "double free or corruption (!prev)").  Run with UPLINK_EC_JIT_CACHE set to
 * an empty directory (tests/test_c_abi.py), so the compile cannot come from
 * the cache.  Exit status 0 and nothing on stderr = pass. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uplink_ec.h"

int main(int argc, char **argv) {
    const int k = argc > 2 ? atoi(argv[1]) : 11, n = argc > 2 ? atoi(argv[2]) : 23, ess = 256;
    const size_t stripes = 64;
    ec_ctx *ctx = NULL;
    int rc = ec_create(k, n, ess, &ctx);
    if (rc != EC_OK) {
        fprintf(stderr, "ec_create: %s\n", ec_strerror(rc));
        return 2;
    }
    uint8_t *seg = malloc((size_t)k * ess * stripes), *pieces = malloc((size_t)n * ess * stripes);
    for (size_t i = 0; i < (size_t)k * ess * stripes; i++) seg[i] = (uint8_t)(i * 131 + 7);
    /* a small encode (8 tiles) runs on the runtime-matrix kernel and starts no compile */
    rc = ec_encode_segments_host(ctx, seg, 1, stripes, pieces, 0);
    if (rc != EC_OK) {
        fprintf(stderr, "ec_encode_segments_host: %s\n", ec_strerror(rc));
        return 3;
    }
    if (memcmp(pieces, seg, (size_t)ess * stripes) != 0) {
        fprintf(stderr, "piece 0 is not the first share of each stripe\n");
        return 4;
    }
    /* ec_prepare_encoder without wait starts the compile; 0 = the compiled encoder is not
     * loaded yet: the compile is still running */
    if (ec_prepare_encoder(ctx, 0) != 0) {
        fprintf(stderr, "RS(%d,%d)'s encoder was already compiled: the test needs an empty cache\n", k, n);
        return 5;
    }
    /* let the compile thread get going (a compile still queued when exit starts is skipped,
     * not waited for); it takes ~1 s or more cold, so it is still running when main returns */
    struct timespec ts = {0, 100 * 1000 * 1000};
    nanosleep(&ts, NULL);
    printf("returning from main while RS(%d,%d)'s encoder compiles\n", k, n);
    return 0;
}
