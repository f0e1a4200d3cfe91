// Experiment: BLAKE3 piece-hash kernel variants (workgroup group size,
// 128-B line loads) timed through b3_launch / b3_launch2 on 640 pieces of
// 2,314,240 B (8 RS(29,80) segments), contiguous and in the segment form.
// Built several times with -DUPLINK_B3_GROUP=.. -DUPLINK_B3_LINES=.. by
// tools/exp/b3_var.sh; prints µs per segment and a hash checksum.
#include "../../uplink_amd/csrc/blake3.hip"

#include <cstdio>
#include <cstdlib>

using namespace uplink_ec;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

int main() {
    const uint64_t K = 29, N = 80, ESS = 256, S = 9040, NSEG = 8, PLEN = S * ESS;
    uint8_t *segs, *par, *h;
    void *ws;
    CK(hipMalloc(&segs, NSEG * S * K * ESS));
    CK(hipMalloc(&par, NSEG * (N - K) * PLEN));
    CK(hipMalloc(&h, NSEG * N * 32));
    CK(hipMalloc(&ws, 64 << 20));
    CK(hipMemset(segs, 0x3c, NSEG * S * K * ESS));
    CK(hipMemset(par, 0xa7, NSEG * (N - K) * PLEN));
    B3View data{segs, (int64_t)ESS, PLEN, ESS, (int64_t)(K * ESS), NSEG * K, K, (int64_t)(PLEN * K), 0};
    B3View parity{par, (int64_t)PLEN, PLEN, PLEN, (int64_t)PLEN, NSEG * (N - K), 0, 0, 0};
    B3View contig{par, (int64_t)PLEN, PLEN, PLEN, (int64_t)PLEN, NSEG * (N - K), 0, 0, 0};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](auto f) {
        for (int i = 0; i < 30; i++) f();
        CK(hipEventRecord(a));
        for (int i = 0; i < 30; i++) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 30 * 1e3;
    };
    float tseg = timeit([&] { CK(b3_launch2(data, parity, h, ws, 0)); });
    uint8_t hh[NSEG * N * 32];
    CK(hipMemcpy(hh, h, sizeof hh, hipMemcpyDeviceToHost));
    uint64_t sum = 0;
    for (size_t i = 0; i < sizeof hh; i++) sum = sum * 131 + hh[i];
    float tpar = timeit([&] { CK(b3_launch(contig, h, ws, 0)); });
    printf("group %4d lines %d: segment form %7.1f us/seg (%6.0f GB/s)  parity-only contiguous %7.1f us per 51 "
           "pieces x 8 (%6.0f GB/s)  sum %016llx\n",
           UPLINK_B3_GROUP, UPLINK_B3_LINES, tseg / NSEG, NSEG * N * PLEN / (tseg * 1e3), tpar,
           NSEG * (N - K) * PLEN / (tpar * 1e3), (unsigned long long)sum);
    return 0;
}
