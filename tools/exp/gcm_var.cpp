// Experiment: AES-GCM kernel T-table layouts (-DUPLINK_GCM_COPIES=0/32/64),
// seal and open of 8 x 9059 blocks of 7408 B; prints µs per segment and a
// checksum of the ciphertext (must agree across variants).
#include "../../uplink_amd/csrc/aesgcm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

int main() {
    const uint32_t NSEG = 8, NB = 9059, IB = 7408;
    const size_t pbytes = (size_t)NSEG * NB * IB, cbytes = (size_t)NSEG * NB * (IB + 16);
    uint8_t *plain, *ct, *back, *nonces;
    GcmSched *keys;
    int32_t *status;
    CK(hipMalloc(&plain, pbytes));
    CK(hipMalloc(&ct, cbytes));
    CK(hipMalloc(&back, pbytes));
    CK(hipMalloc(&keys, NSEG * sizeof(GcmSched)));
    CK(hipMalloc(&nonces, NSEG * 12));
    CK(hipMalloc(&status, NSEG * 4));
    std::vector<uint8_t> h(pbytes);
    for (size_t i = 0; i < pbytes; i++) h[i] = (uint8_t)(i * 2654435761u >> 13);
    CK(hipMemcpy(plain, h.data(), pbytes, hipMemcpyHostToDevice));
    std::vector<GcmSched> ks(NSEG);
    std::vector<uint8_t> nn(NSEG * 12);
    for (uint32_t g = 0; g < NSEG; g++) {
        uint8_t key[32];
        for (int i = 0; i < 32; i++) key[i] = (uint8_t)(g * 31 + i * 7);
        gcm_prepare(key, &ks[g]);
        for (int i = 0; i < 12; i++) nn[12 * g + i] = (uint8_t)(g + i);
    }
    CK(hipMemcpy(keys, ks.data(), NSEG * sizeof(GcmSched), hipMemcpyHostToDevice));
    CK(hipMemcpy(nonces, nn.data(), NSEG * 12, hipMemcpyHostToDevice));
    GcmBatch s{plain, ct, (int64_t)NB * IB, (int64_t)NB * (IB + 16), IB, IB + 16, keys, nonces, status, NSEG, NB, IB};
    GcmBatch o{ct, back, (int64_t)NB * (IB + 16), (int64_t)NB * IB, IB + 16, IB, keys, nonces, status, NSEG, NB, IB};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms[2];
    for (int m = 0; m < 2; m++) {
        for (int i = 0; i < 5; i++) CK(gcm_launch(m ? o : s, m == 1, 0));
        CK(hipEventRecord(a));
        for (int i = 0; i < 10; i++) CK(gcm_launch(m ? o : s, m == 1, 0));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms[m], a, b));
        ms[m] /= 10;
    }
    std::vector<uint8_t> c(cbytes), r(pbytes);
    CK(hipMemcpy(c.data(), ct, cbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), back, pbytes, hipMemcpyDeviceToHost));
    uint64_t sum = 0;
    for (size_t i = 0; i < cbytes; i += 7) sum = sum * 1099511628211ull + c[i];
    printf("lin %d tables %d copies %2d exp %d: seal %7.1f us/seg (%5.0f GB/s)  open %7.1f us/seg (%5.0f GB/s)  round trip %s  sum %016llx\n",
           UPLINK_GCM_LIN, UPLINK_GCM_TABLES, UPLINK_GCM_COPIES, UPLINK_GCM_EXP, ms[0] * 1e3 / NSEG, pbytes / (ms[0] * 1e6), ms[1] * 1e3 / NSEG, pbytes / (ms[1] * 1e6),
           r == h ? "ok" : "BAD", (unsigned long long)sum);
    return 0;
}
