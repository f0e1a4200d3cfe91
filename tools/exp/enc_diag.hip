// Developer experiment (not product), round 4: the
// product's RS(29,80) encoder body (rs_encoder.hpp encode_body, 8 compute + 4
// loader waves, one workgroup per CU, 16 x 64 MiB segments per launch as in
// bench.py) in its diagnostic forms:
//   stamp      in-kernel clock = d(s_memtime) / d(s_memrealtime) x 100 MHz
//              around the tile loop (MI355X_MICROARCH.md 'DVFS give-back'
//              item 6), median over workgroups, and the share of the loop
//              compute wave 0 / loader wave 0 spend waiting
//   nopar      parity rows computed and kept live by an empty asm, not stored
//   nocopy     the data pieces' copy-through not stored
//   nostore    both
// on random, constant (0x5a) and all-zero segments, after >= 2 s of
// back-to-back launches, interleaved over rounds on one device.  The forms
// that store everything are checked byte for byte against the plain body.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/exp/enc_diag.hip -o tools/exp/bin/enc_diag
//   tools/exp/bin/enc_diag [rounds] [mode mask: 1 random b2b, 2 random alternating, 4 const, 8 zeros]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../uplink_amd/csrc/rs_encoder.hpp"

using namespace uplink_ec;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr int K = 29, N = 80, R = N - K, ESS = 256, NC = 8, NL = 4, NSEG = 16;
constexpr int64_t NSTRIPES = (64ll * 1024 * 1024 + 4 + K * ESS - 1) / (K * ESS);
constexpr int64_t SPAD = NSTRIPES * K * ESS, PLEN = NSTRIPES * ESS;

template <bool COPY, int DIAG, int NCV = NC, int NLV = NL>
__global__ __launch_bounds__((NCV + NLV) * 64, 1) void enc_diag(const RsArgs a) {
    enc::encode_body<K, N, NCV, NLV, COPY, DIAG>(a);
}

__global__ void fill_rand(uint8_t *p, int64_t n16, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        uint32_t w[4];
        for (int k = 0; k < 4; k++) {
            x ^= x >> 30, x *= 0xBF58476D1CE4E5B9ull, x ^= x >> 27, x *= 0x94D049BB133111EBull, x ^= x >> 31;
            w[k] = (uint32_t)x;
        }
        *(uint4 *)(p + i * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

struct Variant {
    const char *name;
    bool copy;
    int diag;
    void (*launch)(const RsArgs &, int, hipStream_t);
};

template <bool COPY, int DIAG, int NCV = NC, int NLV = NL>
void launch(const RsArgs &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((enc_diag<COPY, DIAG, NCV, NLV>), dim3(grid), dim3((NCV + NLV) * 64), 0, s, a);
}

static RsArgs make_args(const uint8_t *segs, uint8_t *out, bool copy, uint32_t *queue, uint64_t *diag) {
    RsArgs a{};
    a.in_base = segs;
    a.out_base = out;
    a.in_stripe_stride = (int64_t)K * ESS;
    a.out_stripe_stride = ESS;
    a.in_seg_stride = SPAD;
    a.out_seg_stride = (int64_t)(copy ? N : R) * PLEN;
    a.nin = K;
    a.nout = R;
    for (int j = 0; j < K; j++) {
        a.in_off[j] = (int64_t)j * ESS;
        a.copy_off[j] = copy ? (int64_t)j * PLEN : -1;
    }
    for (int r = 0; r < R; r++) a.out_off[r] = (int64_t)(copy ? K + r : r) * PLEN;
    a.ess = ESS;
    a.cps = ESS / 16;
    a.nstripes = NSTRIPES;
    a.chunks_per_seg = NSTRIPES * (ESS / 16);
    a.tiles_per_seg = (a.chunks_per_seg + 127) / 128;
    a.total_tiles = a.tiles_per_seg * NSEG;
    a.blocks_per_seg = (a.chunks_per_seg + 63) / 64;
    a.total_blocks = a.blocks_per_seg * NSEG;
    a.queue = queue;
    a.diag = diag;
    return a;
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = cus;  // one workgroup per CU, as the library launches it
    uint8_t *segs, *pieces, *pieces2;
    uint32_t *queue;
    uint64_t *diag;
    CK(hipMalloc(&segs, SPAD * NSEG));
    CK(hipMalloc(&pieces, (int64_t)N * PLEN * NSEG));
    CK(hipMalloc(&pieces2, (int64_t)N * PLEN * NSEG));
    CK(hipMalloc(&queue, 256));
    CK(hipMemset(queue, 0, 256));
    CK(hipMalloc(&diag, sizeof(uint64_t) * 8 * grid));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    constexpr int S = enc::kDiagStamp, NP = enc::kDiagNoParityStores, NCP = enc::kDiagNoCopyStores;
    constexpr int NCB = enc::kDiagNoCombos, NR = enc::kDiagNoRowOps, HC = enc::kDiagHalfCombos,
                  LC = enc::kDiagLdsCombos;
    const Variant vars[] = {
        {"full", true, 0, launch<true, 0>},
        {"full stamp", true, S, launch<true, S>},
        {"full nopar", true, S | NP, launch<true, S | NP>},
        {"full nocopy", true, S | NCP, launch<true, S | NCP>},
        {"full nostore", true, S | NP | NCP, launch<true, S | NP | NCP>},
        {"full nocombo", true, S | NCB, launch<true, S | NCB>},
        {"full norowops", true, S | NR, launch<true, S | NR>},
        {"full norow+nost", true, S | NR | NP | NCP, launch<true, S | NR | NP | NCP>},
        {"full halfcombo", true, S | HC, launch<true, S | HC>},
        {"full ldscombo", true, S | LC, launch<true, S | LC>},
        {"full 4c+4l", true, S, launch<true, S, 4, 4>},
        {"full 6c+4l", true, S, launch<true, S, 6, 4>},
        {"full 6c+6l", true, S, launch<true, S, 6, 6>},
        {"full 8c+8l", true, S, launch<true, S, 8, 8>},
        {"parity", false, 0, launch<false, 0>},
        {"parity stamp", false, S, launch<false, S>},
        {"parity nopar", false, S | NP, launch<false, S | NP>},
        {"parity nocombo", false, S | NCB, launch<false, S | NCB>},
        {"parity norowops", false, S | NR, launch<false, S | NR>},
        {"parity halfcombo", false, S | HC, launch<false, S | HC>},
        {"parity ldscombo", false, S | LC, launch<false, S | LC>},
        {"parity 4c+4l", false, S, launch<false, S, 4, 4>},
        {"parity 6c+4l", false, S, launch<false, S, 6, 4>},
    };
    const double alg_full = (double)SPAD * NSEG * (1.0 + (double)N / K);
    const double alg_par = (double)SPAD * NSEG * (1.0 + (double)R / K);
    // mode 1: each encode followed by a device copy of 2 x the segments' bytes (about the rebuild's
    // traffic and time in bench.py's encode/rebuild alternation), only the encodes timed
    const char *modes[] = {"random, back to back", "random, alternating with a copy", "const 0x5a", "zeros"};
    uint8_t *cpy_a, *cpy_b;
    CK(hipMalloc(&cpy_a, SPAD * NSEG));
    CK(hipMalloc(&cpy_b, SPAD * NSEG));
    std::vector<hipEvent_t> evs(40);
    for (auto &e : evs) CK(hipEventCreate(&e));
    const int mode_mask = argc > 2 ? atoi(argv[2]) : 15;
    for (int mode = 0; mode < 4; mode++) {
        if (!(mode_mask & (1 << mode))) continue;
        const bool alt = mode == 1;
        if (mode <= 1) hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, s, segs, SPAD * NSEG / 16, 12345u);
        else CK(hipMemsetAsync(segs, mode == 2 ? 0x5a : 0, SPAD * NSEG, s));
        CK(hipStreamSynchronize(s));
        // the stamping and plain forms produce the same pieces
        for (const Variant &v : vars) {
            if (v.diag & (enc::kDiagNoParityStores | enc::kDiagNoCopyStores)) continue;
            if (v.diag != 0) continue;
            RsArgs a = make_args(segs, pieces, v.copy, queue, nullptr);
            v.launch(a, grid, s);
            RsArgs b = make_args(segs, pieces2, v.copy, queue, diag);
            (v.copy ? launch<true, enc::kDiagStamp> : launch<false, enc::kDiagStamp>)(b, grid, s);
            CK(hipStreamSynchronize(s));
            const int64_t bytes = (int64_t)(v.copy ? N : R) * PLEN * NSEG;
            std::vector<uint8_t> h1(bytes), h2(bytes);
            CK(hipMemcpy(h1.data(), pieces, bytes, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), pieces2, bytes, hipMemcpyDeviceToHost));
            printf("[%s] %s: stamp form %s the plain body\n", modes[mode], v.name,
                   memcmp(h1.data(), h2.data(), bytes) == 0 ? "equals" : "DIFFERS from");
        }
        // >= 2 s of back-to-back launches first
        {
            RsArgs a = make_args(segs, pieces, true, queue, nullptr);
            const auto t0 = std::chrono::steady_clock::now();
            while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
                for (int i = 0; i < 10; i++) {
                    launch<true, 0>(a, grid, s);
                    if (alt) CK(hipMemcpyAsync(cpy_b, cpy_a, SPAD * NSEG, hipMemcpyDeviceToDevice, s));
                }
                CK(hipStreamSynchronize(s));
            }
        }
        const int nv = sizeof(vars) / sizeof(vars[0]);
        std::vector<std::vector<double>> us(nv), clk(nv), wcomp(nv), wload(nv);
        for (int r = 0; r < rounds; r++) {
            for (int vi = 0; vi < nv; vi++) {
                const Variant &v = vars[vi];
                RsArgs a = make_args(segs, pieces, v.copy, queue, (v.diag & enc::kDiagStamp) ? diag : nullptr);
                for (int i = 0; i < 3; i++) v.launch(a, grid, s);
                const int it = 10;
                float ms = 0;
                if (alt) {
                    for (int i = 0; i < it; i++) {
                        CK(hipEventRecord(evs[2 * i], s));
                        v.launch(a, grid, s);
                        CK(hipEventRecord(evs[2 * i + 1], s));
                        CK(hipMemcpyAsync(cpy_b, cpy_a, SPAD * NSEG, hipMemcpyDeviceToDevice, s));
                    }
                    CK(hipStreamSynchronize(s));
                    for (int i = 0; i < it; i++) {
                        float m1;
                        CK(hipEventElapsedTime(&m1, evs[2 * i], evs[2 * i + 1]));
                        ms += m1;
                    }
                } else {
                    CK(hipEventRecord(e0, s));
                    for (int i = 0; i < it; i++) v.launch(a, grid, s);
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                }
                us[vi].push_back(ms * 1e3 / it);
                if (v.diag & enc::kDiagStamp) {
                    std::vector<uint64_t> h(8 * grid);
                    CK(hipMemcpy(h.data(), diag, h.size() * 8, hipMemcpyDeviceToHost));
                    std::vector<double> c, wc, wl;
                    for (int g = 0; g < grid; g++) {
                        const uint64_t *d = &h[8 * g];
                        if (d[3] == 1 && d[1] > 0) {
                            c.push_back((double)d[0] / (double)d[1] * 0.1);  // GHz: ticks per 10-ns tick
                            wc.push_back((double)d[2] / (double)d[0]);
                        }
                        if (d[7] == 1 && d[4] > 0) wl.push_back((double)d[6] / (double)d[4]);
                    }
                    clk[vi].push_back(median(c));
                    wcomp[vi].push_back(median(wc));
                    wload[vi].push_back(median(wl));
                }
            }
        }
        printf("[%s] us per launch of %d segments (median over %d rounds of 10), TB/s of the algorithmic bytes\n",
               modes[mode], NSEG, rounds);
        for (int vi = 0; vi < nv; vi++) {
            const Variant &v = vars[vi];
            const double m = median(us[vi]);
            printf("  %-14s %8.1f us  %6.3f TB/s", v.name, m, (v.copy ? alg_full : alg_par) / m / 1e6);
            if (!clk[vi].empty())
                printf("  clock %.3f GHz  wait share: compute wave 0 %.3f, loader wave 0 %.3f", median(clk[vi]),
                       median(wcomp[vi]), median(wload[vi]));
            printf("\n");
        }
        fflush(stdout);
    }
    return 0;
}
