// Developer experiment (not product): memory shapes for the RS(29,80) encode,
// with no GF arithmetic, on the encode's exact addresses (16 stripe-major
// 64 MiB segments [stripe][29][256] -> 80 piece streams of 9040 x 256 B each).
// Round-3 VERDICT item 1: find a per-wave grouping of the encode's 1 : 2.76
// read:write mix that moves > 5.6 TB/s before rebuilding the kernel around it.
//
// Every shape: a tile is CPL x 1 KiB of byte columns (CPL 16-B chunks per lane
// per share row); its 29 input rows are loaded (16 B per lane, non-temporal),
// copied through to the data pieces, parked in LDS; one barrier; the 51
// parity rows are written (each the XOR of two LDS rows: a data dependence on
// the staged tile, no GF math).  Rows are dealt round-robin over the NW waves
// of a workgroup.  FAKE = VALU instructions per wave between barrier and
// stores (emulates the multiply); PERSIST = grid of G workgroups looping over
// tiles instead of one workgroup per tile.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 enc_shape_probe.hip -o enc_shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

constexpr int K = 29, N = 80, R = N - K, ESS = 256, NS = 9040, NSEG = 16;
constexpr int64_t SPAD = (int64_t)NS * K * ESS, PLEN = (int64_t)NS * ESS;
constexpr int64_t CPS = PLEN / 16;  // 16-B chunks per share row of a segment: 144,640

__device__ __forceinline__ v4 ldnt(const uint8_t *p) { return __builtin_nontemporal_load((const v4 *)p); }
__device__ __forceinline__ void stnt(uint8_t *p, v4 v) { __builtin_nontemporal_store(v, (v4 *)p); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Opt {
    int64_t pstride;  // bytes between piece streams (PLEN in the real layout)
    int contig;       // 1: a tile's 80 rows written contiguously ([tile][80][CPL KiB])
    int copy;         // write the 29 data pieces
    int read;         // load the inputs (0: rows made from registers)
    int order;        // 1: consecutive blocks take consecutive segments (seg = b % NSEG)
};

template <int NW, int CPL>
__device__ __forceinline__ void do_tile(const uint8_t *in, uint8_t *out, int64_t tile, v4 *lds, int fake, int lane,
                                        int wave, const Opt o) {
    constexpr int64_t TPS = CPS / (64 * CPL);
    constexpr int PER = (K + NW - 1) / NW, PR = (R + NW - 1) / NW;
    int64_t seg = tile / TPS, tt = tile - seg * TPS;
    if (o.order) seg = tile % NSEG, tt = tile / NSEG;
    const uint8_t *is = in + seg * SPAD;
    uint8_t *os = out + seg * (int64_t)N * o.pstride;
    int64_t qin[CPL], qout[CPL];
    const int64_t pst = o.contig ? (int64_t)CPL * 1024 : o.pstride;
    if (o.contig) os = out + (seg * TPS + tt) * (int64_t)N * CPL * 1024;
#pragma unroll
    for (int c = 0; c < CPL; c++) {
        const int64_t q = tt * 64 * CPL + c * 64 + lane;
        qin[c] = (q >> 4) * (K * ESS) + (q & 15) * 16;
        qout[c] = o.contig ? (c * 64 + lane) * 16 : q * 16;
    }
    v4 x[PER][CPL];
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < K)
#pragma unroll
            for (int c = 0; c < CPL; c++)
                x[i][c] = o.read ? ldnt(is + j * ESS + qin[c]) : (v4){(uint32_t)j, (uint32_t)c, (uint32_t)lane, 7u};
    }
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < K)
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                if (o.copy) stnt(os + j * pst + qout[c], x[i][c]);
                lds[(j * CPL + c) * 64 + lane] = x[i][c];
            }
    }
    lds_barrier();
    // emulated multiply: `fake` independent bitop3 per wave, fed from LDS
    v4 f = lds[wave * 64 + lane];
    uint32_t a0 = f.x, a1 = f.y, a2 = f.z, a3 = f.w, a4 = f.x ^ 1, a5 = f.y ^ 2, a6 = f.z ^ 3, a7 = f.w ^ 4;
    for (int it = 0; it < fake; it += 8) {
        a0 = __builtin_amdgcn_bitop3_b32(a0, a1, a2, 0x96);
        a1 = __builtin_amdgcn_bitop3_b32(a1, a2, a3, 0x96);
        a2 = __builtin_amdgcn_bitop3_b32(a2, a3, a4, 0x96);
        a3 = __builtin_amdgcn_bitop3_b32(a3, a4, a5, 0x96);
        a4 = __builtin_amdgcn_bitop3_b32(a4, a5, a6, 0x96);
        a5 = __builtin_amdgcn_bitop3_b32(a5, a6, a7, 0x96);
        a6 = __builtin_amdgcn_bitop3_b32(a6, a7, a0, 0x96);
        a7 = __builtin_amdgcn_bitop3_b32(a7, a0, a1, 0x96);
    }
    const uint32_t salt = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
#pragma unroll
    for (int i = 0; i < PR; i++) {
        const int r = wave + NW * i;
        if (r < R)
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                v4 v = lds[((r % K) * CPL + c) * 64 + lane] ^ lds[(((r + 7) % K) * CPL + c) * 64 + lane];
                v.x ^= salt;
                stnt(os + (K + r) * pst + qout[c], v);
            }
    }
}

template <int NW, int CPL>
__global__ __launch_bounds__(NW * 64) void oneshot(const uint8_t *in, uint8_t *out, int fake, const Opt o) {
    extern __shared__ v4 lds[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    do_tile<NW, CPL>(in, out, blockIdx.x, lds, fake, lane, wave, o);
}

template <int NW, int CPL>
__global__ __launch_bounds__(NW * 64) void persist(const uint8_t *in, uint8_t *out, int fake, int64_t ntiles,
                                                   const Opt o) {
    extern __shared__ v4 lds[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        do_tile<NW, CPL>(in, out, t, lds, fake, lane, wave, o);
        lds_barrier();
    }
}

int main(int argc, char **argv) {
    uint8_t *in, *out;
    CK(hipMalloc(&in, SPAD * NSEG));
    const int64_t OUTB = (int64_t)N * (PLEN + (1 << 20)) * NSEG;  // room for padded piece strides
    CK(hipMalloc(&out, OUTB));
    CK(hipMemset(in, 0x5a, SPAD * NSEG));
    CK(hipMemset(out, 0x33, OUTB));
    Opt o = {PLEN, 0, 1, 1, 0};
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)SPAD * NSEG * (1.0 + (double)N / K);
    auto timeit = [&](const char *name, auto launch) {
        for (int i = 0; i < 5; i++) launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-58s %8.1f us/launch %6.2f us/seg %6.3f TB/s\n", name, us, us / NSEG, bytes / us / 1e6);
        fflush(stdout);
    };
    // fake VALU per wave: the real encode's ~18.3 k wave-VALU per 2 KiB-wide tile, spread over the waves
    auto fake_for = [](int nw, int cpl, double scale) { return (int)(scale * 9150.0 * cpl / nw + 7) / 8 * 8; };
#define ONESHOT(NW, CPL, SCALE, PADKB)                                                                              \
    {                                                                                                             \
        const int64_t nt = (int64_t)NSEG * (CPS / (64 * (CPL)));                                                  \
        const int fake = fake_for(NW, CPL, SCALE);                                                                \
        const size_t lb = (size_t)K * (CPL) * 1024 + (size_t)(PADKB) * 1024;                                     \
        char nm[128];                                                                                             \
        snprintf(nm, sizeof nm, "oneshot NW=%d CPL=%d fake=%d lds=%zuK", NW, CPL, fake, lb / 1024);              \
        timeit(nm, [&] { hipLaunchKernelGGL((oneshot<NW, CPL>), dim3(nt), dim3(NW * 64), lb, 0, in, out, fake, o); }); \
    }
#define PERSIST(NW, CPL, SCALE, WPC, PADKB)                                                                         \
    {                                                                                                             \
        const int64_t nt = (int64_t)NSEG * (CPS / (64 * (CPL)));                                                  \
        const int fake = fake_for(NW, CPL, SCALE);                                                                \
        const size_t lb = (size_t)K * (CPL) * 1024 + (size_t)(PADKB) * 1024;                                     \
        char nm[128];                                                                                             \
        snprintf(nm, sizeof nm, "persist NW=%d CPL=%d fake=%d wg/cu=%d lds=%zuK", NW, CPL, fake, WPC, lb / 1024); \
        timeit(nm, [&] {                                                                                          \
            hipLaunchKernelGGL((persist<NW, CPL>), dim3(cus * (WPC)), dim3(NW * 64), lb, 0, in, out, fake, nt, o);\
        });                                                                                                       \
    }
    const int which = argc > 1 ? atoi(argv[1]) : 0;
    if (which == 0 || which == 1) {
        // memory only
        ONESHOT(4, 1, 0, 0) ONESHOT(8, 1, 0, 0) ONESHOT(16, 1, 0, 0)
        ONESHOT(4, 2, 0, 0) ONESHOT(8, 2, 0, 0) ONESHOT(16, 2, 0, 0)
        ONESHOT(8, 4, 0, 0) ONESHOT(16, 4, 0, 0)
        PERSIST(8, 2, 0, 2, 0) PERSIST(16, 2, 0, 2, 0) PERSIST(8, 1, 0, 4, 0) PERSIST(16, 1, 0, 2, 0)
    }
    if (which == 0 || which == 2) {
        // with the emulated multiply, and occupancy capped by LDS as a real kernel's registers would
        ONESHOT(8, 2, 1.0, 0) ONESHOT(16, 2, 1.0, 0) ONESHOT(8, 1, 1.0, 0) ONESHOT(16, 1, 1.0, 0)
        ONESHOT(8, 2, 1.0, 22) ONESHOT(16, 2, 1.0, 22)  // 80 KiB: 2 WGs per CU
        ONESHOT(16, 2, 1.0, 60)                          // 118 KiB: 1 WG per CU
        ONESHOT(16, 1, 1.0, 24) ONESHOT(8, 1, 1.0, 24)  // 53 KiB: 3 WGs per CU
        ONESHOT(16, 2, 0.6, 22) ONESHOT(16, 1, 0.6, 24)
        PERSIST(16, 2, 1.0, 2, 22) PERSIST(16, 1, 1.0, 3, 24)
    }
    if (which == 3) {
        // what the memory system penalises, on the 1-KiB tile of 8 waves (CPL=1) and CPL=2
        auto show = [&](const char *what) { printf("-- %s\n", what); };
        show("real layout");
        ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0)
        o.contig = 1; show("a tile's 80 rows contiguous"); ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0) o.contig = 0;
        o.copy = 0; show("no copy-through (parity only; TB/s over the full bytes)"); ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0) o.copy = 1;
        o.read = 0; show("no reads (TB/s over the full bytes)"); ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0)
        o.contig = 1; show("no reads, contiguous rows"); ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0) o.contig = 0; o.read = 1;
        o.order = 1; show("blocks dealt over segments"); ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0) o.order = 0;
        for (int64_t pad : {1024, 4096, 16384, 65536, 256 * 1024}) {
            o.pstride = PLEN + pad;
            printf("-- piece stride PLEN + %lld\n", (long long)pad);
            ONESHOT(8, 1, 0, 0) ONESHOT(8, 2, 0, 0)
        }
        o.pstride = PLEN;
    }
    return 0;
}
