// Developer experiment (not product), round 3: the RS(29,80) encode's memory
// shape, second sweep.  enc_shape_probe.hip showed the 80 piece streams'
// writes are the limit (write-only in that shape 5.6 TB/s, while round 1's
// wr_probe wrote the same streams at 6.0-6.45 TB/s in other groupings).
// Here the full read+write mix of the encode (no GF math) is run with:
//   CPL  tile width in KiB (16-B chunks per lane per share row)
//   MAP  0: share rows dealt to waves (wave w: rows w, w+NW, ..., every chunk)
//        1: (row, chunk) items dealt in row-major order (wave w: items
//           w, w+NW, ...): with CPL >= NW the waves of a workgroup write one
//           row's CPL KiB together, rows in sequence (a dense front)
//        2: as 0, the row order rotated per workgroup
//   POL  0: plain loads/stores, 1: non-temporal, 2: nt loads + plain stores
//   grid one workgroup per tile, or a persistent grid of WPC per CU
// The staged inputs go through LDS ([29][CPL][64 lanes] x 16 B); each parity
// chunk is the XOR of two staged chunks of its column (a data dependence on
// the tile, no GF arithmetic).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 enc_shape_probe2.hip -o enc_shape_probe2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

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

template <int POL>
__device__ __forceinline__ v4 ld(const uint8_t *p) {
    if constexpr (POL == 0) return *(const v4 *)p;
    else return __builtin_nontemporal_load((const v4 *)p);
}
template <int POL>
__device__ __forceinline__ void st(uint8_t *p, v4 v) {
    if constexpr (POL == 1) __builtin_nontemporal_store(v, (v4 *)p);
    else *(v4 *)p = v;
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// PAIR (CPL == 2): 0 the tile is 2 KiB of adjacent columns; 1 the second
// 1-KiB column block is half a segment further on; 2 it is the same block of
// segment + NSEG/2
template <int NW, int CPL, int MAP, int POL, int PAIR = 0>
__device__ __forceinline__ void do_tile(const uint8_t *in, uint8_t *out, int64_t tile, v4 *lds, int lane, int wave,
                                        int fake = 0) {
    constexpr int64_t TPS = CPS / (64 * CPL);
    constexpr int LI = K * CPL, SI = N * CPL;  // load items, store items of a tile
    constexpr int64_t NSEGP = PAIR == 2 ? NSEG / 2 : NSEG;
    (void)NSEGP;
    int64_t seg = tile / TPS, tt = tile - seg * TPS;
    if constexpr (PAIR == 2) seg = tile / (2 * TPS), tt = tile - seg * 2 * TPS;  // tiles of 1 KiB, half the segments
    const uint8_t *is = in + seg * SPAD;
    uint8_t *os = out + seg * (int64_t)N * PLEN;
    const int rot = MAP == 2 ? (int)((tile * 13) % N) : 0;
    // item m -> (row, chunk)
    auto item = [&](int m, int &row, int &c) {
        if constexpr (MAP == 1) {
            row = m / CPL;
            c = m - row * CPL;
        } else {
            // rows dealt to waves: the wave's i-th row is w + NW i, all its chunks
            const int per = m / NW, w = m - per * NW;  // m = w + NW * per
            const int rw = per / CPL;
            c = per - rw * CPL;
            row = w + NW * rw;
        }
    };
    // byte offsets of chunk c: in the segment's share row (qin + j*ESS) and in a piece (qo)
    auto qof = [&](int c) -> int64_t {
        if constexpr (PAIR == 0) return tt * 64 * CPL + c * 64 + lane;
        else if constexpr (PAIR == 1) return tt * 64 + c * (CPS / 2) + lane;  // TPS = half the 1-KiB blocks
        else return tt * 64 + lane;
    };
    auto segoff_in = [&](int c) -> int64_t { return PAIR == 2 ? c * (NSEG / 2) * SPAD : 0; };
    auto segoff_out = [&](int c) -> int64_t { return PAIR == 2 ? c * (NSEG / 2) * (int64_t)N * PLEN : 0; };
    constexpr int PL = (LI + NW - 1) / NW;
    v4 x[PL];
#pragma unroll
    for (int i = 0; i < PL; i++) {
        const int m = wave + NW * i;
        int j = 0, c = 0;
        item(m, j, c);
        if constexpr (MAP == 2) j = (j + rot) % K;
        if (m < LI && j < K) {
            const int64_t q = qof(c);
            x[i] = ld<POL == 1 ? 1 : (POL == 2 ? 1 : 0)>(is + segoff_in(c) + (q >> 4) * (K * ESS) + (q & 15) * 16 + j * ESS);
        }
    }
#pragma unroll
    for (int i = 0; i < PL; i++) {
        const int m = wave + NW * i;
        int j = 0, c = 0;
        item(m, j, c);
        if constexpr (MAP == 2) j = (j + rot) % K;
        if (m < LI && j < K) {
            st<POL>(os + segoff_out(c) + (int64_t)j * PLEN + qof(c) * 16, x[i]);
            lds[(j * CPL + c) * 64 + lane] = x[i];
        }
    }
    lds_barrier();
    uint32_t salt = 0;
    if (fake) {
        // emulated multiply: `fake` independent bitop3 per wave, fed from LDS
        v4 f = lds[(wave % (K * CPL)) * 64 + lane];
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
        salt = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    }
    constexpr int PS = (R * CPL + NW - 1) / NW;
#pragma unroll
    for (int i = 0; i < PS; i++) {
        const int m = wave + NW * i;
        int r = 0, c = 0;
        item(m, r, c);
        if (m < R * CPL && r < R) {
            if constexpr (MAP == 2) r = (r + rot) % R;
            v4 v = lds[((r % K) * CPL + c) * 64 + lane] ^ lds[(((r + 7) % K) * CPL + c) * 64 + lane];
            v.x ^= salt;
            st<POL>(os + segoff_out(c) + (int64_t)(K + r) * PLEN + qof(c) * 16, v);
        }
    }
}

template <int NW, int CPL, int MAP, int POL, int PAIR = 0>
__global__ __launch_bounds__(NW * 64) void enc_shape(const uint8_t *in, uint8_t *out, int64_t ntiles, int fake = 0) {
    extern __shared__ v4 lds[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        do_tile<NW, CPL, MAP, POL, PAIR>(in, out, t, lds, lane, wave, fake);
        lds_barrier();
    }
}

// The rebuild's shape: 29 piece streams in ([seg][80][PLEN], pieces 51..79),
// the stripe-major segment out; a tile is CPL x 1 KiB of columns of every
// share row (PAIR as above), share rows dealt to waves.
template <int NW, int CPL, int PAIR>
__global__ __launch_bounds__(NW * 64) void reb_shape(const uint8_t *pcs, uint8_t *segs, int64_t ntiles) {
    extern __shared__ v4 lds[];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int64_t TPS = CPS / (64 * CPL);
    const int64_t tile = blockIdx.x;
    int64_t seg = tile / TPS, tt = tile - seg * TPS;
    if constexpr (PAIR == 2) seg = tile / (2 * TPS), tt = tile - seg * 2 * TPS;
    auto qof = [&](int c) -> int64_t {
        if constexpr (PAIR == 0) return tt * 64 * CPL + c * 64 + lane;
        else if constexpr (PAIR == 1) return tt * 64 + c * (CPS / 2) + lane;
        else return tt * 64 + lane;
    };
    auto sg = [&](int c) -> int64_t { return PAIR == 2 ? seg + c * (NSEG / 2) : seg; };
    constexpr int PER = (K + NW - 1) / NW;
    v4 x[PER][CPL];
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < K)
#pragma unroll
            for (int c = 0; c < CPL; c++)
                x[i][c] = ld<1>(pcs + sg(c) * (int64_t)N * PLEN + (int64_t)(R + j) * PLEN + qof(c) * 16);
    }
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int j = wave + NW * i;
        if (j < K)
#pragma unroll
            for (int c = 0; c < CPL; c++) lds[(j * CPL + c) * 64 + lane] = x[i][c];
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < PER; i++) {
        const int r = wave + NW * i;
        if (r < K)
#pragma unroll
            for (int c = 0; c < CPL; c++) {
                const v4 v = lds[(r * CPL + c) * 64 + lane] ^ lds[(((r + 7) % K) * CPL + c) * 64 + lane];
                const int64_t q = qof(c);
                st<1>(segs + sg(c) * SPAD + (q >> 4) * (K * ESS) + (q & 15) * 16 + r * ESS, v);
            }
    }
}

// Persistent grid that takes its tiles from a work queue (one returning
// atomic add per tile, issued a tile ahead by lane 0 of wave 0 and handed over
// through LDS): the tiles in flight stay a dense window, as in a one-shot grid.
template <int NW, int PAIR>
__global__ __launch_bounds__(NW * 64) void enc_queue(const uint8_t *in, uint8_t *out, int64_t ntiles,
                                                     unsigned *ctr) {
    extern __shared__ v4 lds[];
    __shared__ int64_t s_next;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x == 0) s_next = atomicAdd(ctr, 1u);
    lds_barrier();
    int64_t cur = s_next;
    while (cur < ntiles) {
        unsigned nx = 0;
        if (threadIdx.x == 0) nx = atomicAdd(ctr, 1u);
        do_tile<NW, 2, 0, 1, PAIR>(in, out, cur, lds, lane, wave, 0);
        if (threadIdx.x == 0) s_next = nx;
        lds_barrier();
        cur = s_next;
        lds_barrier();
    }
}

// PROBE_RAND=1: buffers filled with pseudo-random bytes instead of a constant
// (the product's inputs are random; the round-3 logs before this option ran
// on memset data)
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
static bool g_rand = false;
static void fill(uint8_t *p, int64_t bytes, int c, uint32_t seed) {
    if (g_rand) hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, p, bytes / 16, seed);
    else (void)hipMemset(p, c, bytes);
    (void)hipDeviceSynchronize();
}

int main(int argc, char **argv) {
    g_rand = getenv("PROBE_RAND") && atoi(getenv("PROBE_RAND")) != 0;
    printf("data: %s\n", g_rand ? "pseudo-random" : "constant (memset)");
    uint8_t *in, *out;
    CK(hipMalloc(&in, SPAD * NSEG));
    const int64_t OUTB = (int64_t)N * PLEN * NSEG;
    CK(hipMalloc(&out, OUTB));
    fill(in, SPAD * NSEG, 0x5a, 1);
    fill(out, OUTB, 0x33, 2);
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)SPAD * NSEG * (1.0 + (double)N / K);
    auto timeit = [&](const char *name, auto launch) {
        for (int i = 0; i < 4; i++) launch();
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        const int it = 15;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-54s %8.1f us/launch %6.2f us/seg %6.3f TB/s\n", name, us, us / NSEG, bytes / us / 1e6);
        fflush(stdout);
    };
    // WPC = 0: one workgroup per tile; else a persistent grid of WPC workgroups per CU
#define V(NW, CPL, MAP, POL, WPC)                                                                                 \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / (64 * (CPL)));                                                \
        const size_t lb = (size_t)K * (CPL) * 1024;                                                             \
        const int64_t grid = (WPC) ? (int64_t)cus * (WPC) : nt;                                                 \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "NW=%d CPL=%d MAP=%d POL=%d %s%d", NW, CPL, MAP, POL, (WPC) ? "persist wg/cu=" : "oneshot", WPC); \
        timeit(nm, [&] {                                                                                        \
            hipLaunchKernelGGL((enc_shape<NW, CPL, MAP, POL>), dim3(grid), dim3((NW) * 64), lb, 0, in, out, nt); \
        });                                                                                                     \
    }
#define VP(NW, MAP, PAIR)                                                                                         \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / 128);                                                         \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "NW=%d CPL=2 MAP=%d POL=1 oneshot PAIR=%d", NW, MAP, PAIR);                    \
        timeit(nm, [&] {                                                                                        \
            hipLaunchKernelGGL((enc_shape<NW, 2, MAP, 1, PAIR>), dim3(nt), dim3((NW) * 64), (size_t)K * 2048, 0, in, out, nt); \
        });                                                                                                     \
    }
#define RB(NW, CPL, PAIR)                                                                                         \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / (64 * (CPL)));                                                \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "rebuild NW=%d CPL=%d PAIR=%d oneshot (TB/s of 2 S_pad)", NW, CPL, PAIR);      \
        const double save = bytes;                                                                              \
        (void)save;                                                                                             \
        timeit(nm, [&] {                                                                                        \
            hipLaunchKernelGGL((reb_shape<NW, CPL, PAIR>), dim3(nt), dim3((NW) * 64), (size_t)K * (CPL) * 1024, 0, out, in, nt); \
        });                                                                                                     \
    }
    // PAIR = 2 with the emulated multiply: FAKE = total wave-VALU per 2-KiB tile (the design's), LDSKB = dynamic
    // LDS per workgroup (caps workgroups per CU the way a real kernel's LDS or registers would)
#define VF(NW, PAIR, FAKE, LDSKB)                                                                                  \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / 128);                                                         \
        const int fk = ((FAKE) / (NW) + 7) / 8 * 8;                                                             \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "NW=%d PAIR=%d fake/wave=%d lds=%dK", NW, PAIR, fk, LDSKB);                     \
        timeit(nm, [&] {                                                                                        \
            hipLaunchKernelGGL((enc_shape<NW, 2, 0, 1, PAIR>), dim3(nt), dim3((NW) * 64), (size_t)(LDSKB) * 1024, 0, in, out, nt, fk); \
        });                                                                                                     \
    }
    unsigned *ctr = nullptr;
    CK(hipMalloc(&ctr, 4));
#define VQ(NW, PAIR, WPC)                                                                                          \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / 128);                                                         \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "queue NW=%d PAIR=%d wg/cu=%d", NW, PAIR, WPC);                                 \
        timeit(nm, [&] {                                                                                        \
            CK(hipMemsetAsync(ctr, 0, 4, 0));                                                                   \
            hipLaunchKernelGGL((enc_queue<NW, PAIR>), dim3(cus * (WPC)), dim3((NW) * 64), (size_t)K * 2048, 0, in, out, nt, ctr); \
        });                                                                                                     \
    }
#define VS(NW, PAIR, WPC)                                                                                          \
    {                                                                                                           \
        const int64_t nt = (int64_t)NSEG * (CPS / 128);                                                         \
        char nm[128];                                                                                           \
        snprintf(nm, sizeof nm, "static persistent NW=%d PAIR=%d wg/cu=%d", NW, PAIR, WPC);                     \
        timeit(nm, [&] {                                                                                        \
            hipLaunchKernelGGL((enc_shape<NW, 2, 0, 1, PAIR>), dim3(cus * (WPC)), dim3((NW) * 64), (size_t)K * 2048, 0, in, out, nt, 0); \
        });                                                                                                     \
    }
    const int which = argc > 1 ? atoi(argv[1]) : 0;
    if (which == 7) {
        // every variant on NA independent buffer sets (physical placement differs per allocation), round-robin
        constexpr int NA = 3;
        uint8_t *ins[NA], *outs[NA];
        ins[0] = in, outs[0] = out;
        for (int a = 1; a < NA; a++) {
            CK(hipMalloc(&ins[a], SPAD * NSEG + (a << 21)));
            CK(hipMalloc(&outs[a], OUTB + (a << 21)));
            ins[a] += (a << 21), outs[a] += (a << 21);  // a different 2-MiB phase, too
            fill(ins[a], SPAD * NSEG, 0x5a, 3 + a);
            fill(outs[a], OUTB, 0x33, 7 + a);
        }
        const int64_t nt2 = (int64_t)NSEG * (CPS / 128), nt1 = (int64_t)NSEG * (CPS / 64);
        struct Var {
            const char *name;
            std::function<void(const uint8_t *, uint8_t *)> f;
        };
        std::vector<Var> vars = {
            {"static persistent NW=8 CPL=2 PAIR=0 wg/cu=1 (round-2 pattern)",
             [&](const uint8_t *i, uint8_t *o) { hipLaunchKernelGGL((enc_shape<8, 2, 0, 1, 0>), dim3(cus), dim3(512), (size_t)K * 2048, 0, i, o, nt2, 0); }},
            {"oneshot NW=8 CPL=1",
             [&](const uint8_t *i, uint8_t *o) { hipLaunchKernelGGL((enc_shape<8, 1, 0, 1, 0>), dim3(nt1), dim3(512), (size_t)K * 1024, 0, i, o, nt1, 0); }},
            {"oneshot NW=16 CPL=2 PAIR=2",
             [&](const uint8_t *i, uint8_t *o) { hipLaunchKernelGGL((enc_shape<16, 2, 0, 1, 2>), dim3(nt2), dim3(1024), (size_t)K * 2048, 0, i, o, nt2, 0); }},
            {"oneshot NW=4 CPL=2 PAIR=2",
             [&](const uint8_t *i, uint8_t *o) { hipLaunchKernelGGL((enc_shape<4, 2, 0, 1, 2>), dim3(nt2), dim3(256), (size_t)K * 2048, 0, i, o, nt2, 0); }},
            {"oneshot NW=16 CPL=2 PAIR=0",
             [&](const uint8_t *i, uint8_t *o) { hipLaunchKernelGGL((enc_shape<16, 2, 0, 1, 0>), dim3(nt2), dim3(1024), (size_t)K * 2048, 0, i, o, nt2, 0); }},
            {"queue NW=16 PAIR=2 wg/cu=1",
             [&](const uint8_t *i, uint8_t *o) { CK(hipMemsetAsync(ctr, 0, 4, 0)); hipLaunchKernelGGL((enc_queue<16, 2>), dim3(cus), dim3(1024), (size_t)K * 2048, 0, i, o, nt2, ctr); }},
            {"queue NW=12 PAIR=2 wg/cu=1",
             [&](const uint8_t *i, uint8_t *o) { CK(hipMemsetAsync(ctr, 0, 4, 0)); hipLaunchKernelGGL((enc_queue<12, 2>), dim3(cus), dim3(768), (size_t)K * 2048, 0, i, o, nt2, ctr); }},
            {"queue NW=16 PAIR=0 wg/cu=2",
             [&](const uint8_t *i, uint8_t *o) { CK(hipMemsetAsync(ctr, 0, 4, 0)); hipLaunchKernelGGL((enc_queue<16, 0>), dim3(2 * cus), dim3(1024), (size_t)K * 2048, 0, i, o, nt2, ctr); }},
            {"queue NW=8 PAIR=2 wg/cu=2",
             [&](const uint8_t *i, uint8_t *o) { CK(hipMemsetAsync(ctr, 0, 4, 0)); hipLaunchKernelGGL((enc_queue<8, 2>), dim3(2 * cus), dim3(512), (size_t)K * 2048, 0, i, o, nt2, ctr); }},
            {"queue NW=4 PAIR=2 wg/cu=1",
             [&](const uint8_t *i, uint8_t *o) { CK(hipMemsetAsync(ctr, 0, 4, 0)); hipLaunchKernelGGL((enc_queue<4, 2>), dim3(cus), dim3(256), (size_t)K * 2048, 0, i, o, nt2, ctr); }},
        };
        std::vector<std::vector<double>> res(vars.size());
        for (int round = 0; round < 2; round++)
            for (int a = 0; a < NA; a++)
                for (size_t v = 0; v < vars.size(); v++) {
                    for (int w = 0; w < 3; w++) vars[v].f(ins[a], outs[a]);
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(e0));
                    for (int it = 0; it < 10; it++) vars[v].f(ins[a], outs[a]);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    res[v].push_back(bytes / (ms * 1e3 / 10) / 1e6);
                }
        for (size_t v = 0; v < vars.size(); v++) {
            double m = 0;
            printf("%-62s", vars[v].name);
            for (double x : res[v]) printf(" %5.2f", x), m += x;
            printf("  mean %5.3f TB/s\n", m / res[v].size());
        }
    }
    if (which == 6) {
        VF(16, 2, 0, 58) VF(4, 2, 0, 58)
        VS(16, 2, 1) VS(16, 2, 2) VS(4, 2, 1) VS(4, 2, 2) VS(8, 2, 1) VS(8, 2, 2)
        VQ(16, 2, 1) VQ(16, 2, 2) VQ(4, 2, 1) VQ(4, 2, 2) VQ(8, 2, 1) VQ(8, 2, 2) VQ(12, 2, 1) VQ(16, 0, 2) VQ(4, 0, 2)
        VF(16, 2, 0, 58) VF(4, 2, 0, 58)
    }
    if (which == 5) {
        // memory only, every workgroup width, natural occupancy
        VF(4, 2, 0, 58) VF(6, 2, 0, 58) VF(8, 2, 0, 58) VF(12, 2, 0, 58) VF(16, 2, 0, 58) VF(16, 1, 0, 58) VF(4, 1, 0, 58)
        // one workgroup per CU (LDS 100K) and two (LDS 58K or 80K)
        VF(4, 2, 0, 100) VF(8, 2, 0, 100) VF(16, 2, 0, 100) VF(8, 2, 0, 80) VF(16, 2, 0, 80)
        // with the multiply: 18.3 k wave-VALU per tile (4 row groups) and 26 k (16 row groups)
        VF(4, 2, 18300, 58) VF(4, 2, 18300, 80) VF(16, 2, 26000, 58) VF(16, 2, 26000, 100) VF(16, 2, 21000, 58)
        VF(12, 2, 23000, 58) VF(8, 2, 21000, 58) VF(6, 2, 20000, 58) VF(6, 2, 20000, 80)
        VF(4, 2, 0, 58) VF(16, 2, 0, 58)
    }
    if (which == 4) {
        // rebuild shapes; TB/s printed over the encode's bytes: x 2/(1+80/29) = 0.532 for the rebuild's
        RB(8, 1, 0) RB(4, 1, 0) RB(16, 1, 0) RB(2, 2, 0) RB(3, 2, 0) RB(4, 2, 0) RB(8, 2, 0) RB(4, 2, 1) RB(8, 2, 1)
        RB(4, 2, 2) RB(8, 2, 2) RB(4, 4, 0)
    }
    if (which == 3) {
        V(8, 1, 0, 1, 0) VP(8, 0, 0) VP(8, 0, 1) VP(8, 0, 2) VP(16, 0, 1) VP(16, 0, 2) VP(8, 1, 1) VP(8, 1, 2)
        VP(4, 0, 1) VP(4, 0, 2) V(8, 1, 0, 1, 0)
    }
    if (which == 0 || which == 1) {
        // store policy and row rotation on the round's best shape
        V(8, 1, 0, 0, 0) V(8, 1, 0, 1, 0) V(8, 1, 0, 2, 0) V(8, 1, 2, 1, 0)
        // dense per-workgroup fronts: every wave writes its chunk of the same row
        V(4, 4, 1, 1, 0) V(8, 4, 1, 1, 0) V(16, 4, 1, 1, 0) V(4, 4, 1, 0, 0) V(8, 4, 1, 0, 0)
        V(4, 2, 1, 1, 0) V(8, 2, 1, 1, 0) V(16, 2, 1, 1, 0) V(8, 2, 1, 0, 0)
        V(16, 1, 1, 1, 0) V(8, 1, 1, 1, 0)
    }
    if (which == 0 || which == 2) {
        // persistent grids of the same shapes
        V(8, 1, 0, 1, 4) V(8, 1, 1, 1, 4) V(8, 2, 1, 1, 2) V(16, 2, 1, 1, 2) V(8, 4, 1, 1, 1) V(16, 4, 1, 1, 1)
        V(8, 2, 1, 0, 2) V(16, 4, 1, 0, 1)
    }
    return 0;
}
