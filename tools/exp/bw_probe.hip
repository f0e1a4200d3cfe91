// Developer experiment (not product): HBM ceilings on this MI355X for the
// read:write mixes of the erasure kernels, with the simplest streaming shapes
// (one or a few 16-B chunks per thread, grid covering the whole buffer, no
// grid-stride loop) next to hipMemcpy D2D.  The encode moves 1 read byte per
// 80/29 = 2.76 written; the rebuild 1:1; the parity-only encode 1 : 51/29.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bw_probe.hip -o bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef uint32_t v4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4 ld(const v4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4 *p, v4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// each thread: R reads of consecutive 1 KiB wave blocks, W writes (the XOR of
// what it read, plus w); thread blocks tile the buffers densely.  n = number
// of 16-B chunks of the read buffer; writes cover (W/R) x that.
template <int R, int W, bool NT>
__global__ __launch_bounds__(256) void mix(const v4 *in, v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    v4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t i = (wave * R + r) * 64 + lane;
        if (i < n) acc ^= ld<NT>(in + i);
    }
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int64_t i = (wave * W + w) * 64 + lane;
        if (i < n / R * W) st<NT>(out + i, acc ^ (uint32_t)w);
    }
}

// read-only (sum kept live by a data-dependent store that never happens)
template <int R, bool NT>
__global__ __launch_bounds__(256) void rd(const v4 *in, v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    v4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t i = (wave * R + r) * 64 + lane;
        if (i < n) acc ^= ld<NT>(in + i);
    }
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) out[0] = acc;
}

// write-only: W stores of consecutive 1 KiB wave blocks per thread
template <int W, bool NT>
__global__ __launch_bounds__(256) void wr(v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int64_t i = (wave * W + w) * 64 + lane;
        if (i < n) st<NT>(out + i, v4{(uint32_t)i, (uint32_t)w, 1u, 2u});
    }
}

// the same with the blocks interleaved over all waves: store w of every wave
// lands in one dense front (block w * total_waves + wave)
template <int W>
__global__ __launch_bounds__(256) void wr_il(v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t tw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int64_t i = (w * tw + wave) * 64 + lane;
        if (i < n) st<true>(out + i, v4{(uint32_t)i, (uint32_t)w, 1u, 2u});
    }
}
template <int R, int W>
__global__ __launch_bounds__(256) void mix_il(const v4 *in, v4 *out, int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t tw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    v4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t i = (r * tw + wave) * 64 + lane;
        if (i < n) acc ^= ld<true>(in + i);
    }
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int64_t i = (w * tw + wave) * 64 + lane;
        if (i < n / R * W) st<true>(out + i, acc ^ (uint32_t)w);
    }
}

// persistent form: one workgroup of WPC waves per CU, each wave loops over
// blocks of R read / W written 1 KiB wave-chunks (the data-piece stores of
// the encode go out as their loads land, then the W - R parity stores).
template <int R, int W, bool NT>
__global__ void loop_mix(const v4 *in, v4 *out, int64_t nblk) {
    const int lane = threadIdx.x & 63;
    const int64_t G = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nblk; b += G) {
        v4 x[R];
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = ld<NT>(in + (b * R + r) * 64 + lane);
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc ^= x[r];
            st<NT>(out + (b * W + r) * 64 + lane, x[r]);
        }
#pragma unroll
        for (int w = R; w < W; w++) st<NT>(out + (b * W + w) * 64 + lane, acc ^ (uint32_t)w);
    }
}

template <int T>
__device__ __forceinline__ void wait_vm() {
    if constexpr (T >= 0) __builtin_amdgcn_s_waitcnt((T & 15) | ((T >> 4) << 14) | (7 << 4) | (15 << 8));
}

// the encode's own output shape: block b reads R KiB of the segment and
// writes 1 KiB into each of W piece streams (pitch = nblk KiB); with T >= 0
// a wave waits after each store until at most T of its stores are in flight.
template <int R, int W, int T>
__global__ void loop_pieces(const v4 *in, v4 *out, int64_t nblk) {
    const int lane = threadIdx.x & 63;
    const int64_t G = (int64_t)gridDim.x * (blockDim.x >> 6);
    for (int64_t b = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < nblk; b += G) {
        v4 x[R];
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = ld<true>(in + (b * R + r) * 64 + lane);
        v4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < R; r++) {
            acc ^= x[r];
            st<true>(out + (r * nblk + b) * 64 + lane, x[r]);
        }
#pragma unroll
        for (int w = R; w < W; w++) {
            st<true>(out + (w * nblk + b) * 64 + lane, acc ^ (uint32_t)w);
            wait_vm<T>();
        }
    }
}

// copy with 256-B runs on one side, as the rebuild (pieces -> stripe-major
// segment: RUNW) or the encode (segment -> pieces: RUNR) move data: a wave
// instruction covers 4 runs of 256 B at a 7424-B stride (29 shares x 256 B).
template <int R, bool RUNR, bool RUNW>
__global__ __launch_bounds__(256) void runcopy(const uint8_t *in, uint8_t *out, int64_t nwaves, int64_t plen) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (wave >= nwaves) return;
    // wave -> (group of 4 stripes g, share-row block) ; R consecutive rows
    const int64_t rows_blocks = 29 / R;
    const int64_t g = wave / rows_blocks, rb = wave - g * rows_blocks;
    const int s = lane >> 4, t = (lane & 15) * 16;
    v4 x[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t row = rb * R + r;
        const int64_t off = RUNR ? ((g * 4 + s) * 7424 + row * 256 + t) : (row * plen + g * 1024 + lane * 16);
        x[r] = ld<true>((const v4 *)(in + off));
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int64_t row = rb * R + r;
        const int64_t off = RUNW ? ((g * 4 + s) * 7424 + row * 256 + t) : (row * plen + g * 1024 + lane * 16);
        st<true>((v4 *)(out + off), x[r]);
    }
}

int main() {
    const int64_t RB = (int64_t)1 << 30;  // 1 GiB read buffer
    const int64_t WB = (int64_t)3 << 30;  // 3 GiB write buffer
    v4 *A, *B;
    CK(hipMalloc(&A, RB));
    CK(hipMalloc(&B, WB));
    CK(hipMemset(A, 0x5a, RB));
    CK(hipMemset(B, 0x33, WB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, double bytes, auto launch) {
        for (int i = 0; i < 5; i++) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int i = 0; i < it; i++) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        printf("%-44s %9.1f us  %6.3f TB/s\n", name, us, bytes / us / 1e6);
        fflush(stdout);
    };
    timeit("hipMemcpy D2D 1 GiB", 2.0 * RB, [&] { CK(hipMemcpyAsync(B, A, RB, hipMemcpyDeviceToDevice, 0)); });
    const int64_t n = RB / 16;
#define MIX(R, W, NT)                                                                                          \
    {                                                                                                          \
        const int64_t waves = n / 64 / (R);                                                                    \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "mix R=%d W=%d nt=%d (w:r %.2f)", R, W, NT, (double)(W) / (R));                \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                               \
            hipLaunchKernelGGL((mix<R, W, NT>), dim3((waves + 3) / 4), dim3(256), 0, 0, A, B, n);              \
        });                                                                                                    \
    }
#define RD(R, NT)                                                                                              \
    {                                                                                                          \
        const int64_t waves = n / 64 / (R);                                                                    \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "read R=%d nt=%d", R, NT);                                                     \
        timeit(nm, (double)RB, [&] {                                                                           \
            hipLaunchKernelGGL((rd<R, NT>), dim3((waves + 3) / 4), dim3(256), 0, 0, A, B, n);                 \
        });                                                                                                    \
    }
    RD(1, 0) RD(4, 0) RD(4, 1) RD(16, 1)
    MIX(1, 1, 0) MIX(1, 1, 1) MIX(4, 4, 0) MIX(4, 4, 1)
    MIX(29, 80, 1) MIX(29, 80, 0) MIX(4, 11, 1) MIX(1, 3, 1) MIX(1, 3, 0)
    MIX(29, 51, 1) MIX(4, 7, 1)
#define WR(W, NT)                                                                                              \
    {                                                                                                          \
        const int64_t wn = WB / 16, waves = wn / 64 / (W);                                                     \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "write-only W=%d nt=%d (3 GiB)", W, NT);                                       \
        timeit(nm, (double)WB, [&] { hipLaunchKernelGGL((wr<W, NT>), dim3((waves + 3) / 4), dim3(256), 0, 0, B, wn); }); \
    }
    WR(1, 0) WR(1, 1) WR(4, 1) WR(16, 1)
#define WRIL(W)                                                                                                \
    {                                                                                                          \
        const int64_t wn = WB / 16, waves = wn / 64 / (W);                                                     \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "write-only interleaved W=%d (3 GiB)", W);                                     \
        timeit(nm, (double)WB, [&] { hipLaunchKernelGGL((wr_il<W>), dim3((waves + 3) / 4), dim3(256), 0, 0, B, wn); }); \
    }
    WRIL(4) WRIL(16)
#define MIXIL(R, W)                                                                                            \
    {                                                                                                          \
        const int64_t waves = n / 64 / (R);                                                                    \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "mix interleaved R=%d W=%d (w:r %.2f)", R, W, (double)(W) / (R));              \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                               \
            hipLaunchKernelGGL((mix_il<R, W>), dim3((waves + 3) / 4), dim3(256), 0, 0, A, B, n);               \
        });                                                                                                    \
    }
    MIXIL(4, 11) MIXIL(29, 80) MIXIL(29, 51) MIXIL(4, 4)
    timeit("hipMemsetAsync 3 GiB", (double)WB, [&] { CK(hipMemsetAsync(B, 0x11, WB, 0)); });

#define LOOP(R, W, WPC)                                                                                        \
    {                                                                                                          \
        const int64_t nblk = n / 64 / (R);                                                                     \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "loop R=%d W=%d waves/CU=%d", R, W, WPC);                                      \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                               \
            hipLaunchKernelGGL((loop_mix<R, W, true>), dim3(cus), dim3(64 * (WPC)), 0, 0, A, B, nblk);        \
        });                                                                                                    \
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    LOOP(1, 3, 4) LOOP(1, 3, 8) LOOP(1, 3, 16)
    LOOP(2, 6, 4) LOOP(2, 6, 8) LOOP(2, 6, 16)
    LOOP(4, 11, 4) LOOP(4, 11, 8) LOOP(4, 11, 16)
    LOOP(8, 22, 4) LOOP(8, 22, 8) LOOP(8, 22, 16)
    LOOP(29, 80, 2) LOOP(29, 80, 4) LOOP(29, 80, 8)
    LOOP(1, 2, 16) LOOP(2, 4, 16) LOOP(29, 51, 4) LOOP(29, 51, 8)

#define PIECES(R, W, T, WPC)                                                                                   \
    {                                                                                                          \
        const int64_t nblk = n / 64 / (R);                                                                     \
        char nm[96];                                                                                           \
        snprintf(nm, sizeof nm, "pieces R=%d W=%d throttle=%d waves/CU=%d", R, W, T, WPC);                     \
        timeit(nm, (double)RB * (1.0 + (double)(W) / (R)), [&] {                                               \
            hipLaunchKernelGGL((loop_pieces<R, W, T>), dim3(cus), dim3(64 * (WPC)), 0, 0, A, B, nblk);        \
        });                                                                                                    \
    }
    PIECES(29, 80, -1, 2) PIECES(29, 80, -1, 4) PIECES(29, 80, 4, 4) PIECES(29, 80, 8, 4) PIECES(29, 80, 16, 4)
    PIECES(29, 80, 4, 8) PIECES(29, 80, 8, 8) PIECES(29, 80, 2, 8) PIECES(29, 80, 4, 16) PIECES(29, 80, 8, 16)
    PIECES(29, 51, -1, 4) PIECES(29, 51, 4, 8) PIECES(29, 51, 8, 8)

    {
        // 1024*1024 groups of 4 stripes would be 30 GB; use 9040*16/4 groups = 16 x 64 MiB segments
        const int64_t groups = 9040LL * 15 / 4;
        const double bytes = 2.0 * groups * 4 * 7424;
#define RC(R, RR, RW)                                                                                          \
        {                                                                                                      \
            const int64_t nw = groups * (29 / (R));                                                            \
            char nm[96];                                                                                       \
            snprintf(nm, sizeof nm, "runcopy R=%d runs_read=%d runs_write=%d", R, RR, RW);                     \
            timeit(nm, bytes * (double)((29 / (R)) * (R)) / 29.0, [&] {                                        \
                hipLaunchKernelGGL((runcopy<R, RR, RW>), dim3((nw + 3) / 4), dim3(256), 0, 0, (const uint8_t *)A, \
                                   (uint8_t *)B, nw, groups * 1024);                                                          \
            });                                                                                                \
        }
        RC(1, false, false) RC(1, false, true) RC(1, true, false) RC(29, false, true) RC(29, true, false)
    }
    return 0;
}
