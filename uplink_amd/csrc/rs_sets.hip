// Rebuild / Decode of segments that each bring their own share set, in one
// stream-ordered pass (rs_sets.hpp).  Reference: the per-segment Rebuild of
// StripeReader (private/eestream/stripe.go:382-428), each download's own share
// set (stripe.go:314-354, private/ecclient/client.go:273-308).
//
//  rs_sets_prep: one workgroup per segment.  G is the Lagrange basis on the
//      points x_0 = 0, x_i = alpha^(i-1) (G[i][j] = L_j(x_i), gf256_field.hpp),
//      so the inverse of the k rows of the basis shares S -- what infectious
//      Rebuild inverts per stripe -- is interpolation through S's points: data
//      d = sum over s in S of share_s * L^S_s(x_d), and a share u (Decode's
//      syndrome rows) is predicted the same way at x_u.  In closed form,
//          L^S_s(y) = N(y) / ((y - x_s) W_s),  N(y) = prod_t (y - x_t),
//          W_s = prod_{t != s} (x_s - x_t),
//      i.e. sums of logarithms and one exp per coefficient: independent table
//      lookups, no elimination (a Gauss-Jordan in LDS measured ~60 us per
//      segment, the lookups a few).  The inverse is unique, so the bytes are
//      those of the k x k inversion (tests: against the oracle's, which
//      inverts).  Then the rows' jump-table leaf addresses, in the layout
//      rs_matmul_sets reads ([pass][input][group][8], rows right-aligned per
//      group).
//  rs_matmul_sets<NW>: rs_matmul_dma<NW, 1, false> (rs_kernels.hip) with the
//      per-launch matrix replaced by the tile's segment descriptor: input
//      pointers, copy-through and row offsets, leaf table; one workgroup per
//      2048-column tile, LDS-DMA staging one chunk ahead, the jump-table body.
#include <hip/hip_runtime.h>

#include "../../include/uplink_ec.h"
#include "gf256_field.hpp"
#include "rs_device.hpp"
#include "rs_kernels.hpp"
#include "rs_sets.hpp"

namespace uplink_ec {
namespace {

using namespace dev;

__constant__ GfTables c_gf = make_gf_tables();

constexpr int kRows = 8;  // accumulator rows per wave (jt_inputs)

__device__ __forceinline__ void rows_of(int pass, int npass, int nout, int nw, int g, int &rbase, int &cnt) {
    const int p0 = pass * nout / npass, prow = (pass + 1) * nout / npass - p0;
    rbase = p0 + g * prow / nw;
    cnt = p0 + (g + 1) * prow / nw - rbase;
}

__device__ __forceinline__ int npass_of(int nout, int nw) { return nout > 0 ? (nout + nw * kRows - 1) / (nw * kRows) : 1; }

// One segment's decode rows, solved and written as leaf addresses by one
// workgroup (rs_sets_prep).
__device__ __forceinline__ void solve_rows(const SetStage *st, uint64_t jt_base) {
    __shared__ uint8_t s_exp[512], s_log[256];
    __shared__ uint8_t s_x[kMaxOps];                    // basis points x_p
    __shared__ uint8_t s_y[2 * kMaxOps];                // row points y_r
    __shared__ int16_t s_lw[kMaxOps];                   // log W_p
    __shared__ int16_t s_ln[2 * kMaxOps], s_hit[2 * kMaxOps];  // log N_r, or the basis position row r sits on
    __shared__ int s_num[kMaxOps], s_miss[kMaxOps];
    __shared__ int s_acc[kMaxOps + 2 * kMaxOps];  // the sums of logarithms of W_p, then of N_r
    __shared__ int s_hdr[8];
    __shared__ uint64_t *s_tgt;
    const int tid = threadIdx.x, nt = (int)blockDim.x;
    for (int i = tid; i < kMaxOps; i += nt) {
        s_num[i] = st->num[i];
        s_miss[i] = st->missing[i];
    }
    if (tid == 0) s_hdr[0] = st->d.nin;
    if (tid == 1) s_hdr[1] = st->d.nout;
    if (tid == 2) s_hdr[2] = st->d.nstore;
    if (tid == 3) s_hdr[3] = st->nw;
    if (tid == 4) s_hdr[4] = st->k;
    if (tid == 5) s_tgt = st->d.tgt;
    for (int i = tid; i < 512; i += nt) s_exp[i] = c_gf.exp[i];
    for (int i = tid; i < 256; i += nt) s_log[i] = c_gf.log[i];
    __syncthreads();
    const int nin = s_hdr[0], nout = s_hdr[1], nstore = s_hdr[2], nw = s_hdr[3], k = s_hdr[4];
    auto point = [&](int num) -> uint8_t { return num == 0 ? 0 : s_exp[(num - 1) % 255]; };
    for (int i = tid; i < k; i += nt) s_x[i] = point(s_num[i]);
    // row r's point: a missing data position (its data index), or a non-basis share (a syndrome row)
    for (int i = tid; i < nout; i += nt) s_y[i] = point(i < nstore ? s_miss[i] : s_num[k + i - nstore]);
    // log W_p = sum over t != p of log(x_p ^ x_t) (the points are distinct: the host checked), and
    // log N_r = sum over t of log(y_r ^ x_t), a row whose point is a basis point being that share
    // itself: (k + nout) x k independent terms, spread over the workgroup and added in LDS
    // (one term per thread and step instead of a k-long chain per sum: 13 -> ~5 us per launch)
    for (int i = tid; i < k; i += nt) s_acc[i] = 0;
    for (int i = tid; i < nout; i += nt) {
        s_acc[kMaxOps + i] = 0;
        s_hit[i] = -1;
    }
    __syncthreads();
    for (int e = tid; e < (k + nout) * k; e += nt) {
        const int a = e / k, t = e - a * k;
        if (a < k) {
            if (t != a) atomicAdd(&s_acc[a], (int)s_log[s_x[a] ^ s_x[t]]);
        } else {
            const uint8_t d = s_y[a - k] ^ s_x[t];
            if (d) atomicAdd(&s_acc[kMaxOps + a - k], (int)s_log[d]);
            else s_hit[a - k] = (int16_t)t;
        }
    }
    __syncthreads();
    for (int i = tid; i < k; i += nt) s_lw[i] = (int16_t)(s_acc[i] % 255);
    for (int i = tid; i < nout; i += nt) s_ln[i] = (int16_t)(s_acc[kMaxOps + i] % 255);
    __syncthreads();
    // leaf addresses: coefficient of basis input j in row r is N_r / ((y_r ^ x_j) W_j) (Lagrange
    // interpolation through the basis points, evaluated at y_r); 1 on a non-basis input's own
    // syndrome row; else 0
    const int npass = npass_of(nout, nw), per_pass = nin * nw * kRows;
    uint64_t *tgt = s_tgt;
    for (int e = tid; e < npass * per_pass; e += nt) {
        const int pass = e / per_pass, rem = e - pass * per_pass;
        const int j = rem / (nw * kRows), g = (rem / kRows) % nw, o = rem % kRows;
        int rb, cn;
        rows_of(pass, npass, nout, nw, g, rb, cn);
        const int oo = o - (kRows - cn);
        uint32_t c = 0;
        if (oo >= 0) {
            const int r = rb + oo;
            if (j >= k) {
                c = (uint32_t)(r >= nstore && j - k == r - nstore);
            } else if (s_hit[r] >= 0) {
                c = (uint32_t)(s_hit[r] == j);
            } else {
                const int l = s_ln[r] - s_log[s_y[r] ^ s_x[j]] - s_lw[j];
                c = s_exp[((l % 255) + 255) % 255];
            }
        }
        tgt[e] = jt_base + (uint64_t)c * RS_JT_SLOT;
    }
}

__device__ __forceinline__ void prep_one(const SetStage *st, SetDesc *dd, uint64_t jt_base, uint32_t *done_ctr) {
    const int tid = threadIdx.x;
    // the descriptor from the host's staging at once (one round trip over the bus, or the
    // kernel's arguments)
    {
        const uint64_t *src = (const uint64_t *)&st->d;
        uint64_t *dst = (uint64_t *)dd;
        for (int i = tid; i < (int)(sizeof(SetDesc) / 8); i += blockDim.x) dst[i] = src[i];
    }
    if (tid == 6) {
        uint32_t *zc = st->d.zero_check;
        if (zc) *zc = 0u;
    }
    if (tid == 7 && blockIdx.x == 0 && done_ctr) *done_ctr = 0u;
    solve_rows(st, jt_base);
}

__global__ __launch_bounds__(256) void rs_sets_prep(const SetStage *stage, SetDesc *desc, uint64_t jt_base,
                                                    uint32_t *done_ctr) {
    prep_one(stage + blockIdx.x, desc + blockIdx.x, jt_base, done_ctr);
}

// One segment: its record passed as the kernel's argument (3.1 KB of the 4 KB a
// launch carries), so the prep reads nothing over the bus
__global__ __launch_bounds__(256) void rs_sets_prep1(const SetStage stage, SetDesc *desc, uint64_t jt_base,
                                                     uint32_t *done_ctr) {
    prep_one(&stage, desc, jt_base, done_ctr);
}

// checked build: every access of the tile stays inside its share / segment (one
// outside is skipped and its site recorded, as rs_tile.hpp in_range does)
__device__ __forceinline__ bool in_span(const SetsArgs &a, const uint8_t *p, const uint8_t *lo, int64_t len, int site) {
#ifdef UPLINK_EC_CHECKED
    if (p >= lo && p + 16 <= lo + len) return true;
    if (a.chk_flag) atomicCAS(a.chk_flag, 0u, (uint32_t)site);
    return false;
#else
    (void)a, (void)p, (void)lo, (void)len, (void)site;
    return true;
#endif
}

// The descriptors are read through the constant address space: the kernel never
// writes them, and uniform loads from there are scalar loads (SGPR operands,
// the K$) -- the jump-table body needs its leaf-table address in SGPRs.
typedef const __attribute__((address_space(4))) SetDesc ConstDesc;

typedef const __attribute__((address_space(4))) SetOne ConstOne;

// One tile of a share-set pass; D: ConstDesc (the segment's descriptor in
// device memory, its leaf table made by rs_sets_prep) or ConstOne (one segment,
// rs_sets_one: the record is the launch's arguments, and the workgroup writes
// the leaf table from the host's coefficients while its first chunk's loads
// are in flight -- every workgroup the same bytes -- and reads it back with
// scalar loads once its own stores are complete).
template <int NW, class D>
__device__ __forceinline__ void sets_tile(const SetsArgs &a, D *d) {
    constexpr bool ONE = __is_same(D, ConstOne);
    constexpr int JC = 2 * NW, PER = 2, OPW = kRows, SLOT = JC * 2048;
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    u32x4 *ring = (u32x4 *)smem;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int group = (wave + (int)(blockIdx.x % NW)) % NW;
    const uint32_t ring_addr = (uint32_t)(uintptr_t)smem;
    const int64_t tile = blockIdx.x;
    const int64_t seg = ONE ? 0 : tile / a.tiles_per_seg;
    const int nin = d->nin, nout = d->nout;
    const int64_t piece_len = a.nstripes * a.ess, spad = piece_len * a.k;
    if (d->status == 0 && nin > 0) {
        // the tile's two chunks of 16 byte columns per lane (rs_tile.hpp tile_cols)
        const int64_t qA = (tile - seg * a.tiles_per_seg) * kTileChunks + lane, qB = qA + 64;
        const bool vA = qA < a.chunks_per_seg, vB = qB < a.chunks_per_seg;
        const uint32_t cps = (uint32_t)a.cps;
        const uint32_t sA = (uint32_t)qA / cps, tA = (uint32_t)qA - sA * cps;
        const uint32_t sB = (uint32_t)qB / cps, tB = (uint32_t)qB - sB * cps;
        // a lane past the end of the segment reads column 0 (never stored)
        const int64_t iA = vA ? (int64_t)sA * a.ess + tA * 16 : 0, iB = vB ? (int64_t)sB * a.ess + tB * 16 : 0;
        const int64_t oA = (int64_t)sA * a.k * a.ess + tA * 16, oB = (int64_t)sB * a.k * a.ess + tB * 16;
        const int nchunks = (nin + JC - 1) / JC;
        const int CH = (nin + nchunks - 1) / nchunks;
        const int npass = npass_of(nout, NW);
        auto owned = [&](int ch) -> int {
            const int jn = nin - ch * CH < CH ? nin - ch * CH : CH;
            return wave < jn ? (jn - wave + NW - 1) / NW : 0;
        };
        auto issue = [&](int ch) {
            const uint32_t d0 = ring_addr + (uint32_t)((ch & 1) * SLOT);
#pragma unroll
            for (int i = 0; i < PER; i++) {
                const int j = wave + NW * i;
                if (i < owned(ch)) {
                    const uint8_t *p = d->in[ch * CH + j];
                    const uint8_t *pa = p + iA, *pb = p + iB;
                    if (!in_span(a, pa, p, piece_len, 8)) pa = p;
                    if (!in_span(a, pb, p, piece_len, 8)) pb = p;
                    const uint32_t dst = __builtin_amdgcn_readfirstlane(d0 + (uint32_t)(j * 2048));
                    dma_1k(pa, dst);
                    dma_1k(pb, dst + 1024);
                }
            }
        };
        uint8_t *out = d->out;
        if constexpr (ONE) {
            // Every workgroup writes the whole table, the same bytes, and reads it only after its
            // own stores are complete: the chunk's vmcnt(0) below waits for them with the loads,
            // before the barrier every wave passes ahead of its first scalar load of the table.
            // Whichever copy a read meets -- this XCD's L2 line, or the scalar cache's, filled by
            // a workgroup that had itself finished writing -- holds these bytes; the scalar cache
            // starts the launch empty, so nothing is left from the slot's previous call.
            issue(0);
            uint64_t *t = d->tgt;
            for (int e = threadIdx.x; e < npass * nin * NW * OPW; e += NW * 64) {
                const int pass = e / (nin * NW * OPW), rem = e - pass * (nin * NW * OPW);
                const int j = rem / (NW * OPW), g = (rem / OPW) % NW, o = rem % OPW;
                int rb, cn;
                rows_of(pass, npass, nout, NW, g, rb, cn);
                const int oo = o - (OPW - cn);
                const uint32_t c = oo >= 0 ? d->coef[(rb + oo) * nin + j] : 0u;
                t[e] = a.jt_base + (uint64_t)c * RS_JT_SLOT;
            }
        }
        for (int pass = 0; pass < npass; pass++) {
            int rbase, cnt;
            rows_of(pass, npass, nout, NW, group, rbase, cnt);
            if (!ONE || pass > 0) issue(0);
            u32x8 acc[OPW];
#pragma unroll
            for (int o = 0; o < OPW; o++) acc[o] = (u32x8){0, 0, 0, 0, 0, 0, 0, 0};
            for (int ch = 0; ch < nchunks; ch++) {
                wait_vm(0);
                const int j0 = ch * CH;
                u32x4 *slot = ring + (ch & 1) * (SLOT / 16);
#pragma unroll
                for (int i = 0; i < PER; i++) {
                    const int j = wave + NW * i;
                    if (i < owned(ch)) {
                        const u32x4 A4 = slot[j * 128 + lane], B4 = slot[j * 128 + 64 + lane];
                        const int co = d->copy_off[j0 + j];
                        if (pass == 0 && co >= 0) {
                            uint8_t *p = out + co;
                            if (vA && in_span(a, p + oA, out, spad, 9)) st16<true>(p + oA, A4.x, A4.y, A4.z, A4.w);
                            if (vB && in_span(a, p + oB, out, spad, 9)) st16<true>(p + oB, B4.x, B4.y, B4.z, B4.w);
                        }
                        uint32_t w[8] = {A4.x, A4.y, A4.z, A4.w, B4.x, B4.y, B4.z, B4.w};
                        bitslice8(w);
                        // in place, in the wide layout jt_inputs reads (a lane's planes where its bytes were)
                        slot[j * 128 + lane] = (u32x4){w[0], w[1], w[2], w[3]};
                        slot[j * 128 + 64 + lane] = (u32x4){w[4], w[5], w[6], w[7]};
                    }
                }
                lds_barrier();
                if (ch + 1 < nchunks) issue(ch + 1);
                if (cnt > 0) {
                    const int jn = nin - j0 < CH ? nin - j0 : CH;
                    jt_inputs(acc, ring_addr + (uint32_t)((ch & 1) * SLOT) + (uint32_t)lane * 16,
                              d->tgt + ((pass * nin + j0) * NW + group) * OPW, (uint32_t)(NW * OPW * 8),
                              (uint32_t)(OPW - cnt), (uint32_t)jn);
                }
            }
            uint32_t rows[OPW][8];
#pragma unroll
            for (int o = 0; o < OPW; o++)
#pragma unroll
                for (int p = 0; p < 8; p++) rows[o][p] = acc[o][p];
            uint32_t *zc = d->zero_check;
            const int nst = zc ? d->nstore : rbase + cnt;
            if (zc) {
                uint32_t any = 0;
#pragma unroll
                for (int o = 0; o < OPW; o++)
                    if (o < cnt && rbase + o >= nst)
#pragma unroll
                        for (int p = 0; p < 8; p++) any |= rows[o][p];
                any &= (vA ? 0x0F0F0F0Fu : 0u) | (vB ? 0xF0F0F0F0u : 0u);
                if (__ballot(any != 0) != 0 && lane == 0) atomicAdd(zc, 1u);
            }
            static_for<OPW>([&]<int O>() {
                if (O < cnt && rbase + O < nst) {
                    uint32_t w[8];
#pragma unroll
                    for (int p = 0; p < 8; p++) w[p] = rows[O][p];
                    unbitslice8(w);
                    uint8_t *p = out + d->out_off[rbase + O];
                    if (vA && in_span(a, p + oA, out, spad, 9)) st16<true>(p + oA, w[0], w[1], w[2], w[3]);
                    if (vB && in_span(a, p + oB, out, spad, 9)) st16<true>(p + oB, w[4], w[5], w[6], w[7]);
                }
            });
            // the slot the next pass's first DMAs go to may still be read by a wave's multiply
            lds_barrier();
        }
    }
    // every wave of this workgroup has read all it reads from the slot (descriptor,
    // leaf table) once it is past this barrier (no wait for the stores in flight)
    if (a.done_ctr) {
        lds_barrier();
        if (threadIdx.x == 0) {
            const uint32_t old = atomicAdd(a.done_ctr, 1u);
            if (old + 1 == a.total_wgs) {
                atomicExch(a.done_ctr, 0u);
                __hip_atomic_store(a.host_done, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

template <int NW>
__global__ __launch_bounds__(NW * 64, 4) void rs_matmul_sets(const SetsArgs a) {
    sets_tile<NW>(a, (ConstDesc *)(a.desc + blockIdx.x / a.tiles_per_seg));
}

template <int NW>
__global__ __launch_bounds__(NW * 64, 4) void rs_sets_one(const SetOne p) {
    sets_tile<NW>(p.a, (ConstOne *)&p);
}

}  // namespace

// as the straight-line split (rs_sl_codegen.cpp split_for): 15-16 rows on 3 waves, not 2 -- one
// share set of 15 rows, 32 segments: 794-848 against 821-866 us on 2 waves, 815-834 on 4
// (profiles/r05/r/); the 14-24-row mix of fresh sets on 4 waves instead of 3: 874-882 against
// 855-857 us, one segment 73.5 against 62-64 us wall (profiles/r05/q/)
int sets_waves(int rows) { return rows <= 14 ? 2 : rows <= 24 ? 3 : 4; }

int64_t sets_max_tiles(int nw) { return (int64_t)(0xFFFFFFFFu / (unsigned)(nw * 64)); }

size_t sets_tgt_entries(int nin, int rows, int nw) {
    const int npass = rows > 0 ? (rows + nw * kRows - 1) / (nw * kRows) : 1;
    return (size_t)npass * nin * nw * kRows;
}

hipError_t launch_sets_prep(const SetStage *stage, SetDesc *desc, int nseg, uint64_t jt_base, uint32_t *done_ctr,
                            hipStream_t s) {
    if (nseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(rs_sets_prep, dim3(nseg), dim3(256), 0, s, stage, desc, jt_base, done_ctr);
    return hipGetLastError();
}

hipError_t launch_sets_prep1(const SetStage &stage, SetDesc *desc, uint64_t jt_base, uint32_t *done_ctr,
                             hipStream_t s) {
    hipLaunchKernelGGL(rs_sets_prep1, dim3(1), dim3(256), 0, s, stage, desc, jt_base, done_ctr);
    return hipGetLastError();
}

hipError_t launch_sets_one(const SetOne &p, int nw, hipStream_t s) {
    if (p.a.total_tiles <= 0) return hipSuccess;
    if (p.a.total_tiles > sets_max_tiles(nw) || p.nin > kOneMaxIn || p.nin * p.nout > kOneMaxCoef)
        return hipErrorInvalidValue;
    const dim3 grid((unsigned)p.a.total_tiles);
    switch (nw) {
    case 2: hipLaunchKernelGGL(rs_sets_one<2>, grid, dim3(2 * 64), (size_t)2 * 4 * 2048, s, p); break;
    case 3: hipLaunchKernelGGL(rs_sets_one<3>, grid, dim3(3 * 64), (size_t)2 * 6 * 2048, s, p); break;
    case 4: hipLaunchKernelGGL(rs_sets_one<4>, grid, dim3(4 * 64), (size_t)2 * 8 * 2048, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_matmul_sets(const SetsArgs &a, int nw, hipStream_t s) {
    if (a.total_tiles <= 0) return hipSuccess;
    if (a.total_tiles > sets_max_tiles(nw)) return hipErrorInvalidValue;  // one workgroup per tile
    const dim3 grid((unsigned)a.total_tiles);
    switch (nw) {
    case 2: hipLaunchKernelGGL(rs_matmul_sets<2>, grid, dim3(2 * 64), (size_t)2 * 4 * 2048, s, a); break;
    case 3: hipLaunchKernelGGL(rs_matmul_sets<3>, grid, dim3(3 * 64), (size_t)2 * 6 * 2048, s, a); break;
    case 4: hipLaunchKernelGGL(rs_matmul_sets<4>, grid, dim3(4 * 64), (size_t)2 * 8 * 2048, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace uplink_ec
