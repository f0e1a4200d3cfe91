// Error detection / correction for ErasureScheme.Decode (rsScheme.Decode,
// private/eestream/rs.go:32-38 -> infectious FEC.Decode = Correct + Rebuild;
// used when StripeReader runs with error detection, stripe.go:407-408).
//
//  rs_flag_columns: a byte column is a codeword iff every share beyond the
//      first k equals its re-encoding from those k (the caller computes the
//      re-encoding with the stripe matmul kernel); flags the others.
//  rs_berlekamp_welch: one workgroup per flagged column solves the
//      Berlekamp-Welch system on the points x_0 = 0, x_r = alpha^(r-1) with
//      e = (r-k)/2 (Gauss-Jordan, free unknowns set to zero), divides Q by E
//      and rewrites the column with the corrected codeword.  Status per
//      column: 0, -6 (NotEnoughShares: e <= 0) or -7 (TooManyErrors).
//  rs_flag_rows / rs_put_rows: the fast path of ec_decode when the errors sit
//      in a few shares (a bad piece): check the other shares against each
//      other, and rewrite the bad shares from them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf256_field.hpp"
#include "rs_correct.hpp"

namespace uplink_ec {
namespace {

__constant__ GfTables c_gf = make_gf_tables();

__device__ __forceinline__ uint8_t dmul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : c_gf.exp[c_gf.log[a] + c_gf.log[b]];
}
__device__ __forceinline__ uint8_t dpow(uint8_t x, int e) {
    uint8_t r = 1;
    for (int i = 0; i < e; i++) r = dmul(r, x);
    return r;
}
__device__ __forceinline__ uint8_t dpoint(int num) { return num == 0 ? 0 : c_gf.exp[(num - 1) % 255]; }

// shares: ns rows of len bytes (row stride `stride`), expected: (ns-k) rows
__global__ void rs_flag_columns(const uint8_t *shares, int64_t stride, const uint8_t *expected, int64_t estride,
                                int k, int ns, int64_t len, uint8_t *flags) {
    for (int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; col < len;
         col += (int64_t)gridDim.x * blockDim.x) {
        uint8_t bad = 0;
        for (int r = 0; r < ns - k; r++) bad |= (uint8_t)(shares[(int64_t)(k + r) * stride + col] != expected[(int64_t)r * estride + col]);
        flags[col] = bad;
    }
}

// rows[0..nrows) of shares against expected rows 0..nrows-1: flag the columns that differ
__global__ void rs_flag_rows(const uint8_t *shares, int64_t stride, const int *rows, int nrows,
                             const uint8_t *expected, int64_t estride, int64_t len, uint8_t *flags) {
    for (int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; col < len;
         col += (int64_t)gridDim.x * blockDim.x) {
        uint8_t bad = 0;
        for (int r = 0; r < nrows; r++)
            bad |= (uint8_t)(shares[(int64_t)rows[r] * stride + col] != expected[(int64_t)r * estride + col]);
        flags[col] = bad;
    }
}

// shares[rows[r]][col] = expected[r][col] where !skip[col]
__global__ void rs_put_rows(uint8_t *shares, int64_t stride, const int *rows, int nrows, const uint8_t *expected,
                            int64_t estride, int64_t len, const uint8_t *skip) {
    for (int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; col < len;
         col += (int64_t)gridDim.x * blockDim.x) {
        if (skip[col]) continue;
        for (int r = 0; r < nrows; r++) shares[(int64_t)rows[r] * stride + col] = expected[(int64_t)r * estride + col];
    }
}

// kMaxDim: the largest system the instantiation solves (k + 2e <= shares given):
// 128, and 256 for wide codes given more than 128 shares (n up to 256; its LDS
// -- 66 KB -- leaves a CU two such workgroups, so it is launched only for those)
template <int kMaxDim>
__global__ __launch_bounds__(64) void rs_berlekamp_welch(uint8_t *shares, int64_t stride, int64_t len,
                                                         const int *nums, int k, int n, int ns, const int64_t *cols,
                                                         int ncols, int *status, uint8_t *changed) {
    __shared__ uint8_t A[kMaxDim][kMaxDim + 1];
    __shared__ uint8_t f[kMaxDim];
    __shared__ uint8_t u[kMaxDim];
    __shared__ int pivcol[kMaxDim];
    __shared__ int s_row, s_piv;
    const int tid = threadIdx.x;
    for (int ci = blockIdx.x; ci < ncols; ci += gridDim.x) {
        const int64_t col = cols[ci];
        if (col < 0 || col >= len) {  // host-supplied column list: never index outside the shares
            if (tid == 0) status[ci] = -10;
            continue;
        }
        const int e = (ns - k) / 2;
        if (e <= 0) {
            if (tid == 0) status[ci] = -6;
            continue;
        }
        const int q = e + k;
        const int dim = q + e;
        if (dim > kMaxDim) {
            if (tid == 0) status[ci] = -12;
            continue;
        }
        for (int i = tid; i < dim; i += blockDim.x) {
            const uint8_t x = dpoint(nums[i]);
            const uint8_t ri = shares[(int64_t)i * stride + col];
            f[i] = dmul(dpow(x, e), ri);
            uint8_t xp = 1;
            for (int j = 0; j < q; j++) {
                A[i][j] = xp;
                xp = dmul(xp, x);
            }
            xp = 1;
            for (int t = 0; t < e; t++) {
                A[i][q + t] = dmul(xp, ri);
                xp = dmul(xp, x);
            }
        }
        if (tid == 0) s_row = 0;
        __syncthreads();
        for (int c = 0; c < dim; c++) {
            const int row = s_row;
            if (row >= dim) break;
            if (tid == 0) {
                int p = -1;
                for (int r = row; r < dim; r++)
                    if (A[r][c]) { p = r; break; }
                s_piv = p;
            }
            __syncthreads();
            const int p = s_piv;
            if (p >= 0) {
                if (p != row) {
                    for (int j = tid; j < dim; j += blockDim.x) {
                        uint8_t t = A[p][j]; A[p][j] = A[row][j]; A[row][j] = t;
                    }
                    if (tid == 0) { uint8_t t = f[p]; f[p] = f[row]; f[row] = t; }
                }
                __syncthreads();
                const uint8_t iv = c_gf.inv[A[row][c]];
                __syncthreads();
                for (int j = tid; j < dim; j += blockDim.x) A[row][j] = dmul(iv, A[row][j]);
                if (tid == 0) f[row] = dmul(iv, f[row]);
                __syncthreads();
                for (int r = tid; r < dim; r += blockDim.x) {
                    if (r == row) continue;
                    const uint8_t fac = A[r][c];
                    if (!fac) continue;
                    for (int j = 0; j < dim; j++) A[r][j] ^= dmul(fac, A[row][j]);
                    f[r] ^= dmul(fac, f[row]);
                }
                if (tid == 0) { pivcol[row] = c; s_row = row + 1; }
            }
            __syncthreads();
        }
        if (tid == 0) {
            const int rows = s_row;
            int fail = 0;
            for (int r = rows; r < dim; r++) if (f[r]) fail = 1;
            for (int j = 0; j < dim; j++) u[j] = 0;
            for (int r = 0; r < rows; r++) u[pivcol[r]] = f[r];
            uint8_t rem[2 * kMaxDim], E[kMaxDim + 1], P[kMaxDim];
            for (int j = 0; j < 2 * kMaxDim; j++) rem[j] = 0;
            for (int j = 0; j < q; j++) rem[j] = u[j];
            for (int t = 0; t < e; t++) E[t] = u[q + t];
            E[e] = 1;
            for (int j = 0; j < k; j++) P[j] = 0;
            for (int d = q - 1; d >= e; d--) {
                const uint8_t co = rem[d];
                if (!co) continue;
                P[d - e] = co;
                for (int t = 0; t <= e; t++) rem[d - e + t] ^= dmul(co, E[t]);
            }
            for (int d = 0; d < e; d++) if (rem[d]) fail = 1;
            if (!fail) {
                for (int i = 0; i < ns; i++) {
                    const uint8_t x = dpoint(nums[i]);
                    uint8_t acc = 0;
                    for (int d = k - 1; d >= 0; d--) acc = dmul(acc, x) ^ P[d];
                    if (changed) changed[(int64_t)ci * ns + i] = shares[(int64_t)i * stride + col] != acc;
                    shares[(int64_t)i * stride + col] = acc;
                }
            }
            status[ci] = fail ? -7 : 0;
            (void)n;
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_flag_columns(const uint8_t *shares, int64_t stride, const uint8_t *expected, int64_t estride, int k,
                               int ns, int64_t len, uint8_t *flags, hipStream_t s) {
    int64_t blocks = (len + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(rs_flag_columns, dim3((unsigned)blocks), dim3(256), 0, s, shares, stride, expected, estride, k,
                       ns, len, flags);
    return hipGetLastError();
}

hipError_t launch_berlekamp_welch(uint8_t *shares, int64_t stride, int64_t len, const int *nums, int k, int n, int ns,
                                  const int64_t *cols, int ncols, int *status, hipStream_t s, uint8_t *changed) {
    int blocks = ncols < 2048 ? ncols : 2048;
    if (blocks < 1) return hipSuccess;
    const int e = (ns - k) / 2;
    if (k + 2 * e <= 128)
        hipLaunchKernelGGL(rs_berlekamp_welch<128>, dim3(blocks), dim3(64), 0, s, shares, stride, len, nums, k, n, ns,
                           cols, ncols, status, changed);
    else
        hipLaunchKernelGGL(rs_berlekamp_welch<256>, dim3(blocks), dim3(64), 0, s, shares, stride, len, nums, k, n, ns,
                           cols, ncols, status, changed);
    return hipGetLastError();
}

static int64_t col_blocks(int64_t len) {
    int64_t b = (len + 255) / 256;
    return b > 4096 ? 4096 : (b < 1 ? 1 : b);
}

hipError_t launch_flag_rows(const uint8_t *shares, int64_t stride, const int *rows, int nrows, const uint8_t *expected,
                            int64_t estride, int64_t len, uint8_t *flags, hipStream_t s) {
    hipLaunchKernelGGL(rs_flag_rows, dim3((unsigned)col_blocks(len)), dim3(256), 0, s, shares, stride, rows, nrows,
                       expected, estride, len, flags);
    return hipGetLastError();
}

hipError_t launch_put_rows(uint8_t *shares, int64_t stride, const int *rows, int nrows, const uint8_t *expected,
                           int64_t estride, int64_t len, const uint8_t *skip, hipStream_t s) {
    hipLaunchKernelGGL(rs_put_rows, dim3((unsigned)col_blocks(len)), dim3(256), 0, s, shares, stride, rows, nrows,
                       expected, estride, len, skip);
    return hipGetLastError();
}

}  // namespace uplink_ec
