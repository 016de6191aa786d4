// tci_device.hip -- gfx950 kernels around the rrLU of tci_rrlu.hip: MatrixLUCI factors (matrixluci.jl:161-283), batch evaluation of
// the integrand catalog (batcheval.jl:131-175 + util.jl:34-43), the site-tensor solve
// (tensorci2.jl:620-627) and the synthetic-input generator.
// Compiled with -ffp-contract=off: no multiply-add is fused unless written as such.
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "tci_funcdev.h"
#include "tci_internal.h"

namespace tci {

static constexpr int32_t kBig = 0x7fffffff;

static int grid_for(long long work, int cap) {
    long long g = (work + 255) / 256;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

// -------------------------------------------------------- MatrixLUCI factors
// Inputs: position-order L (m x np, ld ldl) and U (np x n, ld ldu) with the reference's
// diagonals (L unit if leftorth, U unit otherwise).
// leftorth: left = colstimespivotinv (matrixluci.jl:194-213): rows >= np solve X L11 = L21 in
// place (one thread per row, back substitution over columns), then scatter by rowperm.
__global__ void k_trsm_rows_lower(double* __restrict__ L, int64_t ldl, int m, int np) {
    const int i = np + blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    for (int j = np - 1; j >= 0; --j) {
        double s = L[i + (int64_t)j * ldl];
        for (int t = j + 1; t < np; ++t)
            s = __dsub_rn(s, __dmul_rn(L[i + (int64_t)t * ldl], L[t + (int64_t)j * ldl]));
        L[i + (int64_t)j * ldl] = s;  // L11[j,j] == 1
    }
}

// !leftorth: right = pivotinvtimesrows (matrixluci.jl:227-241): columns >= np solve
// U11 x = U[:, c] in place (unit diagonal), one thread per column.
__global__ void k_trsm_cols_upper(double* __restrict__ U, int64_t ldu, int n, int np) {
    const int c = np + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    double* col = U + (int64_t)c * ldu;
    for (int a = np - 1; a >= 0; --a) {
        double s = col[a];
        for (int t = a + 1; t < np; ++t) s = __dsub_rn(s, __dmul_rn(U[a + (int64_t)t * ldu], col[t]));
        col[a] = s;
    }
}

// Blocked form of both triangular solves for np <= kTrsmMaxNp: a workgroup keeps RHS
// right-hand sides (rows of L21 / columns of U12) x np in LDS (RHS = 32 up to np = 512, then 16
// and 8, so that RHS x np doubles stay within 128 KiB) and walks 16-column blocks from the
// right: solve the block's unit-triangular diagonal part per right-hand side, then subtract the
// block's contribution from every column to its left in parallel (right-looking). Same
// recurrence X[., j] = B[., j] - sum_{t > j} X[., t] coef(t, j) as the one-thread-per-row
// kernels, in block order.
//   LOWER (leftorth): X(r, j) = L[r + j ld], coef(t, j) = L[t + j ld]
//   upper (!leftorth): X(c, j) = U[j + c ld], coef(t, j) = U[j + t ld]
constexpr int kTrsmBlk = 16;
constexpr int kTrsmMaxNp = 2048;

template <bool LOWER, int kTrsmRhs>
__global__ __launch_bounds__(256) void k_trsm_blocked(double* __restrict__ Mx, int64_t ld, int rhs0,
                                                      int rhs1, int np) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* Xs = reinterpret_cast<double*>(smem);  // [j][r], r fastest
    const int r0 = rhs0 + blockIdx.x * kTrsmRhs;
    const int nr = min(kTrsmRhs, rhs1 - r0);
    auto X = [&](int r, int j) -> double& {
        return LOWER ? Mx[(int64_t)(r0 + r) + (int64_t)j * ld] : Mx[(int64_t)j + (int64_t)(r0 + r) * ld];
    };
    auto coef = [&](int t, int j) -> double {
        return LOWER ? Mx[(int64_t)t + (int64_t)j * ld] : Mx[(int64_t)j + (int64_t)t * ld];
    };
    for (int e = threadIdx.x; e < kTrsmRhs * np; e += blockDim.x) {
        const int r = e % kTrsmRhs, j = e / kTrsmRhs;
        Xs[e] = r < nr ? X(r, j) : 0.0;
    }
    __syncthreads();
    for (int jb = ((np - 1) / kTrsmBlk) * kTrsmBlk; jb >= 0; jb -= kTrsmBlk) {
        const int je = min(jb + kTrsmBlk, np);
        if (threadIdx.x < kTrsmRhs) {
            const int r = threadIdx.x;
            for (int j = je - 1; j >= jb; --j) {
                double s = Xs[j * kTrsmRhs + r];
                for (int t = j + 1; t < je; ++t)
                    s = __dsub_rn(s, __dmul_rn(Xs[t * kTrsmRhs + r], coef(t, j)));
                Xs[j * kTrsmRhs + r] = s;
            }
        }
        __syncthreads();
        for (int e = threadIdx.x; e < kTrsmRhs * jb; e += blockDim.x) {
            const int r = e % kTrsmRhs, j = e / kTrsmRhs;
            double s = Xs[e];
            for (int t = jb; t < je; ++t) s = __dsub_rn(s, __dmul_rn(Xs[t * kTrsmRhs + r], coef(t, j)));
            Xs[e] = s;
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < kTrsmRhs * np; e += blockDim.x) {
        const int r = e % kTrsmRhs, j = e / kTrsmRhs;
        if (r < nr) X(r, j) = Xs[e];
    }
}

template <bool LOWER>
static void launch_trsm(hipStream_t s, double* Mx, int64_t ld, int rhs0, int rhs1, int np) {
    if (rhs1 <= rhs0) return;
    if (np > kTrsmMaxNp) {
        if (LOWER)
            hipLaunchKernelGGL(k_trsm_rows_lower, dim3((rhs1 - rhs0 + 127) / 128), dim3(128), 0, s, Mx, ld,
                               rhs1, np);
        else
            hipLaunchKernelGGL(k_trsm_cols_upper, dim3((rhs1 - rhs0 + 127) / 128), dim3(128), 0, s, Mx, ld,
                               rhs1, np);
        return;
    }
    auto go = [&](auto kern, int rhs) {
        const size_t bytes = (size_t)rhs * np * sizeof(double);
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes);
        hipLaunchKernelGGL(kern, dim3((rhs1 - rhs0 + rhs - 1) / rhs), dim3(256), bytes, s, Mx, ld, rhs0, rhs1, np);
    };
    if (np <= 512)
        go(k_trsm_blocked<LOWER, 32>, 32);
    else if (np <= 1024)
        go(k_trsm_blocked<LOWER, 16>, 16);
    else
        go(k_trsm_blocked<LOWER, 8>, 8);
}

// left (m x np, ld m) scatter for leftorth: out[rowperm[i], j] = i < np ? (i==j) : X[i,j]
__global__ void k_left_scatter_lo(const double* __restrict__ L, int64_t ldl, int m, int np,
                                  const int64_t* __restrict__ rowperm, double* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)m * np; e += stride) {
        const int i = (int)(e % m), j = (int)(e / m);
        const double v = (i < np) ? (i == j ? 1.0 : 0.0) : L[i + (int64_t)j * ldl];
        out[rowperm[i] + (int64_t)j * m] = v;
    }
}

// right (np x n, ld np) for leftorth: rowmatrix = L11 * U, column-scattered (matrixluci.jl:175)
__global__ void k_right_gemm_lo(const double* __restrict__ L, int64_t ldl,
                                const double* __restrict__ U, int64_t ldu, int n, int np,
                                const int64_t* __restrict__ colperm, double* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)np * n; e += stride) {
        const int a = (int)(e % np), j = (int)(e / np);
        double s = 0.0;
        const int tmax = a < j ? a : j;  // L11[a,t] = 0 for t > a; U[t,j] = 0 for t > j
        for (int t = 0; t <= tmax; ++t)
            s = __dadd_rn(s, __dmul_rn(L[a + (int64_t)t * ldl], U[t + (int64_t)j * ldu]));
        out[a + colperm[j] * (int64_t)np] = s;
    }
}

// left (m x np) for !leftorth: colmatrix = left(lu) * U11 (matrixluci.jl:161-165)
__global__ void k_left_gemm_ro(const double* __restrict__ L, int64_t ldl,
                               const double* __restrict__ U, int64_t ldu, int m, int np,
                               const int64_t* __restrict__ rowperm, double* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)m * np; e += stride) {
        const int i = (int)(e % m), j = (int)(e / m);
        double s = 0.0;
        const int tmax = i < j ? i : j;  // L[i,t] = 0 for t > i; U11[t,j] = 0 for t > j
        for (int t = 0; t <= tmax; ++t)
            s = __dadd_rn(s, __dmul_rn(L[i + (int64_t)t * ldl], U[t + (int64_t)j * ldu]));
        out[rowperm[i] + (int64_t)j * m] = s;
    }
}

// right (np x n) scatter for !leftorth: out[a, colperm[j]] = j < np ? (a==j) : X[a,j]
__global__ void k_right_scatter_ro(const double* __restrict__ U, int64_t ldu, int n, int np,
                                   const int64_t* __restrict__ colperm, double* __restrict__ out) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)np * n; e += stride) {
        const int a = (int)(e % np), j = (int)(e / np);
        const double v = (j < np) ? (a == j ? 1.0 : 0.0) : U[a + (int64_t)j * ldu];
        out[a + colperm[j] * (int64_t)np] = v;
    }
}


void trsm_luci_left(hipStream_t s, double* L, int64_t ldl, int m, int np);
void trsm_luci_right(hipStream_t s, double* U, int64_t ldu, int n, int np);

void launch_luci_factors(hipStream_t s, double* L, int64_t ldl, double* U, int64_t ldu, int m,
                         int n, int np, int leftorth, const int64_t* rowperm,
                         const int64_t* colperm, double* left, double* right, int dense) {
    if (np <= 0) return;
    const bool mf = dense & kDenseLuci;
    if (leftorth) {
        // right first: it reads the untouched L11; the TRSM then overwrites L21 in place
        if (right) {
            if (mf)  // rowmatrix = L11 * U (K = np), columns scattered by colperm
                launch_dgemm(s, false, np, n, np, 1.0, L, ldl, U, ldu, 0.0, nullptr, 0, right, np, nullptr,
                             colperm);
            else
                hipLaunchKernelGGL(k_right_gemm_lo, dim3(grid_for((long long)np * n, 8192)), dim3(256),
                                   0, s, L, ldl, U, ldu, n, np, colperm, right);
        }
        if (left) {
            if (mf) trsm_luci_left(s, L, ldl, m, np);
            else launch_trsm<true>(s, L, ldl, np, m, np);
            hipLaunchKernelGGL(k_left_scatter_lo, dim3(grid_for((long long)m * np, 8192)), dim3(256),
                               0, s, L, ldl, m, np, rowperm, left);
        }
    } else {
        if (left) {
            if (mf)  // colmatrix = L * U11 (K = np), rows scattered by rowperm
                launch_dgemm(s, false, m, np, np, 1.0, L, ldl, U, ldu, 0.0, nullptr, 0, left, m, rowperm,
                             nullptr);
            else
                hipLaunchKernelGGL(k_left_gemm_ro, dim3(grid_for((long long)m * np, 8192)), dim3(256), 0,
                                   s, L, ldl, U, ldu, m, np, rowperm, left);
        }
        if (right) {
            if (mf) trsm_luci_right(s, U, ldu, n, np);
            else launch_trsm<false>(s, U, ldu, np, n, np);
            hipLaunchKernelGGL(k_right_scatter_ro, dim3(grid_for((long long)np * n, 8192)),
                               dim3(256), 0, s, U, ldu, n, np, colperm, right);
        }
    }
}

// ---------------------------------------------------------- synthetic fill
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void k_fill_uniform(double* A, int64_t m, int64_t n, int64_t lda, uint64_t seed, uint64_t offset) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const uint64_t base = seed * 0xD1B54A32D192ED03ull + offset;
    for (int64_t e = gid; e < m * n; e += stride) {
        const int64_t i = e % m, j = e / m;
        A[i + j * lda] = (double)(splitmix64(base + (uint64_t)e) >> 11) * 0x1.0p-53;
    }
}

// Diagnostic: stream-read roofline calibration (max |a| over n doubles, 16-B loads).
__global__ __launch_bounds__(256) void k_stream_read(const double2* __restrict__ a, int64_t n2,
                                                     unsigned long long* out) {
    double mx = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; e + 7 * stride < n2; e += 8 * stride) {  // 8 independent 16-B loads in flight
        double2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = a[e + u * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) mx = fmax(mx, fmax(fabs(v[u].x), fabs(v[u].y)));
    }
    for (; e < n2; e += stride) {
        const double2 v = a[e];
        mx = fmax(mx, fmax(fabs(v.x), fabs(v.y)));
    }
    for (int off = 32; off >= 1; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(mx));
}

// Diagnostic: stream-copy roofline calibration (b = a, 16-B loads and stores).
__global__ __launch_bounds__(256) void k_stream_copy(const double2* __restrict__ a,
                                                     double2* __restrict__ b, int64_t n2) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; e + 7 * stride < n2; e += 8 * stride) {
        double2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = a[e + u * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) b[e + u * stride] = v[u];
    }
    for (; e < n2; e += stride) b[e] = a[e];
}

void launch_stream_read(hipStream_t s, const double* a, int64_t n, unsigned long long* out, int grid) {
    hipLaunchKernelGGL(k_stream_read, dim3(grid > 0 ? grid : grid_for(n / 2, 2048)), dim3(256), 0, s,
                       reinterpret_cast<const double2*>(a), n / 2, out);
}

void launch_stream_copy(hipStream_t s, const double* a, double* b, int64_t n, int grid) {
    hipLaunchKernelGGL(k_stream_copy, dim3(grid > 0 ? grid : grid_for(n / 2, 2048)), dim3(256), 0, s,
                       reinterpret_cast<const double2*>(a), reinterpret_cast<double2*>(b), n / 2);
}

void launch_fill_uniform(hipStream_t s, double* A, int64_t m, int64_t n, int64_t lda,
                         uint64_t seed, uint64_t offset) {
    hipLaunchKernelGGL(k_fill_uniform, dim3(grid_for(m * n, 8192)), dim3(256), 0, s, A, m, n, lda,
                       seed, offset);
}

// --------------------------------------------------------- batch evaluation
// _batchevaluate_dispatch (batcheval.jl:131-175) for the integrand catalog. Catalog kinds whose
// value depends on the left/right parts only through an exactly combinable summary (an integer
// sum, an integer bit index, a table offset, a partial sum of squares) run in two stages:
// per-row and per-column "state" (O((m+n)L)), then one pass that combines and writes
// Pi[R + ldo*j] -- an HBM-write-bound stream. Other kinds evaluate directly per element.
// the kinds, St, leg_state() and combine<KIND>(): tci_funcdev.h

// Row states: R in [0, m*D); i = R % m, c = R / m (centre index, only for M == 1); column states
// per j; the row states, the column states and the Lorentzian quotient table in ONE launch (block ranges
// [0, gr) rows, [gr, gr + gc) columns, then the table): the three are independent, and as three
// launches their ~4 us each of launch latency was ~12 % of an 8192^2 Pi's device time
__global__ void k_state_prep(FuncDev f, const int32_t* __restrict__ I, int m, int nl, int M, int D,
                             St* __restrict__ rs, int gr, const int32_t* __restrict__ J, int n, int nr,
                             int toff, St* __restrict__ cs, int gc, double* __restrict__ tab, int64_t ntab) {
    const int b = (int)blockIdx.x;
    if (b < gr) {
        for (int64_t R = (int64_t)b * blockDim.x + threadIdx.x; R < (int64_t)m * D; R += (int64_t)gr * blockDim.x) {
            const int i = (int)(R % m), c = (int)(R / m);
            rs[R] = leg_state(f, I + (int64_t)i * nl, nl, 0, M ? c + 1 : 0);
        }
    } else if (b < gr + gc) {
        for (int64_t j = (int64_t)(b - gr) * blockDim.x + threadIdx.x; j < n; j += (int64_t)gc * blockDim.x)
            cs[j] = leg_state(f, J + j * nr, nr, toff, 0);
    } else {
        const double p0 = f.params[0];
        const int gt = (int)gridDim.x - gr - gc;
        for (int64_t s = (int64_t)(b - gr - gc) * blockDim.x + threadIdx.x; s < ntab; s += (int64_t)gt * blockDim.x)
            tab[s] = p0 / (double)(s + 1);
    }
}

__device__ __forceinline__ void block_maxabs(double v, unsigned long long* maxbits) {
    // |v| bit patterns order like the values for non-negative doubles, and +NaN sorts above
    // +Inf, so an unsigned max over the bits is Julia's NaN-propagating max (util.jl:34-43).
    unsigned long long b = (unsigned long long)__double_as_longlong(fabs(v));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off);
        b = o > b ? o : b;
    }
    __shared__ unsigned long long sb[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) sb[w] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < (int)(blockDim.x >> 6); ++q) b = sb[q] > b ? sb[q] : b;
        atomicMax(maxbits, b);
    }
}

// Stage 2: out[R + ldo*j]. A tile is 512 rows (2 per lane: one 16-B store when ldo is even) x
// kAsmCols columns; a lane loads its two row states once per tile.
constexpr int kAsmCols = 8;

template <int KIND>
__global__ __launch_bounds__(256) void k_assemble(FuncDev f, const St* __restrict__ rs,
                                                  const St* __restrict__ cs, int64_t mR, int n,
                                                  int nr, double* __restrict__ out, int64_t ldo,
                                                  unsigned long long* maxbits, const double* __restrict__ tab,
                                                  int64_t ntab, int vec) {
    const double* p = f.params;
    const double p0 = (KIND == F_SUM || KIND == F_TABLE) ? 0.0 : p[0];
    double mx = 0.0;
    const int64_t rtiles = (mR + 511) / 512;
    const int64_t ntiles = rtiles * ((n + kAsmCols - 1) / kAsmCols);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t R = (t % rtiles) * 512 + 2 * threadIdx.x;
        const int j0 = (int)(t / rtiles) * kAsmCols;
        const bool h0 = R < mR, h1 = R + 1 < mR;
        if (!h0) continue;
        St r0 = rs[R], r1;
        r1.i = 0;
        if (h1) r1 = rs[R + 1];
        const int je = min(j0 + kAsmCols, n);
        for (int j = j0; j < je; ++j) {
            const St c = cs[j];
            const double v0 = combine<KIND>(p, p0, r0, c, nr, f.L, tab, ntab);
            double* o = out + R + ldo * j;
            const double a0 = fabs(v0);
            mx = (isnan(a0) || a0 > mx) ? a0 : mx;
            if (h1) {
                const double v1 = combine<KIND>(p, p0, r1, c, nr, f.L, tab, ntab);
                const double a1 = fabs(v1);
                mx = (isnan(a1) || a1 > mx) ? a1 : mx;
                if (vec) {
                    *reinterpret_cast<double2*>(o) = double2{v0, v1};
                } else {
                    o[0] = v0;
                    o[1] = v1;
                }
            } else {
                o[0] = v0;
            }
        }
    }
    block_maxabs(mx, maxbits);
}

// The Lorentzian (README.md:21-29) at HBM write speed: out[R + ldo j] = tab[s_R + s_j], the
// quotient table p0 / (s + 1) over every reachable integer sum of squares (bitwise the division,
// DESIGN.md K1) staged in LDS when it fits (a gather from L1/L2 per element otherwise). A tile is
// 512 rows (two per lane, one 16-B non-temporal store) x kLzCols columns, the column states read as
// wave-uniform (scalar) loads, all the tile's table reads issued before its stores.
constexpr int kLzCols = 16;
constexpr int kLzTabLds = 8192;  // table entries staged in LDS (64 KiB)
template <bool LDS>
__global__ __launch_bounds__(256) void k_assemble_lorentz(const St* __restrict__ rs, const St* __restrict__ cs,
                                                          int64_t mR, int n, double* __restrict__ out, int64_t ldo,
                                                          unsigned long long* maxbits, const double* __restrict__ tab,
                                                          int64_t ntab, double p0, int vec) {
    __shared__ double ltab[LDS ? kLzTabLds : 1];
    if constexpr (LDS) {
        for (int64_t s = threadIdx.x; s < ntab; s += blockDim.x) ltab[s] = tab[s];
        __syncthreads();
    }
    // s < ntab for every reachable sum: the table covers them (tci_func_create sizes it, and this
    // kernel runs only with a table)
    (void)p0;
    auto q = [&](int64_t s) -> double {
        if constexpr (LDS)
            return ltab[s];
        else
            return tab[s];
    };
    double mx = 0.0;
    auto upd = [&](double v) {
        const double a = fabs(v);
        mx = (isnan(a) || a > mx) ? a : mx;
    };
    const int64_t rtiles = (mR + 511) / 512;
    const int64_t ctiles = (n + kLzCols - 1) / kLzCols;
    const int64_t ntiles = rtiles * ctiles;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t R = (t % rtiles) * 512 + 2 * threadIdx.x;
        const int j0 = (int)(t / rtiles) * kLzCols;
        const bool h0 = R < mR, h1 = R + 1 < mR;
        const int64_t s0 = h0 ? rs[R].i : 0, s1 = h1 ? rs[R + 1].i : 0;
        if (j0 + kLzCols <= n && h1 && vec) {  // full tile: every load first, then the stores
            double v0[kLzCols], v1[kLzCols];
#pragma unroll
            for (int u = 0; u < kLzCols; ++u) {
                const int64_t c = cs[j0 + u].i;
                v0[u] = q(s0 + c);
                v1[u] = q(s1 + c);
            }
#pragma unroll
            for (int u = 0; u < kLzCols; ++u) {
                upd(v0[u]);
                upd(v1[u]);
                typedef double dv2 __attribute__((ext_vector_type(2)));
                __builtin_nontemporal_store(dv2{v0[u], v1[u]}, reinterpret_cast<dv2*>(out + R + ldo * (j0 + u)));
            }
        } else if (h0) {
            const int je = min(j0 + kLzCols, n);
            for (int j = j0; j < je; ++j) {
                const int64_t c = cs[j].i;
                double* o = out + R + ldo * j;
                const double v0 = q(s0 + c);
                upd(v0);
                if (h1) {
                    const double v1 = q(s1 + c);
                    upd(v1);
                    if (vec) {
                        *reinterpret_cast<double2*>(o) = double2{v0, v1};
                    } else {
                        o[0] = v0;
                        o[1] = v1;
                    }
                } else {
                    o[0] = v0;
                }
            }
        }
    }
    block_maxabs(mx, maxbits);
}

// Direct per-element path (TCI_F_GAUSSMIX, TCI_F_TT): the reference's loop order of f itself.
__device__ double feval_direct(const FuncDev& f, const int32_t* e, int nl, int c, int M,
                               const int32_t* g, int nr) {
    const int L = f.L;
    const double* p = f.params;
    auto leg = [&](int t) -> int {
        if (t < nl) return e[t];
        if (t < nl + M) return c + 1;
        return g[t - nl - M];
    };
    if (f.kind == F_GAUSSMIX) {
        const int K = (int)p[0];
        const double a = p[1];
        const double* cc = p + 2;
        const double* w = p + 2 + (int64_t)K * L;
        double acc = 0.0;
        for (int k = 0; k < K; ++k) {
            double s = 0.0;
            for (int t = 0; t < L; ++t) {
                const double u = (double)leg(t) - cc[(int64_t)k * L + t];
                s = __dadd_rn(s, __dmul_rn(u, u));
            }
            acc = __dadd_rn(acc, __dmul_rn(w[k], exp(-(a * s))));
        }
        return acc;
    }
    if (f.kind == F_TT) {
        // p = [r_0..r_L, cores...]; left-to-right vector-matrix chain (<= 64 bond dimension)
        const double* r = p;
        const double* core = p + L + 1;
        double v[64], w2[64];
        const int r1 = (int)r[1];
        const int d0 = f.localdims[0];
        for (int b = 0; b < r1; ++b) v[b] = core[(leg(0) - 1) + (int64_t)b * d0];
        core += (int64_t)r[0] * d0 * r1;
        for (int t = 1; t < L; ++t) {
            const int ra = (int)r[t], rb = (int)r[t + 1], d = f.localdims[t];
            const int x = leg(t) - 1;
            for (int b = 0; b < rb; ++b) {
                double s = 0.0;
                for (int a = 0; a < ra; ++a)
                    s = __dadd_rn(s, __dmul_rn(v[a], core[a + (int64_t)ra * x + (int64_t)ra * d * b]));
                w2[b] = s;
            }
            for (int b = 0; b < rb; ++b) v[b] = w2[b];
            core += (int64_t)ra * d * rb;
        }
        return v[0];
    }
    return 0.0;
}

__global__ __launch_bounds__(256) void k_assemble_direct(FuncDev f, const int32_t* __restrict__ I,
                                                         int m, int nl, const int32_t* __restrict__ J,
                                                         int n, int nr, int M, int D,
                                                         double* __restrict__ out, int64_t ldo,
                                                         unsigned long long* maxbits) {
    double mx = 0.0;
    const int64_t mR = (int64_t)m * D;
    const int64_t tot = mR * n;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t R = e % mR;
        const int j = (int)(e / mR);
        const int i = (int)(R % m), c = (int)(R / m);
        const double v = feval_direct(f, I + (int64_t)i * nl, nl, c, M, J + (int64_t)j * nr, nr);
        out[R + ldo * j] = v;
        const double av = fabs(v);
        mx = (isnan(av) || av > mx) ? av : mx;
    }
    block_maxabs(mx, maxbits);
}

// ------------------------------------------------ separable kinds: GEMM
// GAUSSMIX: f = sum_k w_k exp(-(a * sum_t (x_t - c_kt)^2)) = sum_k EL[R,k] ER[j,k] with
//   EL = exp(-(a * S_left)), ER = w_k exp(-(a * S_right)) (S: partial sums over the legs of I
//   (+ centre) / J). Splitting the exponential changes the rounding against per-element
//   evaluation by ~|a S| ulps (tests: rtol 1e-12).
// CP: f = sum_k prod_t g[k][t][x_t]: EL / ER = partial products.
// Factors are stored k-major (EL[k * ldR + R], ER[k * ldC + j]) and zero-padded to K4 = 4 |K.

__device__ double cp_factor(const FuncDev& f, int k, const int32_t* e, int t0, int cnt, int cval,
                            bool right) {
    // legs t0 .. t0 + cnt - 1 take values e[0 .. cnt-1]; if cval > 0 one more leg (the centre,
    // position t0 + cnt) takes cval
    const int L = f.L;
    const double* p = f.params;
    const int K = (int)p[0];
    if (f.kind == F_GAUSSMIX) {
        const double a = p[1];
        const double* cc = p + 2 + (int64_t)k * L;
        double s = 0.0;
        for (int q = 0; q < cnt; ++q) {
            const double u = (double)e[q] - cc[t0 + q];
            s = __dadd_rn(s, __dmul_rn(u, u));
        }
        if (cval > 0) {
            const double u = (double)cval - cc[t0 + cnt];
            s = __dadd_rn(s, __dmul_rn(u, u));
        }
        const double v = exp(-(a * s));
        return right ? __dmul_rn(p[2 + (int64_t)K * L + k], v) : v;
    }
    // F_CP
    const int dmax = (int)p[1];
    const double* g = p + 2 + (int64_t)k * L * dmax;
    double prod = 1.0;
    for (int q = 0; q < cnt; ++q) prod = __dmul_rn(prod, g[(int64_t)(t0 + q) * dmax + (e[q] - 1)]);
    if (cval > 0) prod = __dmul_rn(prod, g[(int64_t)(t0 + cnt) * dmax + (cval - 1)]);
    return prod;
}

// rows: R in [0, m*D) (i = R % m, centre c = R / m); cols: j in [0, n) (legs L - nr ..)
__global__ void k_cp_factors(FuncDev f, const int32_t* __restrict__ T, int cnt, int nrows, int D,
                             int M, int K, int K4, int64_t ld, int t0, bool right,
                             double* __restrict__ out) {
    const int64_t tot = (int64_t)ld * K4;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int R = (int)(e % ld), k = (int)(e / ld);
        double v = 0.0;
        if (R < (int64_t)nrows * D && k < K) {
            const int i = R % nrows, c = R / nrows;
            v = cp_factor(f, k, T + (int64_t)i * cnt, t0, cnt, M ? c + 1 : 0, right);
        }
        out[e] = v;
    }
}

// ------------------------------------------------ MPO-MPO contraction (contraction.jl)
// f = Contraction(A, B) (contraction.jl:60-152): f(x) = the product of A_t[:, s1, :, :] and
// B_t[:, :, s3, :] over all sites, every inner index summed, with x_t the fused site index
// s1 + d1 (s3 - 1) (_unfuse_idx / _fuse_idx, contraction.jl:226-237). For a split of the legs
// into row legs and column legs, Pi[R, j] = sum_{a,b} Lenv_R[a, b] Renv_j[a, b]: the left and
// right environments (evaluateleft / evaluateright, contraction.jl:279-354, with the centre leg
// of batchevaluate folded into the rows, :483-575). So a contraction is a separable kind of K =
// ra*rb terms at the cut: k_mpo_env computes the environments as the factor rows (batched small
// contractions, one workgroup per row, intermediates in LDS) and the fp64 MFMA GEMM (k_gemm_cp*)
// assembles Pi.
// params: [N, per site t: ra, d1, d2, ra', rb, d3, rb', offA, offB, then the cores]; core A_t is
// (ra, d1, d2, ra') and B_t (rb, d2, d3, rb'), column-major, at the given offsets past the header.
struct MpoSite {
    int ra, d1, d2, ra2, rb, d3, rb2;
    int64_t offA, offB;
};

__device__ __forceinline__ MpoSite mpo_site(const double* p, int t) {
    const double* q = p + 1 + 9 * t;
    return MpoSite{(int)q[0], (int)q[1], (int)q[2], (int)q[3], (int)q[4],
                   (int)q[5], (int)q[6], (int64_t)q[7], (int64_t)q[8]};
}

// Environment rows: R in [0, nrows * D) (i = R % nrows, centre c = R / nrows when M == 1). Left:
// sites 0 .. nlegs-1 in order; right: sites t0 .. t0+nlegs-1 from the last one backwards. Writes
// out[k * ld + R] for k < K4 (k = a + ra_cut * b; zero past the cut's ra * rb) and zeroes the
// padding rows [nrows * D, ld).
// LDS layouts keep every inner-product read either broadcast or unit-stride across lanes (the
// environments of the left chain padded to an odd leading dimension ra + 1, the intermediate to
// rb*d2 + 1); the summation orders are those of the unpadded form.
__global__ __launch_bounds__(256) void k_mpo_env(FuncDev f, const int32_t* __restrict__ T, int cnt,
                                                 int nrows, int D, int M, int K4, int64_t ld, int t0,
                                                 int right, double* __restrict__ out) {
    extern __shared__ double smem_mpo[];
    double* env = smem_mpo;              // f.mpoEnv doubles
    double* tmp = smem_mpo + f.mpoEnv;   // f.mpoTmp doubles
    const double* p = f.params;
    const int N = (int)p[0];
    const double* data = p + 1 + 9 * (int64_t)N;
    const int nlegs = cnt + (M ? 1 : 0);
    const int64_t rows = (int64_t)nrows * D;
    for (int64_t e = rows * K4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ld * K4;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = (e - rows * K4) / (ld - rows), R = rows + (e - rows * K4) % (ld - rows);
        out[k * ld + R] = 0.0;
    }
    for (int64_t R = blockIdx.x; R < rows; R += gridDim.x) {
        const int i = (int)(R % nrows), c = (int)(R / nrows);
        const int32_t* e = T + (int64_t)i * cnt;
        if (threadIdx.x == 0) env[0] = 1.0;
        int ea = 1, eb = 1;
        __syncthreads();
        for (int q = 0; q < nlegs; ++q) {
            const int leg = right ? nlegs - 1 - q : q;
            const int t = right ? t0 + leg : leg;
            const int idx = (leg < cnt ? e[leg] : c + 1) - 1;
            const MpoSite s = mpo_site(p, t);
            const int s1 = idx % s.d1, s3 = idx / s.d1;
            const double* A = data + s.offA;
            const double* B = data + s.offB;
            if (!right) {
                // tmp[b, s2, a'] = sum_a env[a, b] A[a, s1, s2, a']   (_extend_cache, first step);
                // env[a, b] at a + (ra + 1) b, tmp[b, s2, a'] at b + rb s2 + (rb d2 + 1) a'
                const int nt = s.rb * s.d2 * s.ra2, le = s.ra + 1, lt = s.rb * s.d2 + 1;
                for (int o = threadIdx.x; o < nt; o += blockDim.x) {
                    const int b = o % s.rb, s2 = (o / s.rb) % s.d2, a2 = o / (s.rb * s.d2);
                    const double* Ap = A + (int64_t)s.ra * (s1 + (int64_t)s.d1 * (s2 + (int64_t)s.d2 * a2));
                    double acc = 0.0;
                    for (int a = 0; a < s.ra; ++a) acc = acc + env[a + le * b] * Ap[a];
                    tmp[b + s.rb * s2 + lt * a2] = acc;
                }
                __syncthreads();
                // env[a', b'] = sum_{s2, b} tmp[b, s2, a'] B[b, s2, s3, b']   (second step)
                const int ne = s.ra2 * s.rb2, le2 = s.ra2 + 1;
                for (int o = threadIdx.x; o < ne; o += blockDim.x) {
                    const int a2 = o % s.ra2, b2 = o / s.ra2;
                    const double* Bp = B + (int64_t)s.rb * s.d2 * (s3 + (int64_t)s.d3 * b2);
                    const double* tp = tmp + lt * a2;
                    double acc = 0.0;
                    for (int s2 = 0; s2 < s.d2; ++s2)
                        for (int b = 0; b < s.rb; ++b)
                            acc = acc + tp[b + s.rb * s2] * Bp[b + (int64_t)s.rb * s2];
                    env[a2 + le2 * b2] = acc;
                }
                ea = s.ra2;
                eb = s.rb2;
            } else {
                // tmp[a, s2, b'] = sum_a' A[a, s1, s2, a'] env[a', b']
                const int nt = s.ra * s.d2 * s.rb2;
                const int64_t sa = (int64_t)s.ra * s.d1 * s.d2;
                for (int o = threadIdx.x; o < nt; o += blockDim.x) {
                    const int a = o % s.ra, s2 = (o / s.ra) % s.d2, b2 = o / (s.ra * s.d2);
                    const double* Ap = A + a + (int64_t)s.ra * (s1 + (int64_t)s.d1 * s2);
                    double acc = 0.0;
                    for (int a2 = 0; a2 < s.ra2; ++a2) acc = acc + Ap[sa * a2] * env[a2 + s.ra2 * b2];
                    tmp[o] = acc;
                }
                __syncthreads();
                // env[a, b] = sum_{b', s2} tmp[a, s2, b'] B[b, s2, s3, b']
                const int ne = s.ra * s.rb;
                for (int o = threadIdx.x; o < ne; o += blockDim.x) {
                    const int a = o % s.ra, b = o / s.ra;
                    double acc = 0.0;
                    for (int b2 = 0; b2 < s.rb2; ++b2) {
                        const double* Bp = B + b + (int64_t)s.rb * s.d2 * (s3 + (int64_t)s.d3 * b2);
                        for (int s2 = 0; s2 < s.d2; ++s2)
                            acc = acc + tmp[a + s.ra * (s2 + s.d2 * b2)] * Bp[(int64_t)s.rb * s2];
                    }
                    env[o] = acc;
                }
                ea = s.ra;
                eb = s.rb;
            }
            __syncthreads();
        }
        // factor row: k = a + ea * b (the left chain's environment is stored with ld ea + 1)
        const int lde = right ? ea : ea + 1;
        for (int k = threadIdx.x; k < K4; k += blockDim.x)
            out[(int64_t)k * ld + R] = k < ea * eb ? env[k % ea + lde * (k / ea)] : 0.0;
        __syncthreads();
    }
}

// The same environments with both per-site contractions on v_mfma_f64_16x16x4f64 (used when
// the bonds are not tiny, cpK >= 64): every site is two small GEMMs whose operands come from LDS
// (the environment, the intermediate) and from the L2-resident cores, 16 x 16 output tiles
// spread over the 4 waves, zero-filled past the edges. Operand lanes: A[row l&15][k l>>4],
// B[k l>>4][col l&15]; result: col = l & 15, row = (l >> 4) + 4 * reg. Environments of both
// chains at a + (ra + 1) b; intermediates with leading dimensions rb*d2 + 1 (left) and
// ra*d2 + 1 (right), so that lanes reading different rows hit different banks.
typedef double mpo_dbl4 __attribute__((ext_vector_type(4)));

template <class FA, class FB, class FS>
__device__ __forceinline__ void mpo_mfma_gemm(int M, int N, int K, FA fa, FB fb, FS st) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int tm = (M + 15) >> 4, tn = (N + 15) >> 4;
    for (int t = wave; t < tm * tn; t += nw) {  // wave-uniform
        const int m0 = (t % tm) << 4, n0 = (t / tm) << 4;
        const int r = m0 + (lane & 15), cc = n0 + (lane & 15), kq = lane >> 4;
        mpo_dbl4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = 0; k0 < K; k0 += 4) {
            const int k = k0 + kq;
            const double a = (r < M && k < K) ? fa(r, k) : 0.0;
            const double b = (k < K && cc < N) ? fb(k, cc) : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int rr = m0 + (lane >> 4) + 4 * i;
            if (rr < M && cc < N) st(rr, cc, acc[i]);
        }
    }
}

__global__ __launch_bounds__(256) void k_mpo_env_mfma(FuncDev f, const int32_t* __restrict__ T, int cnt,
                                                      int nrows, int D, int M, int K4, int64_t ld, int t0,
                                                      int right, double* __restrict__ out) {
    extern __shared__ double smem_mpo[];
    double* env = smem_mpo;              // f.mpoEnv doubles
    double* tmp = smem_mpo + f.mpoEnv;   // f.mpoTmp doubles
    const double* p = f.params;
    const int N = (int)p[0];
    const double* data = p + 1 + 9 * (int64_t)N;
    const int nlegs = cnt + (M ? 1 : 0);
    const int64_t rows = (int64_t)nrows * D;
    for (int64_t e = rows * K4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < ld * K4;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = (e - rows * K4) / (ld - rows), R = rows + (e - rows * K4) % (ld - rows);
        out[k * ld + R] = 0.0;
    }
    for (int64_t R = blockIdx.x; R < rows; R += gridDim.x) {
        const int i = (int)(R % nrows), c = (int)(R / nrows);
        const int32_t* e = T + (int64_t)i * cnt;
        if (threadIdx.x == 0) env[0] = 1.0;
        int ea = 1, eb = 1;
        __syncthreads();
        for (int q = 0; q < nlegs; ++q) {
            const int leg = right ? nlegs - 1 - q : q;
            const int t = right ? t0 + leg : leg;
            const int idx = (leg < cnt ? e[leg] : c + 1) - 1;
            const MpoSite s = mpo_site(p, t);
            const int s1 = idx % s.d1, s3 = idx / s.d1;
            const double* A = data + s.offA + (int64_t)s.ra * s1;           // A[a, s1, s2, a'] at a + ra d1 (s2 + d2 a')
            const double* B = data + s.offB + (int64_t)s.rb * s.d2 * s3;    // B[b, s2, s3, b'] at b + rb s2 + rb d2 d3 b'
            const int64_t sA = (int64_t)s.ra * s.d1, sB = (int64_t)s.rb * s.d2 * s.d3;
            if (!right) {
                const int le = s.ra + 1, lt = s.rb * s.d2 + 1, le2 = s.ra2 + 1, d2 = s.d2, rb = s.rb;
                // tmp[b, s2, a'] = sum_a env[a, b] A[a, s1, s2, a']: rows b, columns n = s2 + d2 a'
                mpo_mfma_gemm(
                    s.rb, s.d2 * s.ra2, s.ra, [&](int b, int a) { return env[a + le * b]; },
                    [&](int a, int n) { return A[a + sA * ((n % d2) + (int64_t)d2 * (n / d2))]; },
                    [&](int b, int n, double v) { tmp[b + rb * (n % d2) + lt * (n / d2)] = v; });
                __syncthreads();
                // env[a', b'] = sum_{kk = b + rb s2} tmp[kk, a'] B[kk, s3, b']
                mpo_mfma_gemm(
                    s.ra2, s.rb2, s.rb * s.d2, [&](int a2, int kk) { return tmp[kk + lt * a2]; },
                    [&](int kk, int b2) { return B[kk + sB * b2]; },
                    [&](int a2, int b2, double v) { env[a2 + le2 * b2] = v; });
                ea = s.ra2;
                eb = s.rb2;
            } else {
                const int le2 = s.ra2 + 1, ra = s.ra, d2 = s.d2, lr = s.ra * s.d2 + 1, le = s.ra + 1;
                // tmp[a, s2, b'] = sum_a' A[a, s1, s2, a'] env[a', b']: rows r = a + ra s2
                mpo_mfma_gemm(
                    s.ra * s.d2, s.rb2, s.ra2,
                    [&](int r, int a2) { return A[(r % ra) + sA * ((r / ra) + (int64_t)d2 * a2)]; },
                    [&](int a2, int b2) { return env[a2 + le2 * b2]; },
                    [&](int r, int b2, double v) { tmp[r + lr * b2] = v; });
                __syncthreads();
                // env[a, b] = sum_{kk = s2 + d2 b'} tmp[a, s2, b'] B[b, s2, s3, b']
                mpo_mfma_gemm(
                    s.ra, s.rb, s.d2 * s.rb2,
                    [&](int a, int kk) { return tmp[a + ra * (kk % d2) + lr * (kk / d2)]; },
                    [&](int kk, int b) { return B[b + (int64_t)s.rb * (kk % d2) + sB * (kk / d2)]; },
                    [&](int a, int b, double v) { env[a + le * b] = v; });
                ea = s.ra;
                eb = s.rb;
            }
            __syncthreads();
        }
        for (int k = threadIdx.x; k < K4; k += blockDim.x)
            out[(int64_t)k * ld + R] = k < ea * eb ? env[k % ea + (ea + 1) * (k / ea)] : 0.0;
        __syncthreads();
    }
}

// Pi[R, j] = sum_k EL[k, R] * ER[k, j] on v_mfma_f64_16x16x4_f64: a wave owns a 32 x 32 tile
// (2 x 2 MFMA blocks), a workgroup 4 waves (64 x 64). Operand lanes: A[row l&15][k l>>4],
// B[k l>>4][col l&15]; result: col = l & 15, row = (l >> 4) + 4 * reg (cdna_hip_programming.md).
typedef double dbl4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_gemm_cp(const double* __restrict__ EL, int64_t ldR,
                                                 const double* __restrict__ ER, int64_t ldC, int K4,
                                                 int64_t mR, int n, double* __restrict__ out,
                                                 int64_t ldo, unsigned long long* maxbits) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t R0 = (int64_t)blockIdx.x * 64 + (wv & 1) * 32;
    const int64_t j0 = (int64_t)blockIdx.y * 64 + (wv >> 1) * 32;
    const int r = lane & 15, kk = lane >> 4;
    dbl4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};
    // factors are padded to whole 32-row / 32-column tiles (ldR, ldC multiples of 64): no guards
    for (int k0 = 0; k0 < K4; k0 += 4) {
        const double* el = EL + (int64_t)(k0 + kk) * ldR + R0 + r;
        const double* er = ER + (int64_t)(k0 + kk) * ldC + j0 + r;
        const double a0 = el[0], a1 = el[16], b0 = er[0], b1 = er[16];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    double mx = 0.0;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int64_t R = R0 + 16 * x + (lane >> 4) + 4 * g;
                const int64_t j = j0 + 16 * y + (lane & 15);
                if (R < mR && j < n) {
                    const double v = acc[x][y][g];
                    out[R + ldo * j] = v;
                    const double av = fabs(v);
                    mx = (isnan(av) || av > mx) ? av : mx;
                }
            }
    block_maxabs(mx, maxbits);
}

// Large products go through the K3 kernel (tci_dense.hip k_dgemm: 128 x 128 tiles, two waves per
// SIMD); k staged 16 at a time, so the factors are padded to a multiple of kGemmKB rows.
constexpr int kGemmKB = 16;

// fp64 MFMA throughput probe (diagnostic): every wave issues independent 16x16x4 chains
__global__ __launch_bounds__(256) void k_mfma_f64_probe(int iters, double* sink) {
    dbl4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    if (s == 12345.0) sink[0] = s;  // keeps the chains alive
}

void launch_mfma_f64_probe(hipStream_t s, int grid, int iters, double* sink) {
    hipLaunchKernelGGL(k_mfma_f64_probe, dim3(grid), dim3(256), 0, s, iters, sink);
}

static int64_t cp_ld(int64_t rows) { return (rows + 127) / 128 * 128; }

int64_t batcheval_scratch_bytes(const FuncDev& f, int m, int D, int n) {
    if (cp_kind(f.kind)) {
        const int64_t K4 = (f.cpK + kGemmKB - 1) / kGemmKB * kGemmKB;
        return 8 * K4 * (cp_ld((int64_t)m * D) + cp_ld(n));
    }
    if (!staged_kind(f.kind)) return 0;
    return 8 * ((int64_t)m * D + n + (f.kind == F_LORENTZ ? f.ntab : 0));
}

void launch_batcheval(hipStream_t s, const FuncDev& f, const int32_t* I, int m, int nl,
                      const int32_t* J, int n, int nr, int M, int D, double* out, int64_t ldo,
                      unsigned long long* maxbits, void* scratch) {
    const int64_t mR = (int64_t)m * D;
    if (cp_kind(f.kind)) {
        const int K = f.cpK, K4 = (K + kGemmKB - 1) / kGemmKB * kGemmKB;
        const int64_t ldR = cp_ld(mR), ldC = cp_ld(n);
        double* EL = reinterpret_cast<double*>(scratch);
        double* ER = EL + (int64_t)K4 * ldR;
        if (f.kind == F_MPO) {  // environments: one workgroup per row / column
            const size_t lds = 8 * ((size_t)f.mpoEnv + f.mpoTmp);
            // tiny bonds: one thread per output entry; otherwise the per-site GEMMs on MFMA
            auto kern = f.cpK >= 64 ? k_mpo_env_mfma : k_mpo_env;
            hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
            hipLaunchKernelGGL(kern, dim3((unsigned)std::min<int64_t>(std::max<int64_t>(mR, 1), 16384)),
                               dim3(256), lds, s, f, I, nl, m, D, M, K4, ldR, 0, 0, EL);
            hipLaunchKernelGGL(kern, dim3((unsigned)std::min<int64_t>(std::max<int64_t>(n, 1), 16384)),
                               dim3(256), lds, s, f, J, nr, n, 1, 0, K4, ldC, f.L - nr, 1, ER);
        } else {
            hipLaunchKernelGGL(k_cp_factors, dim3(grid_for(ldR * K4, 4096)), dim3(256), 0, s, f, I, nl,
                               m, D, M, K, K4, ldR, 0, false, EL);
            hipLaunchKernelGGL(k_cp_factors, dim3(grid_for(ldC * K4, 4096)), dim3(256), 0, s, f, J, nr,
                               n, 1, 0, K, K4, ldC, f.L - nr, true, ER);
        }
        if (mR >= 128 && n >= 128 && K4 >= 32)  // Pi = EL^T ER on the K3 kernel (2 waves / SIMD)
            launch_dgemm(s, true, (int)mR, n, K4, 1.0, EL, ldR, ER, ldC, 0.0, nullptr, 0, out, ldo, nullptr, nullptr,
                         maxbits);
        else
            hipLaunchKernelGGL(k_gemm_cp, dim3((unsigned)(ldR / 64), (unsigned)(ldC / 64)), dim3(256), 0,
                               s, EL, ldR, ER, ldC, K4, mR, n, out, ldo, maxbits);
        return;
    }
    if (staged_kind(f.kind)) {
        St* rs = reinterpret_cast<St*>(scratch);
        St* cs = rs + mR;
        double* tab = reinterpret_cast<double*>(cs + n);
        const int64_t ntab = f.kind == F_LORENTZ ? f.ntab : 0;
        {
            const int gr = grid_for(mR, 4096), gc = grid_for(n, 4096), gt = ntab > 0 ? grid_for(ntab, 256) : 0;
            hipLaunchKernelGGL(k_state_prep, dim3(gr + gc + gt), dim3(256), 0, s, f, I, m, nl, M, D, rs, gr, J, n,
                               nr, f.L - nr, cs, gc, tab, ntab);
        }
        const int64_t ntiles = ((mR + 511) / 512) * ((n + kAsmCols - 1) / kAsmCols);
        const int grid = (int)(ntiles < 4096 ? (ntiles > 0 ? ntiles : 1) : 4096);
        const int vec = (ldo % 2 == 0) && ((uintptr_t)out % 16 == 0);
        if (f.kind == F_LORENTZ && ntab > 0) {
            const int64_t lt = ((mR + 511) / 512) * ((n + kLzCols - 1) / kLzCols);
            const int lg = (int)(lt < 2048 ? (lt > 0 ? lt : 1) : 2048);
            if (ntab <= kLzTabLds)
                hipLaunchKernelGGL(k_assemble_lorentz<true>, dim3(lg), dim3(256), 0, s, rs, cs, mR, n, out, ldo,
                                   maxbits, tab, ntab, 0.0, vec);
            else
                hipLaunchKernelGGL(k_assemble_lorentz<false>, dim3(lg), dim3(256), 0, s, rs, cs, mR, n, out, ldo,
                                   maxbits, tab, ntab, 0.0, vec);
            return;
        }
        switch (f.kind) {
#define TCI_ASM(K)                                                                                  \
    case K:                                                                                         \
        hipLaunchKernelGGL(k_assemble<K>, dim3(grid), dim3(256), 0, s, f, rs, cs, mR, n, nr, out, ldo, \
                           maxbits, tab, ntab, vec);                                                \
        break;
            TCI_ASM(F_SUM) TCI_ASM(F_LORENTZ) TCI_ASM(F_TABLE) TCI_ASM(F_GAUSS) TCI_ASM(F_QOSC)
            TCI_ASM(F_QEXP)
#undef TCI_ASM
        default: break;
        }
    } else {
        hipLaunchKernelGGL(k_assemble_direct, dim3(grid_for(mR * n, 4096)), dim3(256), 0, s, f, I, m,
                           nl, J, n, nr, M, D, out, ldo, maxbits);
    }
}

// ------------------------------------------------ tensor-train evaluation
// evaluate(tt, idx) = only(prod(T[:, i, :])) (abstracttensortrain.jl:328-342) at many points, for
// the global pivot search (globalpivotfinder.jl:236): a workgroup carries kTtPts row vectors
// through the chain of vector-matrix products, one output entry per thread and step, the
// vectors in LDS. Core t is (r_t, d_t, r_{t+1}) column-major at offset off[t].
constexpr int kTtPts = 8;

__global__ __launch_bounds__(256) void k_tt_eval(const double* __restrict__ cores,
                                                 const int64_t* __restrict__ off,
                                                 const int32_t* __restrict__ rdim,
                                                 const int32_t* __restrict__ dims, int L,
                                                 const int32_t* __restrict__ X, int npts,
                                                 double* __restrict__ out, int rmax) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* v = reinterpret_cast<double*>(smem);  // [pt][rmax]
    double* w = v + kTtPts * rmax;
    const int p0 = blockIdx.x * kTtPts;
    const int np = min(kTtPts, npts - p0);
    for (int t = 0; t < L; ++t) {
        const int ra = rdim[t], rb = rdim[t + 1], d = dims[t];
        const double* core = cores + off[t];
        for (int e = threadIdx.x; e < np * rb; e += blockDim.x) {
            const int pt = e / rb, b = e % rb;
            const int x = X[(int64_t)(p0 + pt) * L + t] - 1;
            const double* col = core + (int64_t)ra * x + (int64_t)ra * d * b;
            double s;
            if (t == 0) {
                s = col[0];  // r_0 == 1: the row of the first core
            } else {
                s = 0.0;
                for (int a = 0; a < ra; ++a) s = __dadd_rn(s, __dmul_rn(v[pt * rmax + a], col[a]));
            }
            w[pt * rmax + b] = s;
        }
        __syncthreads();
        double* tmp = v;
        v = w;
        w = tmp;
    }
    if (threadIdx.x < np) out[p0 + threadIdx.x] = v[threadIdx.x * rmax];
}

void launch_tt_eval(hipStream_t s, const double* cores, const int64_t* off, const int32_t* rdim,
                    const int32_t* dims, int L, const int32_t* X, int npts, double* out, int rmax) {
    const size_t bytes = 2 * (size_t)kTtPts * rmax * sizeof(double);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tt_eval), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)bytes);
    hipLaunchKernelGGL(k_tt_eval, dim3((npts + kTtPts - 1) / kTtPts), dim3(256), bytes, s, cores, off, rdim,
                       dims, L, X, npts, out, rmax);
}

// ------------------------------------------------------ site-tensor solve
// T = Pi1 * P^-1 (tensorci2.jl:626): A = P^T is factorised in place with partial pivoting
// (first maximal |a| in a column, as getrf/idamax), one workgroup; then each thread solves one
// right-hand side (one row of Pi1, a column of Pi1^T).
__global__ __launch_bounds__(1024) void k_getrf_transposed(double* __restrict__ P, int r,
                                                           int* __restrict__ piv) {
    // P holds P (r x r, ld r); transpose in place into A = P^T first
    for (int e = threadIdx.x; e < r * r; e += blockDim.x) {
        const int i = e % r, j = e / r;
        if (i < j) {
            const double a = P[i + j * r], b = P[j + i * r];
            P[i + j * r] = b;
            P[j + i * r] = a;
        }
    }
    __syncthreads();
    __shared__ double sv[16];
    __shared__ int si[16];
    __shared__ int sp;
    for (int k = 0; k < r; ++k) {
        // pivot search in column k (smallest row index on ties)
        double bv = -1.0;
        int bi = kBig;
        for (int i = k + threadIdx.x; i < r; i += blockDim.x) {
            const double v = fabs(P[i + k * r]);
            if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
        }
        for (int off = 32; off >= 1; off >>= 1) {
            const double v2 = __shfl_xor(bv, off);
            const int i2 = __shfl_xor(bi, off);
            if (v2 > bv || (v2 == bv && i2 < bi)) { bv = v2; bi = i2; }
        }
        const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
        if (l == 0) { sv[w] = bv; si[w] = bi; }
        __syncthreads();
        if (threadIdx.x == 0) {
            double b = sv[0];
            int ii = si[0];
            for (int q = 1; q < (int)(blockDim.x >> 6); ++q)
                if (sv[q] > b || (sv[q] == b && si[q] < ii)) { b = sv[q]; ii = si[q]; }
            if (ii == kBig) ii = k;
            sp = ii;
            piv[k] = ii;
        }
        __syncthreads();
        const int p = sp;
        if (p != k)
            for (int j = threadIdx.x; j < r; j += blockDim.x) {
                const double a = P[k + j * r];
                P[k + j * r] = P[p + j * r];
                P[p + j * r] = a;
            }
        __syncthreads();
        const double d = P[k + k * r];
        for (int i = k + 1 + threadIdx.x; i < r; i += blockDim.x) P[i + k * r] = P[i + k * r] / d;
        __syncthreads();
        const int tr = r - k - 1;
        for (int e = threadIdx.x; e < tr * tr; e += blockDim.x) {
            const int i = k + 1 + e % tr, j = k + 1 + e / tr;
            P[i + j * r] = __dsub_rn(P[i + j * r], __dmul_rn(P[i + k * r], P[k + j * r]));
        }
        __syncthreads();
    }
}

__global__ void k_getrs_rows(const double* __restrict__ A, int r, const int* __restrict__ piv,
                             double* __restrict__ Pi1, int R, double* __restrict__ T) {
    // solves A x = b for b = Pi1[row, :]^T, stores x^T into T[row, :]; x kept in T (ld R)
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= R) return;
    double* x = T + row;  // element a at x[a * R]
    for (int a = 0; a < r; ++a) x[(int64_t)a * R] = Pi1[row + (int64_t)a * R];
    for (int k = 0; k < r; ++k) {
        const int p = piv[k];
        if (p != k) {
            const double t = x[(int64_t)k * R];
            x[(int64_t)k * R] = x[(int64_t)p * R];
            x[(int64_t)p * R] = t;
        }
    }
    for (int k = 0; k < r; ++k) {
        const double xk = x[(int64_t)k * R];
        for (int i = k + 1; i < r; ++i)
            x[(int64_t)i * R] = __dsub_rn(x[(int64_t)i * R], __dmul_rn(A[i + k * r], xk));
    }
    for (int k = r - 1; k >= 0; --k) {
        const double xk = x[(int64_t)k * R] / A[k + k * r];
        x[(int64_t)k * R] = xk;
        for (int i = 0; i < k; ++i)
            x[(int64_t)i * R] = __dsub_rn(x[(int64_t)i * R], __dmul_rn(A[i + k * r], xk));
    }
}

// The same solve for RHS rows per workgroup with x in LDS (Xs[a * RHS + q]): the row
// interchanges, then the unit-lower and the upper solves in 16-column blocks -- the block's
// diagonal part per right-hand side, then its contribution to every remaining row in parallel.
// k_getrs_rows keeps x in global memory (every update a read-modify-write of HBM/L2: 7.8 ms at
// r = 256, R = 8192); the summation order per element changes with the blocking (LAPACK's order
// is not pinned by the reference either).
template <int RHS>
__global__ __launch_bounds__(256) void k_getrs_blocked(const double* __restrict__ A, int r,
                                                       const int* __restrict__ piv,
                                                       const double* __restrict__ Pi1, int R,
                                                       double* __restrict__ T) {
    extern __shared__ double Xs[];
    const int r0 = blockIdx.x * RHS, nq = min(RHS, R - r0), tid = threadIdx.x;
    for (int e = tid; e < RHS * r; e += blockDim.x) {
        const int q = e % RHS, a = e / RHS;
        Xs[e] = q < nq ? Pi1[r0 + q + (int64_t)a * R] : 0.0;
    }
    __syncthreads();
    if (tid < RHS)
        for (int k = 0; k < r; ++k) {
            const int p = piv[k];
            if (p != k) {
                const double t = Xs[k * RHS + tid];
                Xs[k * RHS + tid] = Xs[p * RHS + tid];
                Xs[p * RHS + tid] = t;
            }
        }
    __syncthreads();
    constexpr int B = 16;
    for (int jb = 0; jb < r; jb += B) {  // L (unit lower, below the diagonal of A)
        const int je = min(jb + B, r);
        if (tid < RHS)
            for (int j = jb; j < je; ++j) {
                double v = Xs[j * RHS + tid];
                for (int t = jb; t < j; ++t) v = __dsub_rn(v, __dmul_rn(A[j + t * r], Xs[t * RHS + tid]));
                Xs[j * RHS + tid] = v;
            }
        __syncthreads();
        for (int e = tid; e < RHS * (r - je); e += blockDim.x) {
            const int q = e % RHS, i = je + e / RHS;
            double v = Xs[i * RHS + q];
            for (int t = jb; t < je; ++t) v = __dsub_rn(v, __dmul_rn(A[i + t * r], Xs[t * RHS + q]));
            Xs[i * RHS + q] = v;
        }
        __syncthreads();
    }
    for (int jb = ((r - 1) / B) * B; jb >= 0; jb -= B) {  // U (upper, with the diagonal)
        const int je = min(jb + B, r);
        if (tid < RHS)
            for (int j = je - 1; j >= jb; --j) {
                double v = Xs[j * RHS + tid];
                for (int t = j + 1; t < je; ++t) v = __dsub_rn(v, __dmul_rn(A[j + t * r], Xs[t * RHS + tid]));
                Xs[j * RHS + tid] = v / A[j + j * r];
            }
        __syncthreads();
        for (int e = tid; e < RHS * jb; e += blockDim.x) {
            const int q = e % RHS, i = e / RHS;
            double v = Xs[i * RHS + q];
            for (int t = jb; t < je; ++t) v = __dsub_rn(v, __dmul_rn(A[i + t * r], Xs[t * RHS + q]));
            Xs[i * RHS + q] = v;
        }
        __syncthreads();
    }
    for (int e = tid; e < RHS * r; e += blockDim.x) {
        const int q = e % RHS, a = e / RHS;
        if (q < nq) T[r0 + q + (int64_t)a * R] = Xs[e];
    }
}

bool getrf_blocked_fits(int r);
void launch_getrf_coop(hipStream_t s, double* A, int r, int* piv, unsigned* sync);
void launch_getrf_blocked(hipStream_t s, double* A, int r, int* piv, bool reg_panel);
void launch_getrs_blocked(hipStream_t s, const double* A, int r, const int* piv, const double* Pi1,
                          int R, double* T, int* perm, bool perm_ready);


// piv: 2 r + 2 ints (interchanges, the permutation they compose to, the cooperative getrf's
// arrival counter and fault word). parts: 1 = the getrf, 2 = the getrs, 3 = both. A cooperative
// getrf that gave up leaves no permutation, so its caller launches part 1, checks the fault word,
// and only then part 2 (tci_abi.cpp solve_launch)
void launch_sitetensor_solve_parts(hipStream_t s, double* P, int r, double* Pi1, int R, double* T,
                                   int* piv, int dense, int parts) {
    const int reg = kDenseGetrf | kDenseGetrfReg | kDenseGetrfCoop;
    const bool coop = (dense & reg) == reg && getrf_coop_fits(r);  // also leaves the permutation at piv + r
    if (parts & 1) {
        if (coop)
            launch_getrf_coop(s, P, r, piv, reinterpret_cast<unsigned*>(piv + 2 * r));
        else if ((dense & kDenseGetrf) && getrf_blocked_fits(r))
            launch_getrf_blocked(s, P, r, piv, (dense & kDenseGetrfReg) != 0);
        else hipLaunchKernelGGL(k_getrf_transposed, dim3(1), dim3(1024), 0, s, P, r, piv);
    }
    if (!(parts & 2)) return;
    if (R <= 0) return;
    if (dense & kDenseGetrs) {
        launch_getrs_blocked(s, P, r, piv, Pi1, R, T, piv + r, coop);
        return;
    }
    if (r > 4096) {
        hipLaunchKernelGGL(k_getrs_rows, dim3((R + 127) / 128), dim3(128), 0, s, P, r, piv, Pi1, R, T);
        return;
    }
    // RHS x r doubles of LDS: at most 64 KiB
    auto go = [&](auto kern, int rhs) {
        const size_t bytes = (size_t)rhs * r * sizeof(double);
        hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)bytes);
        hipLaunchKernelGGL(kern, dim3((R + rhs - 1) / rhs), dim3(256), bytes, s, P, r, piv, Pi1, R, T);
    };
    if (r <= 256)
        go(k_getrs_blocked<32>, 32);
    else if (r <= 512)
        go(k_getrs_blocked<16>, 16);
    else if (r <= 1024)
        go(k_getrs_blocked<8>, 8);
    else
        go(k_getrs_blocked<2>, 2);
}

void launch_sitetensor_solve(hipStream_t s, double* P, int r, double* Pi1, int R, double* T, int* piv,
                             int dense) {
    launch_sitetensor_solve_parts(s, P, r, Pi1, R, T, piv, dense, 3);
}

}  // namespace tci
