// tci_rrlu_c128.hip -- rrLU with full pivoting on ComplexF64 matrices (gfx950).
//
// rrlu(A::Matrix{ComplexF64}) runs the same _optimizerrlu! / addpivot! loop as the Float64 path
// (matrixlu.jl:295-322, 346-396); SURVEY §8f rank 4. Entries are double2 (re, im) column-major,
// Julia's ComplexF64 layout. Unlike the Float64 kernels (logical swaps, deferred updates,
// certified fp32 shadow search) this path keeps the reference's physical row/column swaps; per
// pivot:
//   (1) the rank-1 update of pivot t-1 (normalised column/row from the published pivot
//       column/row buffers, so no workgroup reads what another writes), complex multiply then
//       subtract componentwise (matrixlu.jl:318; no fma: -ffp-contract=off),
//   (2) the argmax of abs2 over the trailing block for pivot t (strict '>' in column-major order
//       -> ties to the smallest column, then row; NaN never wins; matrixlu.jl:46-87),
//   (3) in launches of their own (no cross-XCD hand-off inside a kernel): the candidates'
//       reduction and stop test (matrixlu.jl:360-365) in one 1024-thread workgroup, then the
//       row/column swap over the whole matrix (swaprow!/swapcol!, matrixlu.jl:254-275), one
//       thread per row / column, publishing the new pivot column / row.
// Per pivot that is one read+write of the trailing block (32 B/element) -- HBM-bound like the
// Float64 rank-1 update (2x the bytes of the real case; 8 flops/element).
// Julia Base arithmetic restated: ComplexF64 `/` is Baudin & Smith's robust division and
// abs(z) = hypot(re, im) (base/complex.jl, base/math.jl; not under /root/reference), identical
// to oracle/tci_oracle.c (orc_cdiv / orc_hypot) bit for bit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tci_internal.h"

namespace tci {
namespace {

#ifndef TCI_C128_NT
#define TCI_C128_NT 0  // non-temporal stores of the updated trailing block (A/B switch)
#endif
constexpr int kCTR = 64;      // rows per tile (one wave lane per row)
constexpr int kCTC = 32;      // columns per tile (4 waves x 8 columns)
constexpr int kCThreads = 256;
constexpr int kCW = kCTC / (kCThreads / 64);  // columns per wave
constexpr int kRThreads = 1024;               // candidate reduction

__device__ inline bool cbetter(const CCand& b, const CCand& a) {
    return b.v > a.v || (b.v == a.v && (b.col < a.col || (b.col == a.col && b.row < a.row)));
}

__device__ inline void jl_cdiv2(double a, double b, double c, double d, double r, double t,
                                double* out) {
    if (r != 0) {
        double br = b * r;
        *out = (br != 0) ? (a + br) * t : a * t + (b * t) * r;
    } else {
        *out = (a + d * (b / c)) * t;
    }
}

__device__ inline double2 jl_cdiv(double2 z, double2 w) {
    double a = z.x, b = z.y, c = w.x, d = w.y;
    const double absa = fabs(a), absb = fabs(b), ab = absa >= absb ? absa : absb;
    const double absc = fabs(c), absd = fabs(d), cd = absc >= absd ? absc : absd;
    const double halfov = 0.5 * 1.7976931348623157e308;
    const double twounE = 2.2250738585072014e-308 * 2.0 / 2.220446049250313e-16;
    const double bs = 2.0 / (2.220446049250313e-16 * 2.220446049250313e-16);
    double s = 1.0, p, q;
    if (ab >= halfov) { a *= 0.5; b *= 0.5; s *= 2.0; }
    if (cd >= halfov) { c *= 0.5; d *= 0.5; s *= 0.5; }
    if (ab <= twounE) { a *= bs; b *= bs; s /= bs; }
    if (cd <= twounE) { c *= bs; d *= bs; s *= bs; }
    if (absd <= absc) {
        const double r = d / c, t = 1.0 / (c + d * r);
        jl_cdiv2(a, b, c, d, r, t, &p);
        jl_cdiv2(b, -a, c, d, r, t, &q);
    } else {
        const double r = c / d, t = 1.0 / (d + c * r);
        jl_cdiv2(b, a, d, c, r, t, &p);
        jl_cdiv2(a, -b, d, c, r, t, &q);
        q = -q;
    }
    return make_double2(p * s, q * s);
}

__device__ inline double jl_hypot(double x, double y) {
    if (isinf(x) || isinf(y)) return INFINITY;
    double ax = fabs(x), ay = fabs(y);
    if (ay > ax) { double t = ax; ax = ay; ay = t; }
    if (isnan(ax) || isnan(ay)) return ax + ay;
    if (ay <= ax * sqrt(2.220446049250313e-16 / 2)) return ax;
    double scale = 2.220446049250313e-16 * sqrt(2.2250738585072014e-308);
    if (ax > sqrt(1.7976931348623157e308 / 2)) {
        ax *= scale; ay *= scale; scale = 1.0 / scale;
    } else if (ay < sqrt(2.2250738585072014e-308)) {
        ax /= scale; ay /= scale;
    } else {
        scale = 1.0;
    }
    double h = sqrt(fma(ax, ax, ay * ay));
    const double hsq = h * h, axsq = ax * ax;
    h -= (fma(-ay, ay, hsq - axsq) + fma(h, h, -hsq) - fma(ax, ax, -axsq)) / (2 * h);
    return h * scale;
}

__device__ inline double jl_maxd(double x, double y) {  // Base.max: NaN-propagating
    if (x != x || y != y) return NAN;
    return x > y ? x : y;
}

__device__ inline double2 cmul(double2 x, double2 y) {
    return make_double2(x.x * y.x - x.y * y.y, x.x * y.y + x.y * y.x);
}

__device__ inline CCand shfl_cand(const CCand& c, int mask) {
    CCand o;
    o.v = __shfl_xor(c.v, mask);
    o.col = __shfl_xor(c.col, mask);
    o.row = __shfl_xor(c.row, mask);
    return o;
}

// block-wide argmax; the result is valid in every thread
template <int NT>
__device__ CCand block_reduce(CCand c, CCand* sh) {
    for (int mask = 32; mask >= 1; mask >>= 1) {
        CCand o = shfl_cand(c, mask);
        if (cbetter(o, c)) c = o;
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = c;
    __syncthreads();
    c = sh[0];
    for (int i = 1; i < NT / 64; ++i)
        if (cbetter(sh[i], c)) c = sh[i];
    return c;
}

__global__ void k_crrlu_init(CState* st, int64_t* rowperm, int64_t* colperm, int m, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        st->np = 0;
        st->done = 0;
        st->nan = 0;
        st->maxerror = 0.0;
        st->err = NAN;
    }
    if (i < m) rowperm[i] = i;  // 0-based here; the ABI returns them 1-based
    if (i < n) colperm[i] = i;
}

__global__ __launch_bounds__(kCThreads) void k_crrlu_step(CStepArgs g) {
    __shared__ double2 xs[kCTR];
    __shared__ double2 ys[kCTC];
    __shared__ CCand red[kCThreads / 64];
    CState* st = g.st;
    if (st->done) return;  // set by an earlier launch only
    const int t = g.t;
    const int tiles_r = g.tiles_r;
    const int tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
    const int r0 = t + tr * kCTR, c0 = t + tc * kCTC;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double2* A = g.A;
    const int64_t ld = g.ld;

    // (1) rank-1 update of pivot k = t - 1 from the published buffers
    if (t > 0) {
        const int k = t - 1;
        const double2 piv = st->piv;
        if (threadIdx.x < kCTR) {
            const int i = r0 + threadIdx.x;
            if (i < g.m) {
                double2 x = g.colbuf[i];
                if (g.leftorth) {
                    x = jl_cdiv(x, piv);
                    if (tc == 0) A[i + (int64_t)k * ld] = x;  // A[k+1:end, k] ./= A[k, k]
                }
                xs[threadIdx.x] = x;
            }
        } else if (threadIdx.x < kCTR + kCTC) {
            const int j = c0 + threadIdx.x - kCTR;
            if (j < g.n) {
                double2 y = g.rowbuf[j];
                if (!g.leftorth) {
                    y = jl_cdiv(y, piv);
                    if (tr == 0) A[k + (int64_t)j * ld] = y;  // A[k, k+1:end] ./= A[k, k]
                }
                ys[threadIdx.x - kCTR] = y;
            }
        }
        __syncthreads();
    }
    CCand best{-INFINITY, INT32_MAX, INT32_MAX};
    const int i = r0 + lane;
    if (i < g.m) {
#pragma unroll
        for (int cc = 0; cc < kCW; ++cc) {
            const int jl = w * kCW + cc;
            const int j = c0 + jl;
            if (j >= g.n) break;
            double2* pa = A + i + (int64_t)j * ld;
            double2 a = *pa;
            if (t > 0) {
                const double2 z = cmul(xs[lane], ys[jl]);
                a.x = a.x - z.x;
                a.y = a.y - z.y;
#if TCI_C128_NT
                typedef double dv2 __attribute__((ext_vector_type(2)));
                dv2 wv = {a.x, a.y};
                __builtin_nontemporal_store(wv, reinterpret_cast<dv2*>(pa));
#else
                *pa = a;
#endif
            }
            const double v = a.x * a.x + a.y * a.y;
            if (v > best.v) best = CCand{v, j, i};  // columns ascend: strict '>' keeps the first
        }
    }
    if (t < g.mr) {
        best = block_reduce<kCThreads>(best, red);
        if (threadIdx.x == 0) g.cand[blockIdx.x] = best;
    }
}

// (3a) one workgroup (a launch of its own, so every store of the step is visible): reduce the
// candidates, stop test (matrixlu.jl:360-365), permutation swap; the winner goes to st->p/q
__global__ __launch_bounds__(kRThreads) void k_crrlu_reduce(CStepArgs g, int ncand) {
    __shared__ CCand red[kRThreads / 64];
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t;
    CCand c{-INFINITY, INT32_MAX, INT32_MAX};
    int b = threadIdx.x;
    for (; b + 7 * kRThreads < ncand; b += 8 * kRThreads) {  // 8 independent loads in flight
        CCand o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = g.cand[b + u * kRThreads];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (cbetter(o[u], c)) c = o[u];
    }
    for (; b < ncand; b += kRThreads) {
        const CCand o = g.cand[b];
        if (cbetter(o, c)) c = o;
    }
    c = block_reduce<kRThreads>(c, red);  // (v, col, row) is a total order: any order reduces
    if (threadIdx.x == 0) {
        const int p = c.col == INT32_MAX ? t : c.row;  // nothing beat -Inf (all NaN): (k, k)
        const int q = c.col == INT32_MAX ? t : c.col;
        const double2 a = g.A[p + (int64_t)q * g.ld];
        const double err = jl_hypot(a.x, a.y);  // lu.error = abs(A[p, q])
        st->err = err;
        if ((err < g.reltol * st->maxerror || err < g.abstol) && t > 0) {
            st->done = 1;
        } else {
            st->maxerror = jl_maxd(st->maxerror, err);
            st->np = t + 1;
            st->p = p;
            st->q = q;
            int64_t tmp = g.rowperm[t]; g.rowperm[t] = g.rowperm[p]; g.rowperm[p] = tmp;
            tmp = g.colperm[t]; g.colperm[t] = g.colperm[q]; g.colperm[q] = tmp;
        }
    }
}

// (3b) swaprow!(t, p) and swapcol!(t, q) (matrixlu.jl:254-275) over disjoint element sets, one
// thread per column (row swap), per row (column swap) and one for the 2x2 corner
// {t,p} x {t,q}: new[a, b] = old[sr(a), sc(b)]; publishes the new pivot column / row
__global__ void k_crrlu_swap(CStepArgs g) {
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t, p = st->p, q = st->q;
    double2* A = g.A;
    const int64_t ld = g.ld;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < g.n) {
        const int j = e;
        if (j == t || j == q) return;
        double2* pt = A + t + (int64_t)j * ld;
        double2* pp = A + p + (int64_t)j * ld;
        const double2 at = *pt, ap = *pp;
        *pt = ap;
        *pp = at;
        g.rowbuf[j] = ap;
    } else if (e < g.n + g.m) {
        const int r = e - g.n;
        if (r == t || r == p) return;
        double2* pt = A + r + (int64_t)t * ld;
        double2* pq = A + r + (int64_t)q * ld;
        const double2 at = *pt, aq = *pq;
        *pt = aq;
        *pq = at;
        g.colbuf[r] = aq;
    } else if (e == g.n + g.m) {
        const double2 o_tt = A[t + (int64_t)t * ld], o_tq = A[t + (int64_t)q * ld];
        const double2 o_pt = A[p + (int64_t)t * ld], o_pq = A[p + (int64_t)q * ld];
        A[t + (int64_t)t * ld] = o_pq;
        A[t + (int64_t)q * ld] = o_pt;
        A[p + (int64_t)t * ld] = o_tq;
        A[p + (int64_t)q * ld] = o_tt;
        // re-read: with p == t or q == t the four stores alias and the last one wins consistently
        const double2 n_tt = A[t + (int64_t)t * ld];
        g.rowbuf[t] = n_tt;
        g.rowbuf[q] = A[t + (int64_t)q * ld];
        g.colbuf[t] = n_tt;
        g.colbuf[p] = A[p + (int64_t)t * ld];
        st->piv = n_tt;
    }
}

// L = tril(A[:, 1:np]), U = triu(A[1:np, :]), NaN flags (1: L, 2: U) before the unit diagonal
// is set, pivot errors abs.(diag) (matrixlu.jl:372-388, 799)
__global__ void k_crrlu_extract(const double2* A, int64_t ld, int m, int n, int np, int leftorth,
                                double2* L, double2* U, int64_t ldu, double* pe, int* nanflag) {
    const int64_t nl = (int64_t)m * np, nu = (int64_t)np * n;
    int flag = 0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nl + nu;
         e += (int64_t)gridDim.x * blockDim.x) {
        if (e < nl) {
            const int r = (int)(e % m), c = (int)(e / m);
            double2 a = r >= c ? A[r + (int64_t)c * ld] : make_double2(0.0, 0.0);
            if (isnan(a.x) || isnan(a.y)) flag |= 1;
            if (r == c && leftorth) a = make_double2(1.0, 0.0);
            if (L) L[e] = a;
            if (r == c && pe) pe[c] = jl_hypot(A[r + (int64_t)c * ld].x, A[r + (int64_t)c * ld].y);
        } else {
            const int64_t f = e - nl;
            const int r = (int)(f % np), c = (int)(f / np);
            double2 a = r <= c ? A[r + (int64_t)c * ld] : make_double2(0.0, 0.0);
            if (isnan(a.x) || isnan(a.y)) flag |= 2;
            if (r == c && !leftorth) a = make_double2(1.0, 0.0);
            if (U) U[r + (int64_t)c * ldu] = a;
        }
    }
    if (flag) atomicOr(nanflag, flag);
}

// MatrixLUCI{ComplexF64} factors (matrixluci.jl:161-283), one thread per output row (left) /
// column (right) with the oracle's loop order: TRSM rows solved last column first, GEMM sums in
// ascending t. L: m x np (ld m, unit diagonal if leftorth), U: np x n (ld np).
__global__ void k_cluci_left(const double2* __restrict__ L, const double2* __restrict__ U, int m,
                             int np, int leftorth, const int64_t* __restrict__ rowperm,
                             double2* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double2* o = out + rowperm[i];
    for (int j = np - 1; j >= 0; --j) {
        double2 s = make_double2(0.0, 0.0);
        if (leftorth) {  // [I; L21 / LowerTriangular(L11)]
            if (i < np) {
                s.x = (i == j) ? 1.0 : 0.0;
            } else {
                s = L[i + (int64_t)j * m];
                for (int t = j + 1; t < np; ++t) {
                    const double2 z = cmul(o[(int64_t)t * m], L[t + (int64_t)j * m]);
                    s.x = s.x - z.x;
                    s.y = s.y - z.y;
                }
                s = jl_cdiv(s, L[j + (int64_t)j * m]);
            }
        } else {  // colmatrix: L * U11
            for (int t = 0; t < np; ++t) {
                const double2 z = cmul(L[i + (int64_t)t * m], U[t + (int64_t)j * np]);
                s.x = s.x + z.x;
                s.y = s.y + z.y;
            }
        }
        o[(int64_t)j * m] = s;
    }
}

__global__ void k_cluci_right(const double2* __restrict__ L, const double2* __restrict__ U, int m,
                              int n, int np, int leftorth, const int64_t* __restrict__ colperm,
                              double2* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    double2* o = out + (int64_t)np * colperm[c];
    for (int a = np - 1; a >= 0; --a) {
        double2 s = make_double2(0.0, 0.0);
        if (!leftorth) {  // [I, UpperTriangular(U11) \ U12]
            if (c < np) {
                s.x = (a == c) ? 1.0 : 0.0;
            } else {
                s = U[a + (int64_t)c * np];
                for (int t = a + 1; t < np; ++t) {
                    const double2 z = cmul(U[a + (int64_t)t * np], o[t]);
                    s.x = s.x - z.x;
                    s.y = s.y - z.y;
                }
                s = jl_cdiv(s, U[a + (int64_t)a * np]);
            }
        } else {  // rowmatrix: L11 * U
            for (int t = 0; t < np; ++t) {
                const double2 z = cmul(L[a + (int64_t)t * m], U[t + (int64_t)c * np]);
                s.x = s.x + z.x;
                s.y = s.y + z.y;
            }
        }
        o[a] = s;
    }
}

// Pi = coeff * f (ComplexF64 evaluator over a real device integrand) and max|Pi| (Julia's abs =
// hypot; NaN propagates through the bit-pattern max like Base.max, util.jl:34-43)
__global__ void k_c128_scale(const double* __restrict__ re, int64_t ldr, int m, int n, double cre,
                             double cim, double2* __restrict__ out, int64_t ldo,
                             unsigned long long* maxbits) {
    const int64_t tot = (int64_t)m * n;
    double mx = 0.0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e % m), j = (int)(e / m);
        const double x = re[i + (int64_t)j * ldr];
        const double2 z = make_double2(cre * x, cim * x);
        out[i + (int64_t)j * ldo] = z;
        const double a = jl_hypot(z.x, z.y);
        mx = (a != a || a > mx) ? a : mx;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        const double v = __shfl_xor(mx, o);
        mx = (v != v || v > mx) ? v : mx;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxbits, (unsigned long long)__double_as_longlong(mx));
}

// T = Pi1 * P^-1 for ComplexF64 (setsitetensor!, tensorci2.jl:620-627: transpose(transpose(P) \
// transpose(Pi1))): getrf of A = P^T with partial pivoting (LAPACK's pivot: first maximal
// cabs1 = |re| + |im|), one 1024-thread workgroup, A in global memory (r x r).
__global__ __launch_bounds__(1024) void k_cgetrf_T(const double2* __restrict__ P, int r,
                                                   double2* __restrict__ A, int* __restrict__ piv) {
    __shared__ double sv[16];
    __shared__ int si[16];
    __shared__ int sp;
    const int tid = threadIdx.x;
    for (int64_t e = tid; e < (int64_t)r * r; e += 1024) {  // A[i, j] = P[j, i]
        const int i = (int)(e % r), j = (int)(e / r);
        A[e] = P[j + (int64_t)i * r];
    }
    __syncthreads();
    for (int k = 0; k < r; ++k) {
        double bv = -1.0;
        int bi = INT32_MAX;
        for (int i = k + tid; i < r; i += 1024) {
            const double2 a = A[i + (int64_t)k * r];
            const double v = fabs(a.x) + fabs(a.y);
            if (v > bv) { bv = v; bi = i; }
        }
        for (int o = 32; o >= 1; o >>= 1) {
            const double ov = __shfl_xor(bv, o);
            const int oi = __shfl_xor(bi, o);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if ((tid & 63) == 0) { sv[tid >> 6] = bv; si[tid >> 6] = bi; }
        __syncthreads();
        if (tid == 0) {
            double v = sv[0];
            int ix = si[0];
            for (int w = 1; w < 16; ++w)
                if (sv[w] > v || (sv[w] == v && si[w] < ix)) { v = sv[w]; ix = si[w]; }
            sp = ix == INT32_MAX ? k : ix;
            piv[k] = sp;
        }
        __syncthreads();
        const int p = sp;
        if (p != k)
            for (int j = tid; j < r; j += 1024) {
                const double2 t = A[k + (int64_t)j * r];
                A[k + (int64_t)j * r] = A[p + (int64_t)j * r];
                A[p + (int64_t)j * r] = t;
            }
        __syncthreads();
        const double2 d = A[k + (int64_t)k * r];
        for (int i = k + 1 + tid; i < r; i += 1024) A[i + (int64_t)k * r] = jl_cdiv(A[i + (int64_t)k * r], d);
        __syncthreads();
        const int nt = r - k - 1;
        for (int64_t e = tid; e < (int64_t)nt * nt; e += 1024) {
            const int i = k + 1 + (int)(e % nt), j = k + 1 + (int)(e / nt);
            const double2 z = cmul(A[i + (int64_t)k * r], A[k + (int64_t)j * r]);
            double2 a = A[i + (int64_t)j * r];
            a.x = a.x - z.x;
            a.y = a.y - z.y;
            A[i + (int64_t)j * r] = a;
        }
        __syncthreads();
    }
}

// getrs: one thread per right-hand side b = Pi1[q, :]^T; x = T[q, :]
__global__ void k_cgetrs_rows(const double2* __restrict__ A, const int* __restrict__ piv, int r,
                              const double2* __restrict__ Pi1, int R, double2* __restrict__ T) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= R) return;
    double2* x = T + q;  // x[i] at T[q + i * R]
    for (int i = 0; i < r; ++i) x[(int64_t)i * R] = Pi1[q + (int64_t)i * R];
    for (int k = 0; k < r; ++k) {
        const int p = piv[k];
        if (p != k) {
            const double2 t = x[(int64_t)k * R];
            x[(int64_t)k * R] = x[(int64_t)p * R];
            x[(int64_t)p * R] = t;
        }
    }
    for (int i = 0; i < r; ++i) {  // unit lower
        double2 s = x[(int64_t)i * R];
        for (int t = 0; t < i; ++t) {
            const double2 z = cmul(A[i + (int64_t)t * r], x[(int64_t)t * R]);
            s.x = s.x - z.x;
            s.y = s.y - z.y;
        }
        x[(int64_t)i * R] = s;
    }
    for (int i = r - 1; i >= 0; --i) {  // upper
        double2 s = x[(int64_t)i * R];
        for (int t = i + 1; t < r; ++t) {
            const double2 z = cmul(A[i + (int64_t)t * r], x[(int64_t)t * R]);
            s.x = s.x - z.x;
            s.y = s.y - z.y;
        }
        x[(int64_t)i * R] = jl_cdiv(s, A[i + (int64_t)i * r]);
    }
}

// evaluate(tt, x) (abstracttensortrain.jl:328-342) for ComplexF64 cores: one workgroup per
// point, the running row vector in LDS (bond dimensions <= 1024)
__global__ __launch_bounds__(256) void k_ctt_eval(const double2* __restrict__ cores,
                                                  const int64_t* __restrict__ off,
                                                  const int32_t* __restrict__ bd,
                                                  const int32_t* __restrict__ dims, int L,
                                                  const int32_t* __restrict__ X, double2* out) {
    __shared__ double2 v[2][1024];
    const int pt = blockIdx.x;
    const int32_t* x = X + (int64_t)pt * L;
    if (threadIdx.x == 0) v[0][0] = make_double2(1.0, 0.0);
    __syncthreads();
    int cur = 0;
    for (int p = 0; p < L; ++p) {
        const int ra = bd[p], rb = bd[p + 1], d = dims[p];
        const double2* Tp = cores + off[p] + (int64_t)(x[p] - 1) * ra;  // T[:, x, :], ld ra * d
        for (int b = threadIdx.x; b < rb; b += 256) {
            double2 s = make_double2(0.0, 0.0);
            for (int a = 0; a < ra; ++a) {
                const double2 z = cmul(v[cur][a], Tp[a + (int64_t)b * ra * d]);
                s.x = s.x + z.x;
                s.y = s.y + z.y;
            }
            v[cur ^ 1][b] = s;
        }
        __syncthreads();
        cur ^= 1;
    }
    if (threadIdx.x == 0) out[pt] = v[cur][0];
}


// ------------------------------------------------ deferred updates
// The trailing block stays stale in HBM between write-backs; up to nb rank-1 updates pend as
// per-row x_s (X[s][i]) and per-column y_s (Y[s][j]) and are applied on the fly, in pivot order
// and with the reference's rounding (complex multiply, then componentwise subtract), so every
// value is bitwise the reference's. Swaps stay physical: the swap kernel moves the pending
// entries of the two rows / columns with them. It also finalises pivot t's column and row
// (stale values minus the pending updates, normalised) into A -- the L / U storage of the
// reference -- and into pending slot P.
template <int P, bool FLUSH>
__global__ __launch_bounds__(kCThreads) void k_crrlu_step_d(CStepArgs g) {
    __shared__ double2 ys[(P > 0 ? P : 1) * kCTC];
    __shared__ CCand red[kCThreads / 64];
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t;
    const int tiles_r = g.tiles_r;
    const int tr = blockIdx.x % tiles_r, tc = blockIdx.x / tiles_r;
    const int r0 = t + tr * kCTR, c0 = t + tc * kCTC;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double2* A = g.A;
    const int64_t ld = g.ld;
    const int i = r0 + lane;
    double2 xr[P > 0 ? P : 1];
    if constexpr (P > 0) {
        for (int e = threadIdx.x; e < P * kCTC; e += kCThreads) {
            const int s = e / kCTC, jl = e % kCTC, j = c0 + jl;
            ys[e] = j < g.n ? g.Y[(int64_t)s * g.ldy + j] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int s = 0; s < P; ++s) xr[s] = i < g.m ? g.X[(int64_t)s * g.ldx + i] : make_double2(0.0, 0.0);
        __syncthreads();
    }
    CCand best{-INFINITY, INT32_MAX, INT32_MAX};
    if (i < g.m) {
#pragma unroll
        for (int cc = 0; cc < kCW; ++cc) {
            const int jl = w * kCW + cc;
            const int j = c0 + jl;
            if (j >= g.n) break;
            double2* pa = A + i + (int64_t)j * ld;
            double2 a = *pa;
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(xr[s], ys[s * kCTC + jl]);
                a.x = a.x - z.x;
                a.y = a.y - z.y;
            }
            if constexpr (FLUSH) *pa = a;
            const double v = a.x * a.x + a.y * a.y;
            if (v > best.v) best = CCand{v, j, i};  // columns ascend: strict '>' keeps the first
        }
    }
    best = block_reduce<kCThreads>(best, red);
    if (threadIdx.x == 0) g.cand[blockIdx.x] = best;
}

// value of stale element (r, c) with the P pending updates applied, in pivot order
__device__ inline double2 cpend(double2 a, const double2* X, int64_t ldx, int r, const double2* Y,
                                int64_t ldy, int c, int P) {
    for (int s = 0; s < P; ++s) {
        const double2 z = cmul(X[(int64_t)s * ldx + r], Y[(int64_t)s * ldy + c]);
        a.x = a.x - z.x;
        a.y = a.y - z.y;
    }
    return a;
}

__global__ __launch_bounds__(kRThreads) void k_crrlu_reduce_d(CStepArgs g, int ncand) {
    __shared__ CCand red[kRThreads / 64];
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t, P = g.P;
    CCand c{-INFINITY, INT32_MAX, INT32_MAX};
    int b = threadIdx.x;
    for (; b + 7 * kRThreads < ncand; b += 8 * kRThreads) {
        CCand o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = g.cand[b + u * kRThreads];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (cbetter(o[u], c)) c = o[u];
    }
    for (; b < ncand; b += kRThreads) {
        const CCand o = g.cand[b];
        if (cbetter(o, c)) c = o;
    }
    c = block_reduce<kRThreads>(c, red);
    const int p = c.col == INT32_MAX ? t : c.row;  // nothing beat -Inf (all NaN): (k, k)
    const int q = c.col == INT32_MAX ? t : c.col;
    // the slots of the rows / columns the swap exchanges, for the swap kernel (see CStepArgs)
    if (threadIdx.x < P) {
        const int s = threadIdx.x;
        g.stash[s] = g.X[(int64_t)s * g.ldx + t];
        g.stash[kMaxPend + s] = g.X[(int64_t)s * g.ldx + p];
        g.stash[2 * kMaxPend + s] = g.Y[(int64_t)s * g.ldy + t];
        g.stash[3 * kMaxPend + s] = g.Y[(int64_t)s * g.ldy + q];
    }
    if (threadIdx.x == 0) {
        const double2 a = cpend(g.A[p + (int64_t)q * g.ld], g.X, g.ldx, p, g.Y, g.ldy, q, P);
        const double err = jl_hypot(a.x, a.y);  // lu.error = abs(A[p, q])
        st->err = err;
        if ((err < g.reltol * st->maxerror || err < g.abstol) && t > 0) {
            st->done = 1;
        } else {
            st->maxerror = jl_maxd(st->maxerror, err);
            st->np = t + 1;
            st->p = p;
            st->q = q;
            st->piv = a;
            int64_t tmp = g.rowperm[t]; g.rowperm[t] = g.rowperm[p]; g.rowperm[p] = tmp;
            tmp = g.colperm[t]; g.colperm[t] = g.colperm[q]; g.colperm[q] = tmp;
        }
    }
}

// swaprow!(t, p), swapcol!(t, q) of the stale matrix and of the pending slots; pivot t's row
// (columns > t) and column (rows > t) finalised: pending updates applied, normalised by the
// pivot (matrixlu.jl:302-308), stored into A and into slot P. Threads: one per column (row swap),
// per row (column swap), one for the 2 x 2 corner {t, p} x {t, q}.
__global__ void k_crrlu_swap_d(CStepArgs g) {
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t, p = st->p, q = st->q, P = g.P;
    const double2 piv = st->piv;
    double2* A = g.A;
    const int64_t ld = g.ld;
    const double2* sXt = g.stash;                 // X[s][t] before the swap
    const double2* sXp = g.stash + kMaxPend;      // X[s][p]
    const double2* sYt = g.stash + 2 * kMaxPend;  // Y[s][t]
    const double2* sYq = g.stash + 3 * kMaxPend;  // Y[s][q]
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < g.n) {  // column j: rows t <-> p
        const int j = e;
        if (j == t || j == q) return;
        double2* pt = A + t + (int64_t)j * ld;
        double2* pp = A + p + (int64_t)j * ld;
        const double2 at = *pt, ap = *pp;
        *pp = at;
        if (j < t) {
            *pt = ap;  // the L part: final values
        } else {  // U row t: the new row t is old row p, pending updates with old row p's x's
            double2 y = ap;
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(sXp[s], g.Y[(int64_t)s * g.ldy + j]);
                y.x = y.x - z.x;
                y.y = y.y - z.y;
            }
            if (!g.leftorth) y = jl_cdiv(y, piv);  // A[k, k+1:end] ./= A[k, k]
            *pt = y;
            g.Y[(int64_t)P * g.ldy + j] = y;
        }
    } else if (e < g.n + g.m) {  // row r: columns t <-> q
        const int r = e - g.n;
        if (r == t || r == p) return;
        double2* pt = A + r + (int64_t)t * ld;
        double2* pq = A + r + (int64_t)q * ld;
        const double2 at = *pt, aq = *pq;
        *pq = at;
        if (r < t) {
            *pt = aq;  // the U part
        } else {
            double2 x = aq;
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(g.X[(int64_t)s * g.ldx + r], sYq[s]);
                x.x = x.x - z.x;
                x.y = x.y - z.y;
            }
            if (g.leftorth) x = jl_cdiv(x, piv);  // A[k+1:end, k] ./= A[k, k]
            *pt = x;
            g.X[(int64_t)P * g.ldx + r] = x;
        }
    } else if (e == g.n + g.m) {
        // new[a, b] = old[sr(a), sc(b)] on {t, p} x {t, q}, all read before any store
        const double2 o_tt = A[t + (int64_t)t * ld], o_tq = A[t + (int64_t)q * ld];
        const double2 o_pt = A[p + (int64_t)t * ld];
        A[t + (int64_t)t * ld] = piv;  // (t, t): the pivot, updated (reduce computed it)
        if (q != t) {  // (t, q): row t = old row p, column q = old column t -> U element
            double2 y = o_pt;
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(sXp[s], sYt[s]);
                y.x = y.x - z.x;
                y.y = y.y - z.y;
            }
            if (!g.leftorth) y = jl_cdiv(y, piv);
            A[t + (int64_t)q * ld] = y;
            g.Y[(int64_t)P * g.ldy + q] = y;
        }
        if (p != t) {  // (p, t): row p = old row t, column t = old column q -> L element
            double2 x = o_tq;
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(sXt[s], sYq[s]);
                x.x = x.x - z.x;
                x.y = x.y - z.y;
            }
            if (g.leftorth) x = jl_cdiv(x, piv);
            A[p + (int64_t)t * ld] = x;
            g.X[(int64_t)P * g.ldx + p] = x;
        }
        if (p != t && q != t) A[p + (int64_t)q * ld] = o_tt;  // (p, q): trailing, stays stale
        // the pending slots follow their rows / columns
        for (int s = 0; s < P; ++s) {
            g.X[(int64_t)s * g.ldx + t] = sXp[s];
            g.X[(int64_t)s * g.ldx + p] = sXt[s];
            g.Y[(int64_t)s * g.ldy + t] = sYq[s];
            g.Y[(int64_t)s * g.ldy + q] = sYt[s];
        }
    }
}

template <int P>
static void crrlu_step_p(hipStream_t s, const CStepArgs& g, bool flush, int grid) {
    if (flush) hipLaunchKernelGGL((k_crrlu_step_d<P, true>), dim3(grid), dim3(kCThreads), 0, s, g);
    else hipLaunchKernelGGL((k_crrlu_step_d<P, false>), dim3(grid), dim3(kCThreads), 0, s, g);
}

}  // namespace

int crrlu_grid(int m, int n, int t) {
    const int tr = m - t > 0 ? (m - t + kCTR - 1) / kCTR : 1;
    const int tc = n - t > 0 ? (n - t + kCTC - 1) / kCTC : 1;
    return tr * tc;
}

void launch_crrlu_init(hipStream_t s, CState* st, int64_t* rowperm, int64_t* colperm, int m,
                       int n) {
    const int N = m > n ? m : n;
    k_crrlu_init<<<(N + 255) / 256 + 1, 256, 0, s>>>(st, rowperm, colperm, m, n);
}

void launch_crrlu_step(hipStream_t s, CStepArgs g) {
    g.tiles_r = g.m - g.t > 0 ? (g.m - g.t + kCTR - 1) / kCTR : 1;
    const int grid = crrlu_grid(g.m, g.n, g.t);
    k_crrlu_step<<<grid, kCThreads, 0, s>>>(g);
    if (g.t < g.mr) {
        k_crrlu_reduce<<<1, kRThreads, 0, s>>>(g, grid);
        k_crrlu_swap<<<(g.m + g.n + 256) / 256, 256, 0, s>>>(g);
    }
}

// step<P, flush> for pivot t, then (t < mr) reduce + swap with the step's pending count after it
void launch_crrlu_step_d(hipStream_t s, CStepArgs g, int P, bool flush) {
    g.tiles_r = g.m - g.t > 0 ? (g.m - g.t + kCTR - 1) / kCTR : 1;
    const int grid = crrlu_grid(g.m, g.n, g.t);
    switch (P) {
#define TCI_CSTEP(p) \
    case p: crrlu_step_p<p>(s, g, flush, grid); break;
        TCI_CSTEP(0) TCI_CSTEP(1) TCI_CSTEP(2) TCI_CSTEP(3) TCI_CSTEP(4) TCI_CSTEP(5) TCI_CSTEP(6)
        TCI_CSTEP(7) TCI_CSTEP(8) TCI_CSTEP(9) TCI_CSTEP(10) TCI_CSTEP(11) TCI_CSTEP(12) TCI_CSTEP(13)
        TCI_CSTEP(14) TCI_CSTEP(15)
#undef TCI_CSTEP
    default: break;
    }
    g.P = flush ? 0 : P;
    hipLaunchKernelGGL(k_crrlu_reduce_d, dim3(1), dim3(kRThreads), 0, s, g, grid);
    hipLaunchKernelGGL(k_crrlu_swap_d, dim3((g.m + g.n + 256) / 256), dim3(256), 0, s, g);
}

void launch_crrlu_extract(hipStream_t s, const double2* A, int64_t ld, int m, int n, int np,
                          int leftorth, double2* L, double2* U, int64_t ldu, double* pe,
                          int* nanflag) {
    const int64_t tot = (int64_t)m * np + (int64_t)np * n;
    int grid = (int)((tot + 255) / 256);
    if (grid < 1) grid = 1;
    if (grid > 4096) grid = 4096;
    k_crrlu_extract<<<grid, 256, 0, s>>>(A, ld, m, n, np, leftorth, L, U, ldu, pe, nanflag);
}

void launch_c128_scale(hipStream_t s, const double* re, int64_t ldr, int m, int n, double cre,
                       double cim, double2* out, int64_t ldo, unsigned long long* maxbits) {
    const int64_t tot = (int64_t)m * n;
    int grid = (int)((tot + 255) / 256);
    if (grid < 1) grid = 1;
    if (grid > 8192) grid = 8192;
    k_c128_scale<<<grid, 256, 0, s>>>(re, ldr, m, n, cre, cim, out, ldo, maxbits);
}

void launch_csitetensor_solve(hipStream_t s, const double2* P, int r, const double2* Pi1, int R,
                              double2* T, double2* work, int* piv) {
    k_cgetrf_T<<<1, 1024, 0, s>>>(P, r, work, piv);
    k_cgetrs_rows<<<(R + 63) / 64, 64, 0, s>>>(work, piv, r, Pi1, R, T);
}

void launch_ctt_eval(hipStream_t s, const double2* cores, const int64_t* off, const int32_t* bd,
                     const int32_t* dims, int L, const int32_t* X, int npts, double2* out) {
    if (npts > 0) k_ctt_eval<<<npts, 256, 0, s>>>(cores, off, bd, dims, L, X, out);
}

void launch_cluci_factors(hipStream_t s, const double2* L, const double2* U, int m, int n, int np,
                          int leftorth, const int64_t* rowperm, const int64_t* colperm,
                          double2* left, double2* right) {
    if (left) k_cluci_left<<<(m + 63) / 64, 64, 0, s>>>(L, U, m, np, leftorth, rowperm, left);
    if (right) k_cluci_right<<<(n + 63) / 64, 64, 0, s>>>(L, U, m, n, np, leftorth, colperm, right);
}

}  // namespace tci
