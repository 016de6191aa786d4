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
#include <stdio.h>

#include <type_traits>

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

// ------------------------------------------------ shadow search helpers
constexpr int kCShK = 64;  // split slots per row / column plane: 6 per pending update, P <= 10

__device__ inline uint16_t f16_bits(double v) {
    const _Float16 h = (_Float16)(float)v;
    return __builtin_bit_cast(uint16_t, h);
}

// scale of an epoch whose stale values have modulus <= B: s = 2^(14 - ilogb B), so the real and
// imaginary parts stay below 2^15 in fp16; 0 (search off) outside [2^-100, 2^100] or not finite
__device__ inline double c_sh_scale(double B) {
    if (!(B >= 0x1p-100 && B <= 0x1p100)) return 0.0;
    return ldexp(1.0, 14 - ilogb(B));
}

// bound on the stale values' modulus of the epoch whose first pending pivot is t0: A itself
// (|pivot 0| is its maximum) or the Schur complement after t0 - 1 (a - x y, each <= |pivot t0-1|)
__device__ inline double c_sh_bound(const double* pm, int t0) {
    return t0 == 0 ? pm[0] : 2.0 * pm[t0 - 1];
}

// f16 split of v (v = hi + lo to ~2^-22)
__device__ inline void c_split(double v, uint16_t& hi, uint16_t& lo) {
    const _Float16 h = (_Float16)(float)v;
    const _Float16 l = (_Float16)(float)(v - (double)h);
    hi = __builtin_bit_cast(uint16_t, h);
    lo = __builtin_bit_cast(uint16_t, l);
}

// fragment slots 6 slot .. 6 slot + 5 of pending update `slot`: row side -(x) (scaled unless
// leftorth) as (xr_h, xr_h, xr_l, xi_h, xi_h, xi_l); column side y (scaled if leftorth) as
// re-plane (yr_h, yr_l, yr_h, -yi_h, -yi_l, -yi_h) and im-plane (yi_h, yi_l, yi_h, yr_h, yr_l, yr_h):
// sum over the slots of A * B_re = Re(-x y), A * B_im = Im(-x y)
__device__ inline void c_frag_x(uint16_t* XA, int r, int slot, double2 x, double s, int leftorth) {
    if (slot >= kCShK / 6) return;
    const double xr = -(leftorth ? x.x : x.x * s), xi = -(leftorth ? x.y : x.y * s);
    uint16_t rh, rl, ih, il;
    c_split(xr, rh, rl);
    c_split(xi, ih, il);
    uint16_t* d = XA + (int64_t)r * kCShK + 6 * slot;
    d[0] = rh; d[1] = rh; d[2] = rl; d[3] = ih; d[4] = ih; d[5] = il;
}

__device__ inline void c_frag_y(uint16_t* YB, int c, int slot, double2 y, double s, int leftorth) {
    if (slot >= kCShK / 6) return;
    const double yr = leftorth ? y.x * s : y.x, yi = leftorth ? y.y * s : y.y;
    uint16_t rh, rl, ih, il, nih, nil;
    c_split(yr, rh, rl);
    c_split(yi, ih, il);
    c_split(-yi, nih, nil);
    uint16_t* d = YB + (int64_t)c * 2 * kCShK + 6 * slot;
    d[0] = rh; d[1] = rl; d[2] = rh; d[3] = nih; d[4] = nil; d[5] = nih;
    d += kCShK;
    d[0] = ih; d[1] = il; d[2] = ih; d[3] = rh; d[4] = rl; d[5] = rh;
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

// A ComplexF64 integrand given as real parts (TCI_F_C128, tci_func_create_c128): the real value
// of one part added into the real (comp 0) or imaginary (comp 1) component of the complex Pi ...
__global__ void k_c128_accum(const double* __restrict__ re, int64_t ldr, int m, int n, int comp,
                             double2* __restrict__ out, int64_t ldo) {
    const int64_t tot = (int64_t)m * n;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e % m), j = (int)(e / m);
        double2 z = out[i + (int64_t)j * ldo];
        const double x = re[i + (int64_t)j * ldr];
        if (comp) z.y = z.y + x;
        else z.x = z.x + x;
        out[i + (int64_t)j * ldo] = z;
    }
}

// ... then the coefficient (complex multiply, no fma) and max|.| (abs = hypot, NaN-propagating)
__global__ void k_c128_finish(int m, int n, double cre, double cim, double2* __restrict__ out,
                              int64_t ldo, unsigned long long* maxbits) {
    const int64_t tot = (int64_t)m * n;
    double mx = 0.0;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e % m), j = (int)(e / m);
        const double2 w = out[i + (int64_t)j * ldo];
        const double2 z = make_double2(__dsub_rn(__dmul_rn(cre, w.x), __dmul_rn(cim, w.y)),
                                       __dadd_rn(__dmul_rn(cre, w.y), __dmul_rn(cim, w.x)));
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
// SHW (shadow search): 1 = a write-back that also writes the fp16 shadow of the new stale values
// and clears the MFMA fragments of the epoch it starts; 2 = step 1, which writes the shadow of A's
// stale values (epoch 0: its scale needs |pivot 0|)
template <int P, bool FLUSH, int SHW = 0>
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
    [[maybe_unused]] double shs = 0.0;
    if constexpr (SHW != 0) {
        shs = c_sh_scale(SHW == 1 ? 2.0 * g.pmod[t - 1] : g.pmod[0]);
        if (SHW == 1) {  // fragments of the epoch starting here: every slot zero
            constexpr int RQ = kCShK / 8, CQ = 2 * kCShK / 8;  // 16-B stores per row / column
            for (int e = threadIdx.x; e < kCTR * RQ; e += kCThreads)
                if (tc == 0 && r0 + e / RQ < g.m)
                    reinterpret_cast<uint4*>(g.XA + (int64_t)(r0 + e / RQ) * kCShK)[e % RQ] = uint4{0, 0, 0, 0};
            for (int e = threadIdx.x; e < kCTC * CQ; e += kCThreads)
                if (tr == 0 && c0 + e / CQ < g.n)
                    reinterpret_cast<uint4*>(g.YB + (int64_t)(c0 + e / CQ) * 2 * kCShK)[e % CQ] = uint4{0, 0, 0, 0};
        }
    }
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
            if constexpr (SHW == 2) {
                g.SR[i + (int64_t)j * g.lds] = f16_bits(a.x * shs);
                g.SI[i + (int64_t)j * g.lds] = f16_bits(a.y * shs);
            }
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(xr[s], ys[s * kCTC + jl]);
                a.x = a.x - z.x;
                a.y = a.y - z.y;
            }
            if constexpr (FLUSH) *pa = a;
            if constexpr (SHW == 1) {
                g.SR[i + (int64_t)j * g.lds] = f16_bits(a.x * shs);
                g.SI[i + (int64_t)j * g.lds] = f16_bits(a.y * shs);
            }
            const double v = a.x * a.x + a.y * a.y;
            if (v > best.v) best = CCand{v, j, i};  // columns ascend: strict '>' keeps the first
        }
    }
    best = block_reduce<kCThreads>(best, red);
    if (threadIdx.x == 0) g.cand[blockIdx.x] = best;
}

// value of stale element (r, c) with the P pending updates applied, in pivot order (all the
// slots' loads in flight at once, then the chain: P is a runtime count here)
__device__ inline double2 cpend(double2 a, const double2* X, int64_t ldx, int r, const double2* Y,
                                int64_t ldy, int c, int P) {
    double2 xv[kMaxPend], yv[kMaxPend];
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            xv[s] = X[(int64_t)s * ldx + r];
            yv[s] = Y[(int64_t)s * ldy + c];
        }
    }
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            const double2 z = cmul(xv[s], yv[s]);
            a.x = a.x - z.x;
            a.y = a.y - z.y;
        }
    }
    return a;
}

// a - sum_s x_s * ys[s * ld], x_s from a short array (the stash), same order and rounding
__device__ inline double2 cpend_xs(double2 a, const double2* xs, const double2* Y, int64_t ldy, int c, int P) {
    double2 xv[kMaxPend], yv[kMaxPend];
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            xv[s] = xs[s];
            yv[s] = Y[(int64_t)s * ldy + c];
        }
    }
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            const double2 z = cmul(xv[s], yv[s]);
            a.x = a.x - z.x;
            a.y = a.y - z.y;
        }
    }
    return a;
}

// a - sum_s X[s * ldx + r] * ys_s, the y's from a short array
__device__ inline double2 cpend_ys(double2 a, const double2* X, int64_t ldx, int r, const double2* ys, int P) {
    double2 xv[kMaxPend], yv[kMaxPend];
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            xv[s] = X[(int64_t)s * ldx + r];
            yv[s] = ys[s];
        }
    }
#pragma unroll
    for (int s = 0; s < kMaxPend; ++s) {
        if (s < P) {
            const double2 z = cmul(xv[s], yv[s]);
            a.x = a.x - z.x;
            a.y = a.y - z.y;
        }
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
            if (g.pmod) g.pmod[t] = err;
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
    // shadow search: the epoch's scale for the fragments of the new pending slot P (pivot t)
    const double fs = g.sh ? c_sh_scale(c_sh_bound(g.pmod, t - P)) : 0.0;
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
            double2 y = cpend_xs(ap, sXp, g.Y, g.ldy, j, P);
            if (!g.leftorth) y = jl_cdiv(y, piv);  // A[k, k+1:end] ./= A[k, k]
            *pt = y;
            g.Y[(int64_t)P * g.ldy + j] = y;
            if (g.sh) {
                c_frag_y(g.YB, j, P, y, fs, g.leftorth);
                if (p != t) {  // the shadow's row p takes old row t (column q: the corner)
                    g.SR[p + (int64_t)j * g.lds] = g.SR[t + (int64_t)j * g.lds];
                    g.SI[p + (int64_t)j * g.lds] = g.SI[t + (int64_t)j * g.lds];
                }
            }
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
            double2 x = cpend_ys(aq, g.X, g.ldx, r, sYq, P);
            if (g.leftorth) x = jl_cdiv(x, piv);  // A[k+1:end, k] ./= A[k, k]
            *pt = x;
            g.X[(int64_t)P * g.ldx + r] = x;
            if (g.sh) {
                c_frag_x(g.XA, r, P, x, fs, g.leftorth);
                if (q != t) {  // the shadow's column q takes old column t
                    g.SR[r + (int64_t)q * g.lds] = g.SR[r + (int64_t)t * g.lds];
                    g.SI[r + (int64_t)q * g.lds] = g.SI[r + (int64_t)t * g.lds];
                }
            }
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
        if (g.sh) {
            // shadow corner (p, q) = old (t, t); the fragments of rows t / p and columns t / q
            // follow them like the slots, then pivot t's own entries of row p / column q
            if (p != t && q != t) {
                g.SR[p + (int64_t)q * g.lds] = g.SR[t + (int64_t)t * g.lds];
                g.SI[p + (int64_t)q * g.lds] = g.SI[t + (int64_t)t * g.lds];
            }
            if (p != t) {
                uint4* ft = reinterpret_cast<uint4*>(g.XA + (int64_t)t * kCShK);
                uint4* fp = reinterpret_cast<uint4*>(g.XA + (int64_t)p * kCShK);
                for (int z = 0; z < kCShK / 8; ++z) {
                    const uint4 u = ft[z];
                    ft[z] = fp[z];
                    fp[z] = u;
                }
                c_frag_x(g.XA, p, P, A[p + (int64_t)t * ld], fs, g.leftorth);
            }
            if (q != t) {
                uint4* ft = reinterpret_cast<uint4*>(g.YB + (int64_t)t * 2 * kCShK);
                uint4* fq = reinterpret_cast<uint4*>(g.YB + (int64_t)q * 2 * kCShK);
                for (int z = 0; z < 2 * kCShK / 8; ++z) {
                    const uint4 u = ft[z];
                    ft[z] = fq[z];
                    fq[z] = u;
                }
                c_frag_y(g.YB, q, P, A[t + (int64_t)q * ld], fs, g.leftorth);
            }
        }
    }
}


// ------------------------------------------------ certified shadow search
// Read-only step t with P pending updates (1 <= P <= 5): instead of the 16-B complex values it
// streams the fp16 planes of their real and imaginary parts (4 B/element) and applies the
// pending updates on the matrix cores: per 16 x 16 tile two v_mfma_f32_16x16x32_f16 with the
// same A fragment (the rows' -x splits) and the columns' B fragments of Re and Im (6 slots per
// update, see c_frag_x / c_frag_y), C = the converted shadow tiles. With |v| <= Mf (the epoch's
// stale bound) every part of W is within epsc of s * v, the fp32 modulus within epsm of s |v|:
//   fp16 storage 2^-11 (1 + 2^-9) s Mf + 2^-25, splits 2^-18 s sumM + 2P 2^-24,
//   fp32 accumulation (6P + 4) 2^-23 s (Mf + 2 sumM);  epsm = sqrt(2) epsc + 2^-21 s mag.
// Blocks (4 rows x 1 column) whose approximate maximum can reach the workgroup's lower bound are
// re-read in fp64 and examined exactly (the reference's operations and tie order), deferred to a
// per-wave list and pruned against the latest bound. Rows and columns before t (the L / U part
// of the physically swapped matrix) are masked by position. Workgroup: 64 rows x 512 columns,
// 4 waves taking 16-column chunks.
// Geometry (the Float64 k_pass_mf's): one 1024-thread workgroup per CU owns a 512-row tile
// (8 slices of 64 rows, 2 waves per slice; the A fragments of a wave's slice stay in registers)
// and the 16-column chunks q, q + nq, ... of the trailing columns, staged 32 chunks at a time:
// the chunks' B fragments (built by the swaps, YB) are copied into LDS once per workgroup, so
// they cost ~0.5 B per element instead of one 256-B load per 64-row tile and column.
#ifndef TCI_CSH_DBG
#define TCI_CSH_DBG 0
#endif
#ifndef TCI_CSH_TAU_SLICE
#define TCI_CSH_TAU_SLICE 0
#endif
#ifndef TCI_CSH_GB
#define TCI_CSH_GB 0  // debug: B fragments from global memory instead of LDS
#endif
#ifndef TCI_CSH_ALL
#define TCI_CSH_ALL 0  // debug: examine every element exactly
#endif
#ifndef TCI_CSH_REPS
#define TCI_CSH_REPS 1  // waves per 64-row slice of the complex shadow step (2: 1024 threads, spills; measured 34.6 vs 38.9 ms)
#endif
constexpr int kCSSlices = 8, kCSReps = TCI_CSH_REPS, kCSThreads = 64 * kCSSlices * kCSReps, kCSGroup = 32,
              kCSExCap = 64;
typedef _Float16 ch8 __attribute__((ext_vector_type(8)));
typedef float cf4 __attribute__((ext_vector_type(4)));

template <int P>
__global__ __launch_bounds__(kCSThreads) void k_crrlu_step_sh(CStepArgs g) {
    static_assert(P >= 1 && P <= kCShMaxP && 6 * kCShMaxP <= kCShK, "6P split slots");
    constexpr int NK = (6 * P + 31) / 32;  // MFMAs (K = 32) per tile and plane
    constexpr int BS = 2 * NK * 4 + 1;     // ch8 per staged column: [plane][u][row quad], padded
    constexpr int GR = NK == 1 ? kCSGroup : kCSGroup / 2;  // chunks staged at once
    __shared__ ch8 lb[GR * 16 * BS];
    __shared__ unsigned tau_sl[kCSSlices];
    __shared__ unsigned exl[kCSThreads / 64 * kCSExCap];
    __shared__ float exm[kCSThreads / 64 * kCSExCap];
    __shared__ CCand red[kCSThreads / 64];
    CState* st = g.st;
    if (st->done) return;
    const int t = g.t, m = g.m, n = g.n, t0 = t - P;
    const double* pm = g.pmod;
    const double shs = c_sh_scale(c_sh_bound(pm, t0));
    const double Mf = pm[t0];
    double sumM = 0.0, maxM = 0.0;
#pragma unroll
    for (int s = 0; s < P; ++s) {
        sumM += pm[t0 + s];
        maxM = fmax(maxM, pm[t0 + s]);
    }
    const double mag = Mf + 2.0 * sumM;
    const double epsc = 0x1p-11 * (1.0 + 0x1p-9) * Mf * shs + 0x1p-25 + 0x1p-18 * sumM * shs +
                        2.0 * P * 0x1p-24 + (6.0 * P + 4.0) * 0x1p-23 * mag * shs;
    const double epsd = 1.4142135623730951 * (1.0 + 0x1p-20) * epsc + 0x1p-21 * mag * shs;
    const bool shok = shs > 0.0 && mag < 0x1p100 && maxM * shs <= 0x1p15 &&
                      epsd < ldexp(pm[t - 1] * shs, -7);
    const int rb0 = t & ~15, cb0 = t & ~15;
    const int tiles_r = (m - rb0 + 511) / 512;
    const int nck = (n - cb0 + 15) / 16;
    const int nq = gridDim.x / tiles_r;
    const int tr = blockIdx.x % tiles_r, q = blockIdx.x / tiles_r;
    const int myck = q < nck ? (nck - 1 - q) / nq + 1 : 0;  // chunks q, q + nq, ...
    const int r0 = rb0 + 512 * tr;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slice = wave % kCSSlices, rep = wave / kCSSlices;
#if TCI_CSH_TAU_SLICE
    unsigned& tau_s = tau_sl[slice];  // debug: the lower bound shared by a slice's waves only
#else
    unsigned& tau_s = tau_sl[0];
#endif
    const double2* A = g.A;
    const int64_t ld = g.ld;
    CCand best{-INFINITY, INT32_MAX, INT32_MAX};
    // exact value of element (i, j): the stale value minus the pending updates in pivot order.
    // FAST: every slot's loads in flight at once (no streaming registers live); otherwise one
    // slot at a time (a full list mid-stream)
    auto exact = [&](int i, int j, auto fast) {
        double2 a = A[i + (int64_t)j * ld];
        if constexpr (decltype(fast)::value) {
            double2 xv[P], yv[P];
#pragma unroll
            for (int s = 0; s < P; ++s) {
                xv[s] = g.X[(int64_t)s * g.ldx + i];
                yv[s] = g.Y[(int64_t)s * g.ldy + j];
            }
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(xv[s], yv[s]);
                a.x = a.x - z.x;
                a.y = a.y - z.y;
            }
        } else {
#pragma unroll 1
            for (int s = 0; s < P; ++s) {
                const double2 z = cmul(g.X[(int64_t)s * g.ldx + i], g.Y[(int64_t)s * g.ldy + j]);
                a.x = a.x - z.x;
                a.y = a.y - z.y;
            }
        }
        const CCand c{a.x * a.x + a.y * a.y, j, i};
#if TCI_CSH_DBG
        if (t >= 7 && t <= 8 && j == t + 2)
            printf("[dbg-exact t=%d] i=%d j=%d v=%.17g best=(%.17g,%d,%d)\n", t, i, j, c.v, best.v, best.col, best.row);
#endif
        if (cbetter(c, best)) best = c;
    };
    if (!shok) {
        // the bound is not tight (decaying pivots) or fp16 could overflow: every element exactly
        for (int ci = 0; ci < myck; ++ci) {
            const int cj = cb0 + 16 * (q + nq * ci);
            for (int e = threadIdx.x; e < 512 * 16; e += kCSThreads) {
                const int i = r0 + (e & 511), j = cj + (e >> 9);
                if (i >= t && i < m && j >= t && j < n) exact(i, j, std::true_type{});
            }
        }
    } else {
        const float eps = TCI_CSH_ALL ? 1e30f : (float)(epsd * (1.0 + 0x1p-20));
        const float margin = 0x1p-20f;
        const int gq = lane >> 4, lcol = lane & 15;
        const int sb = r0 + 64 * slice;  // the wave's slice
        const int rl = sb + 16 * gq;     // the lane's 16 loaded rows
        const bool rload = rl < g.lds;
        const bool rmask = __any(rl < t);  // rows before t in the wave: masked per element
        ch8 af[4][NK];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int rho = sb + 16 * (lcol >> 2) + 4 * b + (lcol & 3);
#pragma unroll
            for (int u = 0; u < NK; ++u)
                af[b][u] = rho < m ? *reinterpret_cast<const ch8*>(g.XA + (int64_t)rho * kCShK + 32 * u + 8 * gq)
                                   : ch8{};
        }
        bool act = false;
        for (int z = 0; z < 16; ++z) act |= (rl + z >= t && rl + z < m);
        const bool wact = __any(act);
        const _Float16* SR = reinterpret_cast<const _Float16*>(g.SR);
        const _Float16* SI = reinterpret_cast<const _Float16*>(g.SI);
        auto colof = [&](int ci) { return cb0 + 16 * (q + nq * ci) + lcol; };  // chunk ci, this lane
        auto load = [&](int ci, ch8 (&vr)[2], ch8 (&vi)[2]) {
            const int j = colof(ci);
            if (rload && j < n) {
                const ch8* pr = reinterpret_cast<const ch8*>(SR + rl + (int64_t)j * g.lds);
                const ch8* pi = reinterpret_cast<const ch8*>(SI + rl + (int64_t)j * g.lds);
                vr[0] = pr[0];
                vr[1] = pr[1];
                vi[0] = pi[0];
                vi[1] = pi[1];
            } else {
                vr[0] = vr[1] = vi[0] = vi[1] = ch8{};
            }
        };
        // chunk ci (local li in the staged group): the lane's column's maximum modulus over its 16
        // rows, per 4-row block (-1: not a trailing column)
        auto approx = [&](int ci, int li, const ch8 (&vr)[2], const ch8 (&vi)[2], float (&mbs)[4]) -> float {
            const int j = colof(ci);
            const bool jok = j >= t && j < n;
            const ch8* lp = lb + (li * 16 + lcol) * BS;
            ch8 bre[NK], bim[NK];
#pragma unroll
            for (int u = 0; u < NK; ++u) {
#if TCI_CSH_GB
                const int jj = j < n ? j : 0;
                bre[u] = *reinterpret_cast<const ch8*>(g.YB + (int64_t)jj * 2 * kCShK + 32 * u + 8 * gq);
                bim[u] = *reinterpret_cast<const ch8*>(g.YB + (int64_t)jj * 2 * kCShK + kCShK + 32 * u + 8 * gq);
#else
                bre[u] = lp[u * 4 + gq];
                bim[u] = lp[NK * 4 + u * 4 + gq];
#endif
            }
            float c = 0.0f;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int o = 4 * (b & 1);
                const ch8& hr = vr[b >> 1];
                const ch8& hi = vi[b >> 1];
                cf4 dr = {(float)hr[o], (float)hr[o + 1], (float)hr[o + 2], (float)hr[o + 3]};
                cf4 di = {(float)hi[o], (float)hi[o + 1], (float)hi[o + 2], (float)hi[o + 3]};
#pragma unroll
                for (int u = 0; u < NK; ++u) {
                    dr = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[b][u], bre[u], dr, 0, 0, 0);
                    di = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[b][u], bim[u], di, 0, 0, 0);
                }
                float q2[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) q2[e] = dr[e] * dr[e] + di[e] * di[e];
                if (rmask) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (rl + 4 * b + e < t) q2[e] = 0.0f;
                }
                mbs[b] = sqrtf(__builtin_fmaxf(__builtin_fmaxf(q2[0], q2[1]), __builtin_fmaxf(q2[2], q2[3])));
                c = __builtin_fmaxf(c, mbs[b]);
            }
            if (!jok) {
#pragma unroll
                for (int b = 0; b < 4; ++b) mbs[b] = -1.0f;
                c = -1.0f;
            }
#if TCI_CSH_DBG
            if (t >= 7 && t <= 8 && j == t + 2 && rl <= t + 2 && t + 2 < rl + 16)
                printf("[dbg t=%d wg=%d wave=%d lane=%d] j=%d rl=%d mbs %g %g %g %g c=%g eps=%g shs=%g\n", t,
                       (int)blockIdx.x, wave, lane, j, rl, mbs[0], mbs[1], mbs[2], mbs[3], c, eps, shs);
#endif
            return c;
        };
        float tau = 0.0f;
        unsigned* const wl = exl + wave * kCSExCap;
        float* const wm = exm + wave * kCSExCap;
        int nex = 0;
        auto flush = [&](auto fast) {
            const float thr = tau - tau * margin;
            for (int e = lane; e < 4 * nex; e += 64) {
                if (wm[e >> 2] + eps < thr) continue;
                const unsigned key = wl[e >> 2];
                const int j = (int)(key & 0xffffffu), i = sb + 4 * (int)(key >> 24) + (e & 3);
#if TCI_CSH_DBG
                if (t >= 7 && t <= 8 && j == t + 2 && i >= t && i < t + 30)
                    printf("[dbg-flush t=%d wg=%d wave=%d lane=%d] e=%d nex=%d i=%d j=%d wm=%g thr=%g\n", t, (int)blockIdx.x,
                           wave, lane, e, nex, i, j, wm[e >> 2], thr);
#endif
                if (i >= t && i < m) exact(i, j, fast);
            }
            nex = 0;
        };
        auto append = [&](int ci, const float (&mbs)[4], float bound) {
            const int j = colof(ci);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const bool f = mbs[b] >= 0.0f && mbs[b] + eps >= bound;
                const uint64_t bal = __ballot(f);
                if (bal == 0) continue;
                const int cnt = __popcll(bal);
                if (nex + cnt > kCSExCap) flush(std::false_type{});
                if (f) {
                    const int at = nex + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                    wl[at] = (unsigned)j | (unsigned)(4 * gq + b) << 24;
                    wm[at] = mbs[b];
                }
                nex += cnt;
            }
        };
        auto test = [&](float c) {
            if (c < 0.0f) return;
            const float lbd = fmaxf(c - eps, 0.0f);
            const float ts = __uint_as_float(__hip_atomic_load(&tau_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));  // slice
            tau = fmaxf(tau, ts);
            if (lbd > tau) {
                tau = lbd;
                atomicMax(&tau_s, __float_as_uint(lbd));
            }
        };
        ch8 ar[2], ai[2], br[2], bi[2];
        float mb0[4], mb1[4];
        for (int g0 = 0; g0 < myck; g0 += GR) {
            const int gn = min(GR, myck - g0);
            int h0 = g0 + rep, h1 = g0 + rep + kCSReps;  // this wave's chunks: rep, rep + 2, ...
            if (wact) {
                if (h0 < g0 + gn) load(h0, ar, ai);
                if (h1 < g0 + gn) load(h1, br, bi);
            }
            if (g0 > 0) __syncthreads();  // the previous group's readers are done with lb
            // stage the group's B fragments: one column per thread (16 B loads)
            if (threadIdx.x < gn * 16) {
                const int li = threadIdx.x >> 4, c = threadIdx.x & 15;
                const int j = cb0 + 16 * (q + nq * (g0 + li)) + c;
                const ch8* src = reinterpret_cast<const ch8*>(g.YB + (int64_t)(j < n ? j : 0) * 2 * kCShK);
                ch8* dst = lb + (li * 16 + c) * BS;
#pragma unroll
                for (int pl = 0; pl < 2; ++pl)
#pragma unroll
                    for (int z = 0; z < NK * 4; ++z) dst[pl * NK * 4 + z] = j < n ? src[pl * 8 + z] : ch8{};
            }
            if (g0 == 0 && threadIdx.x < kCSSlices) tau_sl[threadIdx.x] = 0u;
            __syncthreads();
            if (g0 == 0) {
                // seed: every wave's first chunk sets the workgroup's bound before anything is listed
                float c0 = -1.0f;
#pragma unroll
                for (int b = 0; b < 4; ++b) mb0[b] = -1.0f;
                const int e0 = h0;
                if (wact && h0 < g0 + gn) {
                    c0 = approx(h0, h0 - g0, ar, ai, mb0);
                    h0 += 2 * kCSReps;
                    if (h0 < g0 + gn) load(h0, ar, ai);
                    float lbd = fmaxf(c0 - eps, 0.0f);
#pragma unroll
                    for (int off = 32; off >= 1; off >>= 1) lbd = fmaxf(lbd, __shfl_xor(lbd, off));
                    if (lane == 0) atomicMax(&tau_s, __float_as_uint(lbd));
                }
                __syncthreads();
                tau = __uint_as_float(tau_s);
                // wave-uniform call: the list length nex must stay the same in every lane (lanes
                // of non-trailing columns carry mb0 = -1 and append nothing)
                if (wact) append(e0, mb0, tau - tau * margin);
            }
            if (!wact) continue;
            // h0's values in ar/ai, h1's in br/bi; the next chunk is always the smaller index
            for (;;) {
                if (h1 < h0) {
                    if (h1 >= g0 + gn) break;
                    const float c = approx(h1, h1 - g0, br, bi, mb1);
                    const int e = h1;
                    h1 += 2 * kCSReps;
                    if (h1 < g0 + gn) load(h1, br, bi);
                    test(c);
                    append(e, mb1, tau - tau * margin);
                } else {
                    if (h0 >= g0 + gn) break;
                    const float c = approx(h0, h0 - g0, ar, ai, mb0);
                    const int e = h0;
                    h0 += 2 * kCSReps;
                    if (h0 < g0 + gn) load(h0, ar, ai);
                    test(c);
                    append(e, mb0, tau - tau * margin);
                }
            }
        }
        tau = fmaxf(tau, __uint_as_float(__hip_atomic_load(&tau_s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
        flush(std::true_type{});
    }
    best = block_reduce<kCSThreads>(best, red);
    if (threadIdx.x == 0) g.cand[blockIdx.x] = best;
}

template <int P>
static void crrlu_step_p(hipStream_t s, const CStepArgs& g, bool flush, int grid) {
    if (flush && g.sh && P > 0)
        hipLaunchKernelGGL((k_crrlu_step_d<P, true, 1>), dim3(grid), dim3(kCThreads), 0, s, g);
    else if (flush)
        hipLaunchKernelGGL((k_crrlu_step_d<P, true>), dim3(grid), dim3(kCThreads), 0, s, g);
    else
        hipLaunchKernelGGL((k_crrlu_step_d<P, false>), dim3(grid), dim3(kCThreads), 0, s, g);
}

template <int P>
static void crrlu_step_sh_p(hipStream_t s, const CStepArgs& g, int grid) {
    if constexpr (P >= 1 && P <= kCShMaxP)
        hipLaunchKernelGGL((k_crrlu_step_sh<P>), dim3(grid), dim3(kCSThreads), 0, s, g);
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

int crrlu_sh_grid(int m, int n, int t) {
    const int rb0 = t & ~15;
    const int tiles_r = m - rb0 > 0 ? (m - rb0 + 511) / 512 : 1;
    const int nck = n - rb0 > 0 ? (n - rb0 + 15) / 16 : 1;
    int nq = 256 / tiles_r;  // one 1024-thread workgroup per CU
    if (nq > nck) nq = nck;
    if (nq < 1) nq = 1;
    return tiles_r * nq;
}

// shadow-search step for pivot t (P pending, 1..kCShMaxP), then reduce + swap (pending P after)
void launch_crrlu_step_sh(hipStream_t s, CStepArgs g, int P) {
    const int grid = crrlu_sh_grid(g.m, g.n, g.t);
    switch (P) {
        case 1: crrlu_step_sh_p<1>(s, g, grid); break;
        case 2: crrlu_step_sh_p<2>(s, g, grid); break;
        case 3: crrlu_step_sh_p<3>(s, g, grid); break;
        case 4: crrlu_step_sh_p<4>(s, g, grid); break;
        case 5: crrlu_step_sh_p<5>(s, g, grid); break;
        case 6: crrlu_step_sh_p<6>(s, g, grid); break;
        case 7: crrlu_step_sh_p<7>(s, g, grid); break;
        case 8: crrlu_step_sh_p<8>(s, g, grid); break;
        case 9: crrlu_step_sh_p<9>(s, g, grid); break;
        case 10: crrlu_step_sh_p<10>(s, g, grid); break;
        default: return;
    }
    g.P = P;
    hipLaunchKernelGGL(k_crrlu_reduce_d, dim3(1), dim3(kRThreads), 0, s, g, grid);
    hipLaunchKernelGGL(k_crrlu_swap_d, dim3((g.m + g.n + 256) / 256), dim3(256), 0, s, g);
}

// debug (env TCI_CSH_CHECK): the shadow step's winner against the exact step's, on the host
void debug_crrlu_check_sh(hipStream_t s, CStepArgs g, int P) {
    const int g1 = crrlu_sh_grid(g.m, g.n, g.t);
    switch (P) {
        case 1: crrlu_step_sh_p<1>(s, g, g1); break;
        case 2: crrlu_step_sh_p<2>(s, g, g1); break;
        case 3: crrlu_step_sh_p<3>(s, g, g1); break;
        case 4: crrlu_step_sh_p<4>(s, g, g1); break;
        case 5: crrlu_step_sh_p<5>(s, g, g1); break;
        case 6: crrlu_step_sh_p<6>(s, g, g1); break;
        case 7: crrlu_step_sh_p<7>(s, g, g1); break;
        case 8: crrlu_step_sh_p<8>(s, g, g1); break;
        case 9: crrlu_step_sh_p<9>(s, g, g1); break;
        case 10: crrlu_step_sh_p<10>(s, g, g1); break;
        default: return;
    }
    static CCand h1[1 << 16], h2[1 << 16];
    hipMemcpyAsync(h1, g.cand, sizeof(CCand) * g1, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    g.tiles_r = g.m - g.t > 0 ? (g.m - g.t + kCTR - 1) / kCTR : 1;
    const int g2 = crrlu_grid(g.m, g.n, g.t);
    switch (P) {
        case 1: crrlu_step_p<1>(s, g, false, g2); break;
        case 2: crrlu_step_p<2>(s, g, false, g2); break;
        case 3: crrlu_step_p<3>(s, g, false, g2); break;
        case 4: crrlu_step_p<4>(s, g, false, g2); break;
        case 5: crrlu_step_p<5>(s, g, false, g2); break;
        case 6: crrlu_step_p<6>(s, g, false, g2); break;
        case 7: crrlu_step_p<7>(s, g, false, g2); break;
        case 8: crrlu_step_p<8>(s, g, false, g2); break;
        case 9: crrlu_step_p<9>(s, g, false, g2); break;
        case 10: crrlu_step_p<10>(s, g, false, g2); break;
    }
    hipMemcpyAsync(h2, g.cand, sizeof(CCand) * g2, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    auto better = [](const CCand& b, const CCand& a) {
        return b.v > a.v || (b.v == a.v && (b.col < a.col || (b.col == a.col && b.row < a.row)));
    };
    CCand w1{-INFINITY, INT32_MAX, INT32_MAX}, w2 = w1;
    for (int i = 0; i < g1; ++i) if (better(h1[i], w1)) w1 = h1[i];
    for (int i = 0; i < g2; ++i) if (better(h2[i], w2)) w2 = h2[i];
    if (w1.v != w2.v || w1.col != w2.col || w1.row != w2.row) {
        printf("[csh-check] t=%d P=%d shadow (%.17g, col %d, row %d) exact (%.17g, col %d, row %d)\n", g.t, P,
               w1.v, w1.col, w1.row, w2.v, w2.col, w2.row);
        // the shadow step's candidates of the workgroups that hold the exact winner's column
        for (int i = 0; i < g1; ++i)
            if (h1[i].col / 16 == w2.col / 16) printf("   wg %d: (%.17g, col %d, row %d)\n", i, h1[i].v, h1[i].col, h1[i].row);
    }
    g.P = P;
    hipLaunchKernelGGL(k_crrlu_reduce_d, dim3(1), dim3(kRThreads), 0, s, g, g2);
    hipLaunchKernelGGL(k_crrlu_swap_d, dim3((g.m + g.n + 256) / 256), dim3(256), 0, s, g);
}

// step 1 of the shadow search: exact (one pending update), and it writes the shadow of the stale
// values with epoch 0's scale (|pivot 0|, known since step 0)
void launch_crrlu_step_stale_sh(hipStream_t s, CStepArgs g) {
    g.tiles_r = g.m - g.t > 0 ? (g.m - g.t + kCTR - 1) / kCTR : 1;
    const int grid = crrlu_grid(g.m, g.n, g.t);
    hipLaunchKernelGGL((k_crrlu_step_d<1, false, 2>), dim3(grid), dim3(kCThreads), 0, s, g);
    g.P = 1;
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

static int c128_grid(int64_t tot) {
    int64_t g = (tot + 255) / 256;
    return (int)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}

void launch_c128_accum(hipStream_t s, const double* re, int64_t ldr, int m, int n, int comp, double2* out,
                       int64_t ldo) {
    k_c128_accum<<<c128_grid((int64_t)m * n), 256, 0, s>>>(re, ldr, m, n, comp, out, ldo);
}

void launch_c128_finish(hipStream_t s, int m, int n, double cre, double cim, double2* out, int64_t ldo,
                        unsigned long long* maxbits) {
    k_c128_finish<<<c128_grid((int64_t)m * n), 256, 0, s>>>(m, n, cre, cim, out, ldo, maxbits);
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
