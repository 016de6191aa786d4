// tci_dense.hip -- fp64 dense linear algebra of the TCI2 path on v_mfma_f64_16x16x4f64 (gfx950):
//  K3  the blocked Schur-complement update C -= W * V (k_dgemm): the trailing update of a blocked
//      right-looking LU, and the GEMM of every blocked triangular solve below;
//  K4  MatrixLUCI factors (matrixluci.jl:161-241): the factor GEMMs (L11 * U, L * U11) and the
//      triangular solves (TRSMs at :207, :235) as diagonal-block solves + K3 updates;
//  K5  setsitetensor!'s solve T = Pi1 * P^-1 (tensorci2.jl:620-627, `transpose(P) \ transpose(Pi1)`):
//      a blocked right-looking getrf of P^T (partial pivoting; the panel factorised in LDS, the
//      trailing update on K3) and a blocked getrs whose off-diagonal work is K3.
// None of this is inside rrLU: exact full pivoting (matrixlu.jl:46-87) needs the fully updated
// trailing block before every pivot. Here the reference itself calls LAPACK / BLAS
// (Julia `\`, `*`), whose summation order it does not pin; parity is rtol 1e-12 (factors) /
// 1e-10 (solve) against the oracle's loop-order restatement.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "tci_internal.h"

namespace tci {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------ K3
// Out = beta * C + alpha * A * op(B):  A (m x k, ld lda), op(B) = B (k x n, ld ldb) or, with TB,
// B(t, j) = Bt[j + t * ldb] (Bt is n x k); C and Out column-major (Out may alias C); optional
// row / column maps put result (i, j) at Out[rmap[i] + cmap[j] * ldo].
// A workgroup of 4 waves owns a (32 FM) x (32 FN) tile, each wave a (16 FM) x (16 FN) block of
// FM x FN MFMA accumulators. k advances 16 at a time through two LDS buffers: the global loads
// of stage s + 1 are in flight while stage s runs on the matrix cores, one barrier per stage.
// The MFMA's A operand is fed from op(B) and its B operand from A, so the accumulator holds the
// transposed tile: lane l owns rows i = l & 15 (16 consecutive rows = a 128-B column segment per
// store) of four columns -- coalesced epilogue stores for column-major C.
constexpr int kDgKB = 16;

struct DgemmArgs {
    int m, n, k;
    double alpha, beta;
    const double* A;
    int64_t lda;
    const double* B;
    int64_t ldb;
    const double* C;
    int64_t ldc;
    double* Out;
    int64_t ldo;
    const int64_t* rmap;
    const int64_t* cmap;
    int tm, tn;  // tiles along m and n
    unsigned long long* maxbits;  // optional: atomicMax of |Out| bit patterns (Julia's NaN-propagating max)
};

template <int WM, int WN, int FM, int FN, bool TB>
__global__ __launch_bounds__(64 * WM * WN) void k_dgemm(DgemmArgs g) {
    constexpr int NT = 64 * WM * WN;
    constexpr int BM = WM * 16 * FM, BN = WN * 16 * FN;
    constexpr int LDA_S = BM + 8, LDB_S = BN + 8;  // padded rows against bank conflicts
    constexpr int QA = kDgKB * BM / NT, QB = kDgKB * BN / NT;
    __shared__ double As[2][kDgKB * LDA_S];
    __shared__ double Bs[2][kDgKB * LDB_S];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // XCD-aware tile order: consecutive workgroup ids go to different XCDs round-robin; give each
    // XCD a contiguous run of tiles (column-major over tiles: a run shares B's column panel)
    const int nt = g.tm * g.tn;
    int b = blockIdx.x;
    if ((nt & 7) == 0) b = (b & 7) * (nt >> 3) + (b >> 3);
    const int ti = b % g.tm, tj = b / g.tm;
    const int i0 = ti * BM, j0 = tj * BN;
    const int wr = (wv % WM) * 16 * FM, wc = (wv / WM) * 16 * FN;
    const int r = lane & 15, kk = lane >> 4;

    dbl4 acc[FM][FN];
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y) acc[x][y] = dbl4{0.0, 0.0, 0.0, 0.0};

    // staging coordinates are the same every stage: element (t, i) of the A stage and (t, j) of
    // the B stage; global addresses advance by 16 lda / 16 ldb (or 16) per stage
    double ra[QA], rb[QB];
    auto load = [&](int k0) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + q * NT, t = e / BM, i = e % BM;
            const int gi = i0 + i, gt = k0 + t;
            ra[q] = (gi < g.m && gt < g.k) ? g.A[(int64_t)gi + (int64_t)gt * g.lda] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int e = tid + q * NT;
            int t, j;
            if (TB) { t = e / BN; j = e % BN; }
            else { t = e % kDgKB; j = e / kDgKB; }
            const int gj = j0 + j, gt = k0 + t;
            double v = 0.0;
            if (gj < g.n && gt < g.k)
                v = TB ? g.B[(int64_t)gj + (int64_t)gt * g.ldb] : g.B[(int64_t)gt + (int64_t)gj * g.ldb];
            rb[q] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int e = tid + q * NT, t = e / BM, i = e % BM;
            As[buf][t * LDA_S + i] = ra[q];
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int e = tid + q * NT;
            int t, j;
            if (TB) { t = e / BN; j = e % BN; }
            else { t = e % kDgKB; j = e / kDgKB; }
            Bs[buf][t * LDB_S + j] = rb[q];
        }
    };

    const int nst = (g.k + kDgKB - 1) / kDgKB;
    load(0);
    // beta != 0 (the Schur update, the blocked solves' updates): the C tile's loads go out now,
    // so their latency hides behind the k loop instead of following it (at nb = 32-64 the C round
    // trip is most of the kernel)
    double cpre[FM][FN][4];
    const bool hasC = g.beta != 0.0;
    if (hasC) {
#pragma unroll
        for (int x = 0; x < FM; ++x) {
            const int i = i0 + wr + 16 * x + r;
#pragma unroll
            for (int y = 0; y < FN; ++y)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int j = j0 + wc + 16 * y + kk + 4 * q;
                    cpre[x][y][q] = (i < g.m && j < g.n) ? g.C[(int64_t)i + (int64_t)j * g.ldc] : 0.0;
                }
        }
    }
    store(0);
    __syncthreads();
    int cur = 0;
    for (int s = 0; s < nst; ++s) {
        if (s + 1 < nst) load((s + 1) * kDgKB);
        const double* as = As[cur];
        const double* bs = Bs[cur];
#pragma unroll
        for (int k4 = 0; k4 < kDgKB; k4 += 4) {
            double af[FM], bf[FN];
#pragma unroll
            for (int x = 0; x < FM; ++x) af[x] = as[(k4 + kk) * LDA_S + wr + 16 * x + r];
#pragma unroll
            for (int y = 0; y < FN; ++y) bf[y] = bs[(k4 + kk) * LDB_S + wc + 16 * y + r];
#pragma unroll
            for (int x = 0; x < FM; ++x)
#pragma unroll
                for (int y = 0; y < FN; ++y)
                    acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(bf[y], af[x], acc[x][y], 0, 0, 0);
        }
        if (s + 1 < nst) store(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }
    // acc[x][y][q]: row i = wr + 16x + (lane & 15), column j = wc + 16y + (lane >> 4) + 4q
    unsigned long long mb = 0;  // |v| bits: unsigned order = value order, +NaN above +Inf
#pragma unroll
    for (int x = 0; x < FM; ++x) {
        const int i = i0 + wr + 16 * x + r;
        if (i >= g.m) continue;
        const int64_t orow = g.rmap ? g.rmap[i] : i;
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = j0 + wc + 16 * y + kk + 4 * q;
                if (j >= g.n) continue;
                double v = g.alpha * acc[x][y][q];
                if (hasC) v = g.beta * cpre[x][y][q] + v;
                const int64_t ocol = g.cmap ? g.cmap[j] : j;
                g.Out[orow + ocol * g.ldo] = v;
                const unsigned long long b = (unsigned long long)__double_as_longlong(fabs(v));
                mb = b > mb ? b : mb;
            }
    }
    if (g.maxbits) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(mb, off);
            mb = o > mb ? o : mb;
        }
        if (lane == 0) atomicMax(g.maxbits, mb);
    }
}

// tile shapes: 128 x 128 (8 waves of 64 x 32), 128 x 64 (4 waves of 64 x 32), 64 x 64 (4 waves
// of 32 x 32); every form stays within 256 registers per lane so that two waves share a SIMD --
// the fp64 MFMA pipe needs two issuing waves per SIMD to reach its rate (tci_diag_mfma_f64_ex:
// 33.5 TF with one wave per SIMD, 72.4 TF with two)
// TCI_DGEMM_TILE (A/B only): 1 / 2 / 3 force 128 x 128 / 128 x 64 / 64 x 64
static int dgemm_tile_override() {
    static const int v = [] {
        const char* e = getenv("TCI_DGEMM_TILE");
        return e ? atoi(e) : 0;
    }();
    return v;
}

template <bool TB>
static void dgemm_go(hipStream_t s, DgemmArgs g) {
    const long long t128 = (long long)((g.m + 127) / 128) * ((g.n + 127) / 128);
    const long long t12864 = (long long)((g.m + 127) / 128) * ((g.n + 63) / 64);
    const long long t64 = (long long)((g.m + 63) / 64) * ((g.n + 63) / 64);
    int ov = dgemm_tile_override();
    // K <= 32 (a Schur update of depth 32, the getrs / TRSM updates of 32-wide blocks): the C round
    // trip dominates and four times as many 64 x 64 tiles keep more of it in flight (8192^2, nb 32:
    // 0.268 vs 0.289 ms, profiles/r04_s6_k3_tile*.json)
    if (ov == 0 && g.k <= 32 && t64 >= 1024) ov = 3;
    // n <= 64 (the getrs updates of 64-column blocks of T, R x 64 x jb): a 128-wide tile would run
    // half its MFMAs on zero padding; 64 x 64 tiles: the r = 1024, R = 32768 solve 8.97 -> 8.05 ms
    // (scripts/k5_tiles.sh, profiles/r06_m2_k5_tiles.txt)
    if (ov == 0 && g.n <= 64 && t64 >= 256) ov = 3;
    if (ov == 1 || (ov == 0 && t128 >= 256)) {
        g.tm = (g.m + 127) / 128;
        g.tn = (g.n + 127) / 128;
        hipLaunchKernelGGL((k_dgemm<2, 4, 4, 2, TB>), dim3(g.tm * g.tn), dim3(512), 0, s, g);
    } else if (ov == 2 || (ov == 0 && t12864 >= 256)) {
        g.tm = (g.m + 127) / 128;
        g.tn = (g.n + 63) / 64;
        hipLaunchKernelGGL((k_dgemm<2, 2, 4, 2, TB>), dim3(g.tm * g.tn), dim3(256), 0, s, g);
    } else {
        g.tm = (g.m + 63) / 64;
        g.tn = (g.n + 63) / 64;
        hipLaunchKernelGGL((k_dgemm<2, 2, 2, 2, TB>), dim3(g.tm * g.tn), dim3(256), 0, s, g);
    }
}

void launch_dgemm(hipStream_t s, bool tb, int m, int n, int k, double alpha, const double* A,
                  int64_t lda, const double* B, int64_t ldb, double beta, const double* C,
                  int64_t ldc, double* Out, int64_t ldo, const int64_t* rmap, const int64_t* cmap,
                  unsigned long long* maxbits) {
    if (m <= 0 || n <= 0) return;
    DgemmArgs g{m, n, k, alpha, beta, A, lda, B, ldb, C, ldc, Out ? Out : const_cast<double*>(C),
                Out ? ldo : ldc, rmap, cmap, 0, 0, maxbits};
    if (tb) dgemm_go<true>(s, g);
    else dgemm_go<false>(s, g);
}


// ------------------------------------------------------------- diagonal-block triangular solve
// For every right-hand side q < nrhs, the nb-vector x_q(j) = X[q * rs + j * es] (j < nb <= NB) is
// replaced by the solution of its nb x nb triangular system, M(j, t) = Mb[j * mj + t * mt]:
//   forward  (lower):  for t = 0, 1, ...:   x_t [/= M(t, t)];  x_j -= M(j, t) x_t  for j > t
//   backward (upper):  for t = nb-1, ...:   x_t [/= M(t, t)];  x_j -= M(j, t) x_t  for j < t
// (the column-oriented form of getrs's substitutions: the updates of one step are independent,
// so a thread's chain has NB-way instruction-level parallelism). One thread per right-hand side,
// x in registers, M in LDS (zero-padded past nb), separate multiply and subtract.
template <int NB, bool BACKWARD, bool UNIT>
__global__ __launch_bounds__(64) void k_trsm_diag(double* __restrict__ X, int64_t rs, int64_t es,
                                                  int nrhs, const double* __restrict__ Mb, int64_t mj,
                                                  int64_t mt, int nb) {
    // the forward solve runs as the backward one on reversed indices (j' = nb - 1 - j), so both
    // share one loop body (hipcc hoists every LDS read of a fully unrolled forward body and spills)
    __shared__ double Ms[NB * NB];  // Ms[t * NB + j] = M(j, t) in the backward numbering
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
        const int j = e % NB, t = e / NB;
        double v = j == t ? 1.0 : 0.0;
        if (j < nb && t < nb) {
            const int jj = BACKWARD ? j : nb - 1 - j, tt = BACKWARD ? t : nb - 1 - t;
            v = Mb[(int64_t)jj * mj + (int64_t)tt * mt];
        }
        Ms[e] = v;
    }
    __syncthreads();
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nrhs) return;
    double* xp = X + (int64_t)q * rs;
    double x[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) x[j] = j < nb ? xp[(int64_t)(BACKWARD ? j : nb - 1 - j) * es] : 0.0;
#pragma unroll
    for (int t = NB - 1; t >= 0; --t) {
        if (!UNIT) x[t] = x[t] / Ms[t * NB + t];
#pragma unroll
        for (int j = 0; j < t; ++j) x[j] = __dsub_rn(x[j], __dmul_rn(Ms[t * NB + j], x[t]));
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
        if (j < nb) xp[(int64_t)(BACKWARD ? j : nb - 1 - j) * es] = x[j];
}

constexpr int kDiagNB = 32;  // diagonal kernel width (x in 64 VGPRs)
constexpr int kTrsmNB = 64;  // block width of the blocked solves (the K3 depth of their updates)

static void trsm_diag32(hipStream_t s, double* X, int64_t rs, int64_t es, int nrhs, const double* Mb,
                        int64_t mj, int64_t mt, int nb, bool backward, bool unit) {
    if (nrhs <= 0 || nb <= 0) return;
    // 64-thread workgroups: the per-thread chains are long, spread them over every CU
    const dim3 grid((nrhs + 63) / 64), blk(64);
    if (backward && unit)
        hipLaunchKernelGGL((k_trsm_diag<kDiagNB, true, true>), grid, blk, 0, s, X, rs, es, nrhs, Mb, mj, mt, nb);
    else if (backward)
        hipLaunchKernelGGL((k_trsm_diag<kDiagNB, true, false>), grid, blk, 0, s, X, rs, es, nrhs, Mb, mj, mt, nb);
    else if (unit)
        hipLaunchKernelGGL((k_trsm_diag<kDiagNB, false, true>), grid, blk, 0, s, X, rs, es, nrhs, Mb, mj, mt, nb);
    else
        hipLaunchKernelGGL((k_trsm_diag<kDiagNB, false, false>), grid, blk, 0, s, X, rs, es, nrhs, Mb, mj, mt,
                           nb);
}

// A diagonal block of up to 64: two 32-wide diagonal solves and the K3 update between them.
// Either the right-hand sides are rows (rs == 1: X(q, j) = X[q + j es]) or columns (es == 1:
// X(q, j) = X[j + q rs]); M(j, t) = Mb[j mj + t mt] with mj == 1 or mt == 1.
static void trsm_diag(hipStream_t s, double* X, int64_t rs, int64_t es, int nrhs, const double* Mb,
                      int64_t mj, int64_t mt, int nb, bool backward, bool unit) {
    if (nb <= kDiagNB) {
        trsm_diag32(s, X, rs, es, nrhs, Mb, mj, mt, nb, backward, unit);
        return;
    }
    const int h = kDiagNB, nb2 = nb - h;
    const bool rows = rs == 1;
    double* X1 = X + (int64_t)h * es;  // second half
    if (!backward) {
        trsm_diag32(s, X, rs, es, nrhs, Mb, mj, mt, h, false, unit);
        // x_j -= sum_{t < h} M(j, t) x_t for j >= h
        const double* Mq = Mb + (int64_t)h * mj;  // M(h + j', t) = Mq[j' mj + t mt]
        if (rows) {
            if (mj == 1) launch_dgemm(s, true, nrhs, nb2, h, -1.0, X, es, Mq, mt, 1.0, X1, es, nullptr, 0, nullptr, nullptr);
            else launch_dgemm(s, false, nrhs, nb2, h, -1.0, X, es, Mq, mj, 1.0, X1, es, nullptr, 0, nullptr, nullptr);
        } else {  // C (nb2 x nrhs) = X1, A (j', t) = Mq (mj == 1, ld mt), B = X (h x nrhs, ld rs)
            launch_dgemm(s, false, nb2, nrhs, h, -1.0, Mq, mt, X, rs, 1.0, X1, rs, nullptr, 0, nullptr, nullptr);
        }
        trsm_diag32(s, X1, rs, es, nrhs, Mb + (int64_t)h * mj + (int64_t)h * mt, mj, mt, nb2, false, unit);
    } else {
        trsm_diag32(s, X1, rs, es, nrhs, Mb + (int64_t)h * mj + (int64_t)h * mt, mj, mt, nb2, true, unit);
        // x_j -= sum_{t >= h} M(j, t) x_t for j < h
        const double* Mq = Mb + (int64_t)h * mt;  // M(j, h + t') = Mq[j mj + t' mt]
        if (rows) {
            if (mj == 1) launch_dgemm(s, true, nrhs, h, nb2, -1.0, X1, es, Mq, mt, 1.0, X, es, nullptr, 0, nullptr, nullptr);
            else launch_dgemm(s, false, nrhs, h, nb2, -1.0, X1, es, Mq, mj, 1.0, X, es, nullptr, 0, nullptr, nullptr);
        } else {
            launch_dgemm(s, false, h, nrhs, nb2, -1.0, Mq, mt, X1, rs, 1.0, X, rs, nullptr, 0, nullptr, nullptr);
        }
        trsm_diag32(s, X, rs, es, nrhs, Mb, mj, mt, h, true, unit);
    }
}

// ------------------------------------------------------------------------ K4 MatrixLUCI factors
// leftorth: left = colstimespivotinv, i.e. X L11 = L21 (L11 unit lower; matrixluci.jl:194-213),
// solved in place over L's rows np..m-1, left-looking over 64-column blocks right to left: the
// K3 update X[:, jb:je] -= X[:, je:np] L11[je:np, jb:je] (K = np - je), then the diagonal block.
void trsm_luci_left(hipStream_t s, double* L, int64_t ldl, int m, int np) {
    const int rows = m - np;
    if (rows <= 0) return;
    double* X = L + np;
    for (int jb = ((np - 1) / kTrsmNB) * kTrsmNB; jb >= 0; jb -= kTrsmNB) {
        const int nb = std::min(kTrsmNB, np - jb), je = jb + nb;
        if (je < np)
            launch_dgemm(s, false, rows, nb, np - je, -1.0, X + (int64_t)je * ldl, ldl,
                         L + je + (int64_t)jb * ldl, ldl, 1.0, X + (int64_t)jb * ldl, ldl, nullptr, 0,
                         nullptr, nullptr);
        // x_j -= sum_{t > j} x_t L11[t, j]: M(j, t) = L[t + j ldl]
        trsm_diag(s, X + (int64_t)jb * ldl, 1, ldl, rows, L + jb + (int64_t)jb * ldl, ldl, 1, nb,
                  true, true);
    }
}

// !leftorth: right = pivotinvtimesrows, U11 X = U12 (U11 unit upper; matrixluci.jl:227-241), in
// place over U's columns np..n-1, diagonal blocks bottom to top, each followed by the K3 update
// of the rows above it: U12[0:jb, :] -= U11[0:jb, jb:je] X[jb:je, :] (right-looking: the
// right-hand sides are columns here, so the rows above give the update its tiles).
void trsm_luci_right(hipStream_t s, double* U, int64_t ldu, int n, int np) {
    const int cols = n - np;
    if (cols <= 0) return;
    double* X = U + (int64_t)np * ldu;
    for (int jb = ((np - 1) / kTrsmNB) * kTrsmNB; jb >= 0; jb -= kTrsmNB) {
        const int nb = std::min(kTrsmNB, np - jb);
        // x_a -= sum_{t > a} U11[a, t] x_t: M(a, t) = U[a + t ldu]
        trsm_diag(s, X + jb, ldu, 1, cols, U + jb + (int64_t)jb * ldu, 1, ldu, nb, true, true);
        if (jb > 0)
            launch_dgemm(s, false, jb, cols, nb, -1.0, U + (int64_t)jb * ldu, ldu, X + jb, ldu, 1.0, X,
                         ldu, nullptr, 0, nullptr, nullptr);
    }
}

// ------------------------------------------------------------------------- K5 site-tensor solve
// getrf of A = P^T (r x r) in place: panels of nbp columns, factorised in LDS by one workgroup
// (partial pivoting: first maximal |a| of the updated column, as idamax), their interchanges
// applied to the other columns, U12 = L11^-1 A12 (unit lower), then the K3 trailing update
// A22 -= L21 U12. Same pivot rule as the unblocked k_getrf_transposed; values differ from it
// only by the summation order of the updates.
__global__ void k_transpose_sq(double* __restrict__ P, int r) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)r * r; e += stride) {
        const int i = (int)(e % r), j = (int)(e / r);
        if (i < j) {
            const double a = P[i + (int64_t)j * r], b = P[j + (int64_t)i * r];
            P[i + (int64_t)j * r] = b;
            P[j + (int64_t)i * r] = a;
        }
    }
}

constexpr int kPanelLds = 128 * 1024;  // bytes of LDS for one panel

// One workgroup factorises the panel in LDS, thread t owning rows t, t + 1024, ... Per column c:
// the argmax partials of the rows >= c (computed in the previous step's update), one barrier,
// every thread reduces the 16 wave results itself (no second barrier), the nbp-wide row swap c <->
// p, one barrier, then each thread scales its rows and applies the rank-1 update to them, taking
// the next column's argmax partial on the way.
__global__ __launch_bounds__(1024) void k_getrf_panel(double* __restrict__ A, int r, int jb, int nbp,
                                                      int* __restrict__ piv) {
    extern __shared__ __attribute__((aligned(16))) double Ps[];  // [c][row - jb], ld = rows
    __shared__ double sv[16];
    __shared__ int si[16];
    const int rows = r - jb, tid = threadIdx.x, nth = blockDim.x, nw = nth >> 6;
    for (int e = tid; e < rows * nbp; e += nth) {
        const int i = e % rows, c = e / rows;
        Ps[e] = A[(int64_t)(jb + i) + (int64_t)(jb + c) * r];
    }
    __syncthreads();
    // partial argmax of column 0
    double bv = -1.0;
    int bi = 0x7fffffff;
    for (int i = tid; i < rows; i += nth) {
        const double v = fabs(Ps[i]);
        if (v > bv) { bv = v; bi = i; }  // ascending i: first maximum
    }
    for (int c = 0; c < nbp; ++c) {
        for (int off = 32; off >= 1; off >>= 1) {
            const double v2 = __shfl_xor(bv, off);
            const int i2 = __shfl_xor(bi, off);
            if (v2 > bv || (v2 == bv && i2 < bi)) { bv = v2; bi = i2; }
        }
        if ((tid & 63) == 0) { sv[tid >> 6] = bv; si[tid >> 6] = bi; }
        __syncthreads();
        double b = sv[0];
        int p = si[0];
        for (int q = 1; q < nw; ++q)
            if (sv[q] > b || (sv[q] == b && si[q] < p)) { b = sv[q]; p = si[q]; }
        if (p == 0x7fffffff) p = c;
        if (tid == 0) piv[jb + c] = jb + p;
        if (p != c && tid < nbp) {
            const double t = Ps[(int64_t)tid * rows + c];
            Ps[(int64_t)tid * rows + c] = Ps[(int64_t)tid * rows + p];
            Ps[(int64_t)tid * rows + p] = t;
        }
        __syncthreads();  // also orders this step's reads of sv/si before the next step's writes
        const double* col = Ps + (int64_t)c * rows;
        const double d = col[c];
        bv = -1.0;
        bi = 0x7fffffff;
        for (int i = c + 1 + tid; i < rows; i += nth) {
            const double l = col[i] / d;
            Ps[(int64_t)c * rows + i] = l;
            for (int cc = c + 1; cc < nbp; ++cc) {
                double* o = Ps + (int64_t)cc * rows;
                o[i] = __dsub_rn(o[i], __dmul_rn(l, o[c]));
            }
            if (c + 1 < nbp) {
                const double v = fabs(Ps[(int64_t)(c + 1) * rows + i]);
                if (v > bv) { bv = v; bi = i; }
            }
        }
        // row c + 1 itself was updated above by its owner; column c + 1's candidates are rows > c
    }
    __syncthreads();
    for (int e = tid; e < rows * nbp; e += nth) {
        const int i = e % rows, c = e / rows;
        A[(int64_t)(jb + i) + (int64_t)(jb + c) * r] = Ps[e];
    }
}

// The same panel factorisation with the panel in REGISTERS (rows <= 1024 RPT): thread t owns rows
// t + 1024 u, u < RPT, and their NBP values. Per column c: the thread's first maximal |a| over its
// rows >= c, a DPP + readlane wave argmax, the 16 wave results through LDS (barrier 1), then the
// owners of rows p and c publish their whole panel rows (barrier 2) and swap them in registers,
// and every thread scales its rows > c and applies the rank-1 update with the pivot row read as
// LDS broadcasts, taking column c + 1's argmax partial on the way. Same arithmetic as
// k_getrf_panel (true division, separate multiply and subtract, the same pivot rule): bitwise the
// same factors, without its per-update LDS round trips.
template <int CTRL>
__device__ __forceinline__ void dpp_take_max(double& bv, int& bi) {
    const uint64_t b = (uint64_t)__double_as_longlong(bv);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    const double ov = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    const int oi = __builtin_amdgcn_update_dpp(0, bi, CTRL, 0xf, 0xf, false);
    if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
    }
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// every lane ends with the wave's (first) maximum; -1 / INT_MAX when no lane has a candidate
__device__ __forceinline__ void wave_argmax(double& bv, int& bi) {
    dpp_take_max<0xb1>(bv, bi);   // quad_perm [1,0,3,2]
    dpp_take_max<0x4e>(bv, bi);   // quad_perm [2,3,0,1]
    dpp_take_max<0x141>(bv, bi);  // row_half_mirror
    dpp_take_max<0x140>(bv, bi);  // row_mirror: every lane of a 16-lane row has the row's best
    double v = readlane_d(bv, 0);
    int i = __builtin_amdgcn_readlane(bi, 0);
#pragma unroll
    for (int rr = 16; rr < 64; rr += 16) {
        const double ov = readlane_d(bv, rr);
        const int oi = __builtin_amdgcn_readlane(bi, rr);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
    bv = v;
    bi = i;
}

constexpr int kRegPanelThreads = 1024;

template <int NBP, int RPT, int NT = kRegPanelThreads>
struct RegPanel {  // one thread's state (the column steps are unrolled by recursion: every index of v
    double v[RPT][NBP];  // is a constant, so v lives in registers)
    double bv;
    int bi;
    int tid, rows, nbp, jb;
    int* piv;
    double* sv;
    int* si;
    double* prow;
    double* crow;
};

template <int NBP, int RPT, int C, int NT>
__device__ __forceinline__ void reg_panel_col(RegPanel<NBP, RPT, NT>& S) {
    if constexpr (C < NBP) {
        constexpr int NW = NT / 64;
        if (C < S.nbp) {
            const int tid = S.tid;
            wave_argmax(S.bv, S.bi);
            if ((tid & 63) == 0) { S.sv[tid >> 6] = S.bv; S.si[tid >> 6] = S.bi; }
            __syncthreads();  // barrier 1
            double b = S.sv[0];
            int p = S.si[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) {
                const double ov = S.sv[w];
                const int oi = S.si[w];
                if (ov > b || (ov == b && oi < p)) { b = ov; p = oi; }
            }
            if (p == 0x7fffffff) p = C;
            if (tid == 0) S.piv[S.jb + C] = S.jb + p;
            // the owners of rows p and C publish their panel rows
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int i = tid + u * NT;
                if (i == p) {
#pragma unroll
                    for (int cc = 0; cc < NBP; ++cc) S.prow[cc] = S.v[u][cc];
                }
                if (i == C && p != C) {
#pragma unroll
                    for (int cc = 0; cc < NBP; ++cc) S.crow[cc] = S.v[u][cc];
                }
            }
            __syncthreads();  // barrier 2
            if (p != C) {
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    const int i = tid + u * NT;
                    if (i == C) {
#pragma unroll
                        for (int cc = 0; cc < NBP; ++cc) S.v[u][cc] = S.prow[cc];
                    } else if (i == p) {
#pragma unroll
                        for (int cc = 0; cc < NBP; ++cc) S.v[u][cc] = S.crow[cc];
                    }
                }
            }
            const double d = S.prow[C];
            S.bv = -1.0;
            S.bi = 0x7fffffff;
#pragma unroll
            for (int u = 0; u < RPT; ++u) {
                const int i = tid + u * NT;
                if (i > C && i < S.rows) {
                    const double l = S.v[u][C] / d;
                    S.v[u][C] = l;
#pragma unroll
                    for (int cc = C + 1; cc < NBP; ++cc) S.v[u][cc] = __dsub_rn(S.v[u][cc], __dmul_rn(l, S.prow[cc]));
                    if constexpr (C + 1 < NBP) {
                        if (C + 1 < S.nbp) {
                            const double a = fabs(S.v[u][C + 1]);
                            if (a > S.bv) { S.bv = a; S.bi = i; }
                        }
                    }
                }
            }
        }
        reg_panel_col<NBP, RPT, C + 1, NT>(S);
    }
}

// NT threads: 1024 (one row per thread up to 1024 rows) or 256 (four waves, one per SIMD, RPT rows
// per thread: cheaper barriers, more update work per thread -- TCI_GETRF_NT A/B)
template <int NBP, int RPT, int NT = kRegPanelThreads>
__global__ __launch_bounds__(NT) void k_getrf_panel_reg(double* __restrict__ A, int r, int jb,
                                                        int nbp, int* __restrict__ piv) {
    constexpr int NW = NT / 64;
    __shared__ double sv[NW];
    __shared__ int si[NW];
    __shared__ double prow[NBP], crow[NBP];
    RegPanel<NBP, RPT, NT> S;
    S.tid = threadIdx.x;
    S.rows = r - jb;
    S.nbp = nbp;
    S.jb = jb;
    S.piv = piv;
    S.sv = sv;
    S.si = si;
    S.prow = prow;
    S.crow = crow;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int i = S.tid + u * NT;
#pragma unroll
        for (int c = 0; c < NBP; ++c)
            S.v[u][c] = (i < S.rows && c < nbp) ? A[(int64_t)(jb + i) + (int64_t)(jb + c) * r] : 0.0;
    }
    // column 0's partial: ascending rows, strict '>' (first maximum)
    S.bv = -1.0;
    S.bi = 0x7fffffff;
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int i = S.tid + u * NT;
        if (i < S.rows) {
            const double a = fabs(S.v[u][0]);
            if (a > S.bv) { S.bv = a; S.bi = i; }
        }
    }
    reg_panel_col<NBP, RPT, 0, NT>(S);
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        const int i = S.tid + u * NT;
        if (i < S.rows) {
#pragma unroll
            for (int c = 0; c < NBP; ++c)
                if (c < nbp) A[(int64_t)(jb + i) + (int64_t)(jb + c) * r] = S.v[u][c];
        }
    }
}

// The panel's interchanges applied to every column outside it (laswp). They compose to a
// permutation of at most 2 nbp rows (the panel's and the rows swapped into it), computed once per
// workgroup in LDS: every thread (one per column) then moves its column's affected values with
// independent loads and stores instead of nbp dependent swaps.
template <int NBP>
__global__ __launch_bounds__(256) void k_getrf_swap(double* __restrict__ A, int r, int jb, int nbp,
                                                    const int* __restrict__ piv) {
    __shared__ int pos[2 * NBP];  // affected row positions
    __shared__ int src[2 * NBP];  // final content of pos[q]: the original row src[q]
    __shared__ int naff;
    const int tid = threadIdx.x;
    if (tid < 64) {
        // wave 0 composes the interchanges: lane l holds slots l and l + 64 (pos, src); the
        // search for row p is a ballot, the swap two readlanes
        const int l = tid;
        int pos0 = l < nbp ? jb + l : -1, src0 = pos0;
        int pos1 = -1, src1 = -1;
        int n = nbp;
        // every interchange loaded at once (lane k holds piv[jb + k], nbp <= 64), read back by
        // readlane: a load per step inside the loop was a dependent round trip per interchange
        const int pl = l < nbp ? piv[jb + l] : 0;
        for (int k = 0; k < nbp; ++k) {
            const int p = __builtin_amdgcn_readlane(pl, k);
            const unsigned long long b0 = __ballot(pos0 == p), b1 = __ballot(pos1 == p);
            int qp;
            if (b0) qp = __ffsll((long long)b0) - 1;
            else if (b1) qp = 64 + __ffsll((long long)b1) - 1;
            else {
                qp = n++;
                if (qp < 64) { if (l == qp) { pos0 = p; src0 = p; } }
                else if (l == qp - 64) { pos1 = p; src1 = p; }
            }
            const int sk = __shfl(src0, k);  // k < nbp <= 64: slot k is in the first half
            const int sp = qp < 64 ? __shfl(src0, qp) : __shfl(src1, qp - 64);
            if (l == k) src0 = sp;
            if (qp < 64) { if (l == qp) src0 = sk; }
            else if (l == qp - 64) src1 = sk;
        }
        if (l < 2 * NBP) { pos[l] = pos0; src[l] = src0; }
        if (l + 64 < 2 * NBP) { pos[l + 64] = pos1; src[l + 64] = src1; }
        if (l == 0) naff = n;
    }
    __syncthreads();
    const int cidx = blockIdx.x * blockDim.x + tid, nother = r - nbp;
    if (cidx >= nother) return;
    const int c = cidx < jb ? cidx : cidx + nbp;
    double* col = A + (int64_t)c * r;
    const int n = naff;
    double v[2 * NBP];
#pragma unroll
    for (int q = 0; q < 2 * NBP; ++q)
        if (q < n) v[q] = col[src[q]];
#pragma unroll
    for (int q = 0; q < 2 * NBP; ++q)
        if (q < n) col[pos[q]] = v[q];
}

static int panel_width(int rows) {
    int nbp = 64;
    while (nbp > 4 && (int64_t)rows * nbp * 8 > kPanelLds) nbp >>= 1;
    return nbp;
}

bool getrf_blocked_fits(int r) { return (int64_t)r * 4 * 8 <= kPanelLds; }

void launch_getrf_blocked(hipStream_t s, double* A, int r, int* piv, bool reg) {
    hipLaunchKernelGGL(k_transpose_sq, dim3(std::min(2048, std::max(1, (r * r + 255) / 256))), dim3(256), 0, s,
                       A, r);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_getrf_panel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        kPanelLds);
    // panels in registers (k_getrf_panel_reg) unless the context's dense mask drops kDenseGetrfReg
    // 256 threads (four waves, RPT rows each) by default: 9.32 -> 8.95 ms for the r = 1024 solve
    // (getrf 6.93 -> 6.58 ms; profiles/r05_l1_ab_getrf_nt.txt); TCI_GETRF_NT=1024 for the A/B
    static const int nt_env = [] {
        const char* e = getenv("TCI_GETRF_NT");
        return e ? atoi(e) : 256;
    }();
    for (int jb = 0; jb < r;) {
        const int rows = r - jb;
        int nbp;
        if (reg && nt_env == 256 && rows <= 1024) {
            nbp = std::min(24, rows);
            hipLaunchKernelGGL((k_getrf_panel_reg<24, 4, 256>), dim3(1), dim3(256), 0, s, A, r, jb, nbp, piv);
        } else if (reg && nt_env == 256 && rows <= 2048) {
            nbp = std::min(16, rows);
            hipLaunchKernelGGL((k_getrf_panel_reg<16, 8, 256>), dim3(1), dim3(256), 0, s, A, r, jb, nbp, piv);
        } else if (reg && rows <= kRegPanelThreads) {
            nbp = std::min(24, rows);
            hipLaunchKernelGGL((k_getrf_panel_reg<24, 1>), dim3(1), dim3(kRegPanelThreads), 0, s, A, r, jb, nbp, piv);
        } else if (reg && rows <= 2 * kRegPanelThreads) {
            nbp = std::min(16, rows);
            hipLaunchKernelGGL((k_getrf_panel_reg<16, 2>), dim3(1), dim3(kRegPanelThreads), 0, s, A, r, jb, nbp, piv);
        } else {
            nbp = std::min(panel_width(rows), rows);
            hipLaunchKernelGGL(k_getrf_panel, dim3(1), dim3(1024), (size_t)rows * nbp * 8, s, A, r, jb, nbp, piv);
        }
        const int je = jb + nbp, nother = r - nbp;
        if (nother > 0) {
            const dim3 g((nother + 255) / 256), b(256);
            if (nbp <= 8) hipLaunchKernelGGL(k_getrf_swap<8>, g, b, 0, s, A, r, jb, nbp, piv);
            else if (nbp <= 16) hipLaunchKernelGGL(k_getrf_swap<16>, g, b, 0, s, A, r, jb, nbp, piv);
            else if (nbp <= 32) hipLaunchKernelGGL(k_getrf_swap<32>, g, b, 0, s, A, r, jb, nbp, piv);
            else hipLaunchKernelGGL(k_getrf_swap<64>, g, b, 0, s, A, r, jb, nbp, piv);
        }
        // U12 = L11^-1 A12: right-hand sides are the columns je..r-1, M(j, t) = A[jb + j, jb + t]
        if (je < r)
            trsm_diag(s, A + jb + (int64_t)je * r, r, 1, r - je, A + jb + (int64_t)jb * r, 1, r, nbp, false, true);
        if (je < r)
            launch_dgemm(s, false, r - je, r - je, nbp, -1.0, A + je + (int64_t)jb * r, r,
                         A + jb + (int64_t)je * r, r, 1.0, A + je + (int64_t)je * r, r,
                         A + je + (int64_t)je * r, r, nullptr, nullptr);
        jb = je;
    }
}

// Round 6: the whole getrf (rows <= 1024) as ONE cooperative launch. launch_getrf_blocked issues
// four dependent launches per 24-column panel (panel, interchanges, U12 solve, K = 24 update): at
// r = 1024 that is 172 launches and ~6.5 ms, of which the panels' own column steps are ~2. Here G
// workgroups (one per 8-column block group, at most 64, all co-resident) loop over the panels:
//  1. every workgroup loads the panel (rows jb..r-1) and factorises it in registers with the
//     k_getrf_panel_reg column step -- redundantly, bitwise the same everywhere, so no hand-off of
//     the factored panel is needed;
//  2. workgroup 0 stores the interchanges;
//  3. each workgroup applies the panel to the 8-column blocks it owns (block b: workgroup b mod G):
//     blocks left of the panel take the composed interchanges (<= 48 rows); blocks right of it are
//     staged in LDS, permuted, their U12 rows solved against L11 (column-oriented substitution, one
//     wave per column, readlane broadcasts) and their rows below updated by L21 U12 with L21 still
//     in the registers of step 1 (sequential separate multiply and subtract);
//  4. one grid barrier (release fence, agent counter, acquire fence: MI355X_MICROARCH.md's
//     barrier-counter row) before the next panel reads its columns;
//  5. the owners of the panel's column blocks store them (after the barrier: every workgroup has
//     read the panel by then).
// Same pivot rule and panel arithmetic as the blocked path; the trailing updates sum in another
// order than K3's MFMAs (rounding). Co-residency is not assumed blindly: a workgroup that waits
// more than 4 ms for the others sets the fault word and every workgroup leaves; the host then
// redoes the solve from a copy of P on the launch-per-panel path (tci_abi.cpp solve_launch).
constexpr int kCoopNBP = 24, kCoopRPT = 4, kCoopNT = 256, kCoopCW = 8, kCoopMaxG = 64;

bool getrf_coop_fits(int r) { return r >= 1 && r <= kCoopNT * kCoopRPT; }

// Cross-workgroup data of the cooperative getrf is stored and loaded write-through (agent-scope
// relaxed atomics: global_store / global_load sc1), so the barrier needs no L2 write-back: every
// wave drains its stores, one lane adds to the counter, polls it, and invalidates the CU's L1
// (MI355X_MICROARCH.md hand-off table, row 1, with the acquire kept). The release fence of round
// 6's first build (buffer_wbl2 from every workgroup) made the barrier ~32 us per panel.
__device__ __forceinline__ double ld_wt(const double* p) {
    return __longlong_as_double(
        __hip_atomic_load(reinterpret_cast<const long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool coop_grid_sync(unsigned* count, unsigned target, int* fault, int* lflag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int bad = 0;
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 400000ull || __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                bad = 1;
                __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *lflag = bad;
    }
    __syncthreads();
    return *lflag == 0;
}

#ifdef TCI_COOP_PROF  // phase sums of workgroup 0 (100 MHz ticks), printed at the end (A/B builds only)
#define COOP_T(i) do { if (tid == 0) { const unsigned long long t_ = wall_clock64(); pacc[i] += t_ - tlast; tlast = t_; } } while (0)
#else
#define COOP_T(i) do { } while (0)
#endif
__global__ __launch_bounds__(kCoopNT) void k_getrf_coop(double* __restrict__ A, int r, int* __restrict__ piv,
                                                        unsigned* count, int* fault, int inject) {
#ifdef TCI_COOP_PROF
    unsigned long long pacc[6] = {0, 0, 0, 0, 0, 0}, tlast = wall_clock64();
#endif
    constexpr int NBP = kCoopNBP, RPT = kCoopRPT, NT = kCoopNT, NW = NT / 64, CW = kCoopCW;
    constexpr int LDB = NT * RPT;  // ld of the staged column block (rows jb..r-1 <= 1024)
    __shared__ double sv[NW];
    __shared__ int si[NW];
    __shared__ double prow[NBP], crow[NBP];
    __shared__ int spiv[NBP];
    __shared__ double sL11[NBP * NBP];  // sL11[i NBP + c] = L(i, c) of the panel, i, c < nbp
    __shared__ int pos[2 * NBP], src[2 * NBP];
    __shared__ int naff, lflag;
    constexpr int CT = 2 * CW;  // columns a workgroup owns at most (2 blocks: nblk <= 2 G at r <= 1024)
    __shared__ double cb[CT * LDB];  // its right-of-panel columns, rows jb..r-1 (ld LDB)
    __shared__ int sperm[LDB];        // workgroup 0: the permutation the interchanges compose to
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nblk = (r + CW - 1) / CW;
    if (g == 0)
        for (int a = tid; a < r; a += NT) sperm[a] = a;
    unsigned epoch = 0;
    for (int jb = 0; jb < r; jb += NBP) {
        const int nbp = min(NBP, r - jb), je = jb + nbp, rows = r - jb;
        // 1. the panel, factorised in registers (every workgroup)
        RegPanel<NBP, RPT, NT> S;
        S.tid = tid;
        S.rows = rows;
        S.nbp = nbp;
        S.jb = jb;
        S.piv = spiv - jb;  // reg_panel_col stores piv[jb + C] = jb + p
        S.sv = sv;
        S.si = si;
        S.prow = prow;
        S.crow = crow;
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int i = tid + u * NT;
#pragma unroll
            for (int c = 0; c < NBP; ++c)
                S.v[u][c] = (i < rows && c < nbp) ? ld_wt(A + (int64_t)(jb + i) + (int64_t)(jb + c) * r) : 0.0;
        }
        S.bv = -1.0;
        S.bi = 0x7fffffff;
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
            const int i = tid + u * NT;
            if (i < rows) {
                const double a = fabs(S.v[u][0]);
                if (a > S.bv) { S.bv = a; S.bi = i; }
            }
        }
        COOP_T(0);
        reg_panel_col<NBP, RPT, 0, NT>(S);
        COOP_T(1);
        if (tid < nbp) {
#pragma unroll
            for (int c = 0; c < NBP; ++c) sL11[tid * NBP + c] = S.v[0][c];
        }
        __syncthreads();  // spiv (the last column's) and sL11
        // 2. the interchanges
        if (g == 0 && tid < nbp) piv[jb + tid] = spiv[tid];
        // the owned blocks: b = g and b = g + G (nblk <= 2 G); left of the panel, the panel's own
        // (stored in step 5) or right of it
        const int b0 = g, b1 = g + G;
        const int n0 = b0 < nblk ? min(CW, r - b0 * CW) : 0, n1 = b1 < nblk ? min(CW, r - b1 * CW) : 0;
        const bool r0 = n0 > 0 && b0 * CW >= je, r1 = n1 > 0 && b1 * CW >= je;
        const bool l0 = n0 > 0 && b0 * CW < jb, l1 = n1 > 0 && b1 * CW < jb;
        // right blocks' staging loads go out first (the interchanges are not needed for them)
        double sv_[CW][RPT];
        auto stage_load = [&](int c0, int nc) {
#pragma unroll
            for (int k = 0; k < CW; ++k)
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    const int i = tid + u * NT;
                    sv_[k][u] = (k < nc && i < rows) ? ld_wt(A + (int64_t)(jb + i) + (int64_t)(c0 + k) * r) : 0.0;
                }
        };
        auto stage_store = [&](int kofs) {
#pragma unroll
            for (int k = 0; k < CW; ++k)
#pragma unroll
                for (int u = 0; u < RPT; ++u) cb[(kofs + k) * LDB + tid + u * NT] = sv_[k][u];
        };
        const int firstR = r0 ? b0 : b1;  // local columns 0..7: the first right block, 8..15: the second
        const int nR = (r0 ? 1 : 0) + (r1 ? 1 : 0);
        if (nR) stage_load(firstR * CW, firstR == b0 ? n0 : n1);
        if (tid < 64) {  // compose the interchanges into <= 2 nbp (position, source) pairs (k_getrf_swap)
            const int l = tid;
            int pos0 = l < nbp ? jb + l : -1, src0 = pos0;
            int pos1 = -1, src1 = -1;
            int n = nbp;
            const int pl = l < nbp ? spiv[l] : 0;
            for (int k = 0; k < nbp; ++k) {
                const int p = __builtin_amdgcn_readlane(pl, k);
                const unsigned long long bb0 = __ballot(pos0 == p), bb1 = __ballot(pos1 == p);
                int qp;
                if (bb0) qp = __ffsll((long long)bb0) - 1;
                else if (bb1) qp = 64 + __ffsll((long long)bb1) - 1;
                else {
                    qp = n++;
                    if (qp < 64) { if (l == qp) { pos0 = p; src0 = p; } }
                    else if (l == qp - 64) { pos1 = p; src1 = p; }
                }
                const int sk = __shfl(src0, k);
                const int sp = qp < 64 ? __shfl(src0, qp) : __shfl(src1, qp - 64);
                if (l == k) src0 = sp;
                if (qp < 64) { if (l == qp) src0 = sk; }
                else if (l == qp - 64) src1 = sk;
            }
            if (l < 2 * NBP) { pos[l] = pos0; src[l] = src0; }
            if (l + 64 < 2 * NBP) { pos[l + 64] = pos1; src[l + 64] = src1; }
            if (l == 0) naff = n;
        }
        if (nR) stage_store(0);
        if (nR == 2) {
            stage_load(b1 * CW, n1);
            stage_store(CW);
        }
        __syncthreads();
        const int na = naff;
        if (g == 0) {  // perm[pos[q]] <- perm[src[q]] (k_piv_to_perm's result, without its serial loop)
            const int pv0 = tid < na ? sperm[src[tid]] : 0;
            __syncthreads();
            if (tid < na) sperm[pos[tid]] = pv0;
        }
        COOP_T(2);
        // 3. left blocks: the composed interchanges on global memory; right blocks: the same on the
        // staged rows in LDS (all loads, one barrier, all stores)
        const int nL = (l0 ? 1 : 0) + (l1 ? 1 : 0);
        const int lcol0 = l0 ? b0 * CW : b1 * CW, lcol1 = b1 * CW;
        const int lnc0 = l0 ? n0 : n1;
        const int ne = CW * na;  // (column, slot) pairs per block, <= 2 NT
        double lv[2][2], pv[4];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = tid + h * NT, c0 = q == 0 ? lcol0 : lcol1, nc = q == 0 ? lnc0 : n1;
                lv[q][h] = (q < nL && e < ne && e / na < nc) ? ld_wt(A + (int64_t)src[e % na] + (int64_t)(c0 + e / na) * r) : 0.0;
            }
        const int nck = nR * CW;  // staged local columns (padding columns of a short block included)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int e = tid + h * NT;
            pv[h] = e < nck * na ? cb[(e / na) * LDB + src[e % na] - jb] : 0.0;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = tid + h * NT, c0 = q == 0 ? lcol0 : lcol1, nc = q == 0 ? lnc0 : n1;
                if (q < nL && e < ne && e / na < nc) st_wt(A + (int64_t)pos[e % na] + (int64_t)(c0 + e / na) * r, lv[q][h]);
            }
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int e = tid + h * NT;
            if (e < nck * na) cb[(e / na) * LDB + pos[e % na] - jb] = pv[h];
        }
        __syncthreads();
        if (nR) {
            for (int k = wv; k < nck; k += NW) {  // U12 = L11^-1 A12: x_j -= L(j, c) x_c, c ascending
                double x = lane < nbp ? cb[k * LDB + lane] : 0.0;
#pragma unroll
                for (int c = 0; c < NBP; ++c) {
                    if (c < nbp) {
                        const double xc = readlane_d(x, c);
                        if (lane > c && lane < nbp) x = __dsub_rn(x, __dmul_rn(sL11[lane * NBP + c], xc));
                    }
                }
                if (lane < nbp) cb[k * LDB + lane] = x;
            }
            __syncthreads();
            // A22 -= L21 U12, L21 from the panel registers, U12 read once per (column, c) for all u
            for (int k = 0; k < nck; ++k) {
                const int blk = k < CW ? firstR : b1, kk = k & (CW - 1);
                const int nc = blk == b0 ? n0 : n1;
                if (kk >= nc) continue;
                double a[RPT];
#pragma unroll
                for (int u = 0; u < RPT; ++u) a[u] = cb[k * LDB + tid + u * NT];
#pragma unroll
                for (int c = 0; c < NBP; ++c) {
                    if (c < nbp) {
                        const double uc = cb[k * LDB + c];
#pragma unroll
                        for (int u = 0; u < RPT; ++u)
                            if (tid + u * NT >= nbp) a[u] = __dsub_rn(a[u], __dmul_rn(S.v[u][c], uc));
                    }
                }
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    const int i = tid + u * NT;
                    if (i < rows) st_wt(A + (int64_t)(jb + i) + (int64_t)(blk * CW + kk) * r, a[u]);
                }
            }
        }
        COOP_T(3);
        // 4. every column the next panel reads is stored: grid barrier
        ++epoch;
        if (inject && g == 0 && epoch == 2 && tid == 0)  // test mode: a barrier timeout, simulated
            __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (je < r && !coop_grid_sync(count, epoch * (unsigned)G, fault, &lflag)) return;
        COOP_T(4);
        // 5. only now (every workgroup has loaded the panel) its owned column blocks are stored; the
        // next panel's interchanges reach them through this workgroup's own step 3 (same CU: a
        // drained store is visible to its other waves after the barrier)
#pragma unroll
        for (int c = 0; c < NBP; ++c) {
            if (c < nbp && ((jb + c) / CW) % G == g) {
#pragma unroll
                for (int u = 0; u < RPT; ++u) {
                    const int i = tid + u * NT;
                    if (i < rows) A[(int64_t)(jb + i) + (int64_t)(jb + c) * r] = S.v[u][c];
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        COOP_T(5);
    }
    if (g == 0) {
        __syncthreads();
        for (int a = tid; a < r; a += NT) piv[r + a] = sperm[a];
    }
#ifdef TCI_COOP_PROF
    if (tid == 0 && g == 0)
        printf("coop getrf r %d G %d: load %.1f factor %.1f compose %.1f blocks %.1f barrier %.1f store %.1f us\n", r, G,
               pacc[0] * 0.01, pacc[1] * 0.01, pacc[2] * 0.01, pacc[3] * 0.01, pacc[4] * 0.01, pacc[5] * 0.01);
#endif
}

// sync: two words (arrival counter, fault), zeroed here
void launch_getrf_coop(hipStream_t s, double* A, int r, int* piv, unsigned* sync) {
    hipLaunchKernelGGL(k_transpose_sq, dim3(std::min(2048, std::max(1, (r * r + 255) / 256))), dim3(256), 0, s,
                       A, r);
    (void)hipMemsetAsync(sync, 0, 2 * sizeof(unsigned), s);
    const int G = std::min(kCoopMaxG, (r + kCoopCW - 1) / kCoopCW);
    // TCI_COOP_FAULT_TEST=1 (tests only): workgroup 0 raises the fault word at the second barrier,
    // as a timed-out wait would, so the host's redo-from-a-copy path runs (read per launch)
    const char* e = getenv("TCI_COOP_FAULT_TEST");
    const int inject = e && atoi(e) != 0;
    hipLaunchKernelGGL(k_getrf_coop, dim3(G), dim3(kCoopNT), 0, s, A, r, piv, sync,
                       reinterpret_cast<int*>(sync + 1), inject);
}

// T (R x r) = Pi1 P^-1 given A = LU(P^T) and its interchanges: T's columns permuted as the rows of
// P^T were (k_gather_cols), then T <- T L^-T (forward, unit) and T <- T U^-T (backward), each as
// kTrsmNB-wide diagonal solves (one thread per row of T) and K3 updates.
// (the interchanges composed in LDS by one thread -- the sequence is inherently serial -- with the
// interchange list and the permutation staged through LDS by the whole workgroup: each step is two
// LDS round trips instead of two global ones; 160 us -> tens of us at r = 1024)
constexpr int kPermLds = 4096;
__global__ __launch_bounds__(256) void k_piv_to_perm(const int* __restrict__ piv, int r, int* __restrict__ perm) {
    if (blockIdx.x != 0) return;
    __shared__ int sp[kPermLds], spv[kPermLds];
    if (r > kPermLds) {  // (not the solve's sizes: r <= 8192 / 2; the global fallback)
        if (threadIdx.x != 0) return;
        for (int a = 0; a < r; ++a) perm[a] = a;
        for (int k = 0; k < r; ++k) {
            const int p = piv[k];
            const int t = perm[k];
            perm[k] = perm[p];
            perm[p] = t;
        }
        return;
    }
    for (int a = threadIdx.x; a < r; a += blockDim.x) {
        sp[a] = a;
        spv[a] = piv[a];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < r; ++k) {
            const int p = spv[k];
            const int t = sp[k];
            sp[k] = sp[p];
            sp[p] = t;
        }
    }
    __syncthreads();
    for (int a = threadIdx.x; a < r; a += blockDim.x) perm[a] = sp[a];
}

__global__ void k_gather_cols(const double* __restrict__ Pi1, int R, int r, const int* __restrict__ perm,
                              double* __restrict__ T) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = gid; e < (int64_t)R * r; e += stride) {
        const int q = (int)(e % R), a = (int)(e / R);
        T[e] = Pi1[(int64_t)q + (int64_t)perm[a] * R];
    }
}

void launch_getrs_blocked(hipStream_t s, const double* A, int r, const int* piv, const double* Pi1,
                          int R, double* T, int* perm, bool perm_ready) {
    if (!perm_ready) hipLaunchKernelGGL(k_piv_to_perm, dim3(1), dim3(256), 0, s, piv, r, perm);
    const long long work = (long long)R * r;
    hipLaunchKernelGGL(k_gather_cols, dim3((unsigned)std::min<long long>(8192, (work + 255) / 256)), dim3(256),
                       0, s, Pi1, R, r, perm, T);
    // left-looking over 64-column blocks of T: each block is brought up to date by one K3 update
    // from the blocks already solved (K = jb, written once), then its diagonal block is solved
    for (int jb = 0; jb < r; jb += kTrsmNB) {  // L: unit lower, M(j, t) = A[j + t r]
        const int nb = std::min(kTrsmNB, r - jb);
        if (jb > 0)  // T[:, jb:je] -= T[:, 0:jb] L[jb:je, 0:jb]^T
            launch_dgemm(s, true, R, nb, jb, -1.0, T, R, A + jb, r, 1.0, T + (int64_t)jb * R, R, nullptr, 0,
                         nullptr, nullptr);
        trsm_diag(s, T + (int64_t)jb * R, 1, R, R, A + jb + (int64_t)jb * r, 1, r, nb, false, true);
    }
    for (int jb = ((r - 1) / kTrsmNB) * kTrsmNB; jb >= 0; jb -= kTrsmNB) {  // U, with its diagonal
        const int nb = std::min(kTrsmNB, r - jb), je = jb + nb;
        if (je < r)  // T[:, jb:je] -= T[:, je:r] U[jb:je, je:r]^T
            launch_dgemm(s, true, R, nb, r - je, -1.0, T + (int64_t)je * R, R, A + jb + (int64_t)je * r, r, 1.0,
                         T + (int64_t)jb * R, R, nullptr, 0, nullptr, nullptr);
        trsm_diag(s, T + (int64_t)jb * R, 1, R, R, A + jb + (int64_t)jb * r, 1, r, nb, true, false);
    }
}

// ------------------------------------------------------------------------- MFMA probe (diag)
// Independent v_mfma_f64_16x16x4f64 chains, W waves per SIMD (256 * W threads per workgroup, one
// workgroup per CU); cycles[blockIdx] = s_memtime cycles of wave 0's loop (the shader clock), so
// the host gets both the rate and the clock it ran at.
template <int W>
__global__ __launch_bounds__(256 * W) void k_mfma_probe2(int iters, double* sink, long long* cycles) {
    dbl4 acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    const long long t1 = clock64();
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
    if (s == 12345.0) sink[0] = s;
}

void launch_mfma_probe2(hipStream_t s, int waves_per_simd, int grid, int iters, double* sink,
                        long long* cycles) {
    switch (waves_per_simd) {
        case 1: hipLaunchKernelGGL(k_mfma_probe2<1>, dim3(grid), dim3(256), 0, s, iters, sink, cycles); break;
        case 2: hipLaunchKernelGGL(k_mfma_probe2<2>, dim3(grid), dim3(512), 0, s, iters, sink, cycles); break;
        default: hipLaunchKernelGGL(k_mfma_probe2<4>, dim3(grid), dim3(1024), 0, s, iters, sink, cycles); break;
    }
}

}  // namespace tci
