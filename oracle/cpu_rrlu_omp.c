/*
 * cpu_rrlu_omp.c -- TEST / BASELINE INFRASTRUCTURE ONLY: the all-core CPU baseline of the rrLU
 * (SURVEY 8(d) "CPU baseline" variant (ii)). Loaded only by bench.py's cpu_baseline
 * leg and tests/; the product path never links or calls it.
 *
 * Same algorithm and arithmetic as oracle/tci_oracle.c:orc_rrlu_inplace, i.e. _optimizerrlu!
 * (reference src/matrixlu.jl:346-396) with submatrixargmax (:46-87) and addpivot! (:254-322):
 * physical row/column swaps, true-division normalisation, rank-1 update as a separate multiply
 * and subtract (-ffp-contract=off), abs2 argmax with strict '>' in column-major order. It is a
 * stronger baseline than the loop-for-loop restatement, the analogue of the reference's
 * ThreadedBatchEvaluator (batcheval.jl:282-308) applied to the factorisation:
 *   - OpenMP over columns (static contiguous blocks), every thread updating its columns;
 *   - the update of pivot k fused with the argmax for pivot k+1 (one read+write pass per pivot
 *     instead of a read pass plus a read+write pass);
 *   - per-thread candidates reduced in thread (= column) order with strict '>', which is exactly
 *     the column-major first-maximum of the sequential scan, so results are bitwise identical to
 *     orc_rrlu_inplace (tests/test_oracle_kats.py checks it).
 * Built for the host it runs on (-march=native) by bench.py; oracle/Makefile builds a portable
 * x86-64-v3 copy.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

typedef int64_t i64;

typedef struct {
    double v;  /* abs2 of the candidate, -inf if none */
    i64 r, c;
} cand_t;

int cpu_rrlu_threads(void) { return omp_get_max_threads(); }

/* column maximum of abs2 over rows [r0, m) of col, first row attaining it (strict '>') */
static inline void col_argmax(const double* col, i64 r0, i64 m, double* best, i64* br) {
    double b = -INFINITY;
    for (i64 i = r0; i < m; ++i) {
        const double v = col[i] * col[i];
        b = v > b ? v : b; /* NaN never wins, like `abs2(x) > best` */
    }
    if (b == -INFINITY) { *best = b; return; }
    i64 r = r0;
    while (!(col[r] * col[r] == b)) ++r;
    *best = b;
    *br = r;
}

/* Same contract as orc_rrlu_inplace (0-based permutations, pivot_limit >= 0 caps the pivots). */
int cpu_rrlu_inplace_omp(double* A, i64 m, i64 n, i64 lda, i64 maxrank, double reltol,
                         double abstol, int leftorth, i64* rowperm, i64* colperm, i64* npivot,
                         double* err, i64 pivot_limit) {
    for (i64 i = 0; i < m; ++i) rowperm[i] = i;
    for (i64 j = 0; j < n; ++j) colperm[j] = j;
    i64 mr = maxrank;
    if (mr > m) mr = m;
    if (mr > n) mr = n;
    double maxerror = 0.0, error = NAN;
    i64 np = 0;
    const int nt = omp_get_max_threads();
    cand_t cands[1024];
    cand_t next = {-INFINITY, 0, 0};
    /* initial argmax over the whole matrix */
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
        const i64 j0 = n * t / T, j1 = n * (t + 1) / T;
        cand_t c = {-INFINITY, 0, 0};
        for (i64 j = j0; j < j1; ++j) {
            double b;
            i64 r = 0;
            col_argmax(A + j * lda, 0, m, &b, &r);
            if (b > c.v) { c.v = b; c.r = r; c.c = j; }
        }
        cands[t] = c;
#pragma omp barrier
#pragma omp single
        {
            for (int s = 0; s < T; ++s)
                if (cands[s].v > next.v) next = cands[s];
        }
    }
    while (np < mr) {
        if (pivot_limit >= 0 && np >= pivot_limit) break;
        const i64 k = np;
        /* submatrixargmax with nothing selectable (all NaN) returns the block's first entry */
        const i64 p = next.v == -INFINITY ? k : next.r, q = next.v == -INFINITY ? k : next.c;
        error = fabs(A[p + q * lda]);
        if ((fabs(error) < reltol * maxerror || fabs(error) < abstol) && np > 0) break;
        maxerror = fmax(maxerror, error) == maxerror && !isnan(error) ? maxerror : error;
        i64 t0 = rowperm[k];
        rowperm[k] = rowperm[p];
        rowperm[p] = t0;
        t0 = colperm[k];
        colperm[k] = colperm[q];
        colperm[q] = t0;
        next.v = -INFINITY;
        next.r = next.c = k + 1;
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num(), T = omp_get_num_threads();
            /* row swap k <-> p over all columns, then the column swap k <-> q */
            {
                const i64 j0 = n * t / T, j1 = n * (t + 1) / T;
                if (p != k)
                    for (i64 j = j0; j < j1; ++j) {
                        double a = A[k + j * lda];
                        A[k + j * lda] = A[p + j * lda];
                        A[p + j * lda] = a;
                    }
            }
#pragma omp barrier
            if (q != k) {
                const i64 i0 = m * t / T, i1 = m * (t + 1) / T;
                for (i64 i = i0; i < i1; ++i) {
                    double a = A[i + k * lda];
                    A[i + k * lda] = A[i + q * lda];
                    A[i + q * lda] = a;
                }
            }
#pragma omp barrier
            const double piv = A[k + k * lda];
            if (leftorth) {
                const i64 i0 = k + 1 + (m - k - 1) * t / T, i1 = k + 1 + (m - k - 1) * (t + 1) / T;
                for (i64 i = i0; i < i1; ++i) A[i + k * lda] = A[i + k * lda] / piv;
            } else {
                const i64 j0 = k + 1 + (n - k - 1) * t / T, j1 = k + 1 + (n - k - 1) * (t + 1) / T;
                for (i64 j = j0; j < j1; ++j) A[k + j * lda] = A[k + j * lda] / piv;
            }
#pragma omp barrier
            /* rank-1 update of columns k+1..n-1 fused with the argmax for pivot k+1 */
            const double* x = A + k * lda;
            const i64 j0 = k + 1 + (n - k - 1) * t / T, j1 = k + 1 + (n - k - 1) * (t + 1) / T;
            cand_t c = {-INFINITY, k + 1, k + 1};
            for (i64 j = j0; j < j1; ++j) {
                const double y = A[k + j * lda];
                double* col = A + j * lda;
                for (i64 i = k + 1; i < m; ++i) {
                    const double prod = x[i] * y;
                    col[i] = col[i] - prod;
                }
                double b;
                i64 r = k + 1;
                col_argmax(col, k + 1, m, &b, &r);
                if (b > c.v) { c.v = b; c.r = r; c.c = j; }
            }
            cands[t] = c;
#pragma omp barrier
#pragma omp single
            {
                for (int s = 0; s < T; ++s)
                    if (cands[s].v > next.v) next = cands[s];
            }
        }
        np += 1;
    }
    const i64 mn = m < n ? m : n;
    if (np >= mn) error = 0.0;
    *npivot = np;
    *err = error;
    return 0;
}
