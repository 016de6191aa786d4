/*
 * tci_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle and the CPU baseline).
 *
 * A plain-C, loop-for-loop restatement of the TensorCrossInterpolation.jl TCI2 hot path
 * (reference: XiaoJiang-Phy/TensorCrossInterpolation.jl, fork of tensor4all v0.9.18).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker. The product path (tensorcrossinterpolation.jl_amd/)
 * never links, loads or calls it.
 *
 * Pinning: the rrLU / argmax / MatrixLUCI / kronecker / pivoterror / convergence pieces are
 * checked against the known-answer tests the reference ships in test/test_matrixlu.jl,
 * test/test_matrixluci.jl, test/test_batcheval.jl and test/test_tensorci2.jl (ported as JSON
 * fixtures under tests/golden/). Julia is absent from this image, so the reference itself
 * cannot be executed; see DESIGN.md "Oracle". The ComplexF64 rrLU / MatrixLUCI restatement
 * (orc_rrlu_c128, orc_luci_c128) is pinned by the complex argmax KAT (test_matrixlu.jl:39-52);
 * its Julia Base pieces (ComplexF64 `/`, abs = hypot) are parity unpinned at their last ulp.
 *
 * Arithmetic contract (matches Julia without @fastmath): compile with -ffp-contract=off so
 * `a - x*y` stays a separate multiply and subtract (matrixlu.jl:318), normalisation is a true
 * division (matrixlu.jl:305/308), argmax compares abs2(x) = x*x with strict '>' in
 * column-major order (matrixlu.jl:70-85).
 *
 * Conventions: matrices are column-major; index sets ("MultiIndex", abstracttensortrain.jl:33)
 * are stored row-major (entry e occupies w consecutive int32 values), values 1-based like Julia.
 * Bonds and sites in this C API are 0-based: Julia site b <-> p = b-1.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int64_t i64;
typedef int32_t i32;

/* ------------------------------------------------------------------ errors */
enum {
    ORC_OK = 0,
    ORC_ERR_ARG = 1,      /* ArgumentError / DimensionMismatch              */
    ORC_ERR_NAN = 2,      /* error("lu.L contains NaNs"), matrixlu.jl:376   */
    ORC_ERR_NONSQ = 3,    /* "Pivot matrix at bond b is not square!"       */
    ORC_ERR_ZERO = 4,     /* "maxsamplevalue is zero!", tensorci2.jl:113    */
    ORC_ERR_TNAN = 5,     /* "Error: NaN in tensor T[b]", tensorci2.jl:706  */
    ORC_ERR_ALLOC = 6,
    ORC_ERR_CONV = 7      /* unreachable convergence, tensorci2.jl:1068    */
};
static char g_err[512];
const char* orc_last_error(void) { return g_err; }
static int fail(int code, const char* msg) {
    snprintf(g_err, sizeof g_err, "%s", msg);
    return code;
}

/* --------------------------------------------------------- Julia helpers */
/* Base.max for Float64: NaN-propagating, max(-0.0, 0.0) == 0.0. */
static double jl_max(double x, double y) {
    int ysel = (y > x) || (signbit(y) < signbit(x));
    if (ysel) return isnan(x) ? x : y;
    return isnan(y) ? y : x;
}

/* counter-based U[0,1) generator used for every synthetic input (also on the GPU). */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
void orc_fill_uniform(double* a, i64 n, uint64_t seed, i64 offset) {
    for (i64 i = 0; i < n; ++i)
        a[i] = (double)(splitmix64(seed * 0xD1B54A32D192ED03ull + (uint64_t)(offset + i)) >> 11) *
               0x1.0p-53;
}

/* ------------------------------------------------------- integrand catalog
 * The user's f is Julia code in the reference; here it is a fixed catalog (DESIGN.md,
 * "Integrand catalog"), evaluated one multi-index at a time exactly as
 * _batchevaluate_dispatch does (batcheval.jl:157-171). x is 1-based, length L. */
enum {
    F_SUM = 0, F_LORENTZ = 1, F_TABLE = 2, F_GAUSS = 3, F_GAUSSMIX = 4,
    F_QOSC = 5, F_QEXP = 6, F_TT = 7, F_CP = 8, F_MPO = 9
};
typedef struct {
    int kind;
    int L;
    const i32* localdims;
    const double* p;
    i64 np;
} orc_func;

static double quantics_x(const i32* x, int L) {
    /* QuanticsGrids.DiscretizedGrid{1}(R, 0, 1): bits big-endian, x = (i-1)/2^R. */
    uint64_t idx = 0;
    for (int t = 0; t < L; ++t) idx = (idx << 1) | (uint64_t)(x[t] - 1);
    return ldexp((double)idx, -L);
}

/* Contraction(A, B) at one point (contraction.jl:365-406): evaluate splits at midpoint = N / 2,
 * the left environment of sites 1..midpoint (evaluateleft, :279-310, built with _extend_cache,
 * :253-259: tmp1 = oldcache^T-contracted with a[:, i, :, :], then with b[:, :, j, :]), the right
 * one of the rest (evaluateright, :323-354, the same on the mirrored cores), and
 * sum(left .* right). p: [N, per site (ra, d1, d2, ra', rb, d3, rb', offA, offB), cores]. */
static double mpo_eval(const double* p, const i32* x) {
    int N = (int)p[0];
    const double* data = p + 1 + 9 * N;
    static double envL[4096], envR[4096], tmp[16384];
    int mid = N / 2;
    int la = 1, lb = 1, ra_ = 1, rb_ = 1;
    envL[0] = 1.0;
    for (int t = 0; t < mid; ++t) {
        const double* q = p + 1 + 9 * t;
        int ra = (int)q[0], d1 = (int)q[1], d2 = (int)q[2], ra2 = (int)q[3];
        int rb = (int)q[4], d3 = (int)q[5], rb2 = (int)q[6];
        const double* A = data + (i64)q[7];
        const double* B = data + (i64)q[8];
        int s1 = (x[t] - 1) % d1, s3 = (x[t] - 1) / d1;
        /* tmp1[b, s2, a'] = sum_a old[a, b] a[a, s1, s2, a'] */
        for (int a2 = 0; a2 < ra2; ++a2)
            for (int s2 = 0; s2 < d2; ++s2)
                for (int b = 0; b < rb; ++b) {
                    double acc = 0.0;
                    for (int a = 0; a < ra; ++a)
                        acc = acc + envL[a + ra * b] * A[a + (i64)ra * (s1 + (i64)d1 * (s2 + (i64)d2 * a2))];
                    tmp[b + rb * (s2 + d2 * a2)] = acc;
                }
        /* new[a', b'] = sum_{s2, b} tmp1[b, s2, a'] b[b, s2, s3, b'] */
        for (int b2 = 0; b2 < rb2; ++b2)
            for (int a2 = 0; a2 < ra2; ++a2) {
                double acc = 0.0;
                for (int s2 = 0; s2 < d2; ++s2)
                    for (int b = 0; b < rb; ++b)
                        acc = acc + tmp[b + rb * (s2 + d2 * a2)] * B[b + (i64)rb * (s2 + (i64)d2 * (s3 + (i64)d3 * b2))];
                envL[a2 + ra2 * b2] = acc;
            }
        la = ra2;
        lb = rb2;
    }
    envR[0] = 1.0;
    for (int t = N - 1; t >= mid; --t) {
        const double* q = p + 1 + 9 * t;
        int ra = (int)q[0], d1 = (int)q[1], d2 = (int)q[2], ra2 = (int)q[3];
        int rb = (int)q[4], d3 = (int)q[5], rb2 = (int)q[6];
        const double* A = data + (i64)q[7];
        const double* B = data + (i64)q[8];
        int s1 = (x[t] - 1) % d1, s3 = (x[t] - 1) / d1;
        /* tmp[a, s2, b'] = sum_a' a[a, s1, s2, a'] old[a', b'] */
        for (int b2 = 0; b2 < rb2; ++b2)
            for (int s2 = 0; s2 < d2; ++s2)
                for (int a = 0; a < ra; ++a) {
                    double acc = 0.0;
                    for (int a2 = 0; a2 < ra2; ++a2)
                        acc = acc + A[a + (i64)ra * (s1 + (i64)d1 * (s2 + (i64)d2 * a2))] * envR[a2 + ra2 * b2];
                    tmp[a + ra * (s2 + d2 * b2)] = acc;
                }
        /* new[a, b] = sum_{b', s2} tmp[a, s2, b'] b[b, s2, s3, b'] */
        for (int b = 0; b < rb; ++b)
            for (int a = 0; a < ra; ++a) {
                double acc = 0.0;
                for (int b2 = 0; b2 < rb2; ++b2)
                    for (int s2 = 0; s2 < d2; ++s2)
                        acc = acc + tmp[a + ra * (s2 + d2 * b2)] * B[b + (i64)rb * (s2 + (i64)d2 * (s3 + (i64)d3 * b2))];
                envR[a + ra * b] = acc;
            }
        ra_ = ra;
        rb_ = rb;
    }
    (void)ra_;
    (void)rb_;
    double res = 0.0;
    for (int e = 0; e < la * lb; ++e) res = res + envL[e] * envR[e];
    return res;
}

static double feval(const orc_func* f, const i32* x) {
    const double* p = f->p;
    int L = f->L;
    switch (f->kind) {
    case F_SUM: {
        i64 s = 0;
        for (int t = 0; t < L; ++t) s += x[t];
        return (double)s;
    }
    case F_LORENTZ: {
        i64 s = 0;
        for (int t = 0; t < L; ++t) s += (i64)x[t] * x[t];
        return p[0] / (double)(s + 1);
    }
    case F_TABLE: {
        i64 off = 0, stride = 1;
        for (int t = 0; t < L; ++t) {
            off += (i64)(x[t] - 1) * stride;
            stride *= f->localdims[t];
        }
        return p[off];
    }
    case F_GAUSS: {
        double s = 0.0;
        for (int t = 0; t < L; ++t) {
            double u = (double)x[t] - p[1];
            s = s + u * u;
        }
        return exp(-(p[0] * s));
    }
    case F_GAUSSMIX: {
        int K = (int)p[0];
        double a = p[1];
        const double* c = p + 2;
        const double* w = p + 2 + (i64)K * L;
        double acc = 0.0;
        for (int k = 0; k < K; ++k) {
            double s = 0.0;
            for (int t = 0; t < L; ++t) {
                double u = (double)x[t] - c[(i64)k * L + t];
                s = s + u * u;
            }
            acc = acc + w[k] * exp(-(a * s));
        }
        return acc;
    }
    case F_QOSC: {
        double xx = quantics_x(x, L);
        return exp(-(p[0] * xx)) * sin(p[1] * pow(xx, p[2]));
    }
    case F_QEXP: {
        double xx = quantics_x(x, L);
        return p[0] * exp(-(p[1] * xx)) + p[2] * exp(-(p[3] * xx));
    }
    case F_TT: {
        /* p = [r_0 .. r_L, core_0, core_1, ...], core_t is (r_t, d_t, r_{t+1}) col-major.
         * evaluate(tt, idx) = only(prod(T[:, i, :])), abstracttensortrain.jl:328-342. */
        const double* r = p;
        const double* core = p + L + 1;
        int r0 = (int)r[0];
        double v[4096], w2[4096];
        /* row vector of length r_1 from core_0[0, x0, :] (r_0 == 1) */
        (void)r0;
        int rl = (int)r[1];
        int d0 = f->localdims[0];
        for (int b = 0; b < rl; ++b) v[b] = core[0 + (i64)(x[0] - 1) * 1 + (i64)b * d0];
        core += (i64)r[0] * d0 * rl;
        for (int t = 1; t < L; ++t) {
            int ra = (int)r[t], rb = (int)r[t + 1], d = f->localdims[t];
            for (int b = 0; b < rb; ++b) {
                double s = 0.0;
                for (int a = 0; a < ra; ++a)
                    s = s + v[a] * core[a + (i64)ra * (x[t] - 1) + (i64)ra * d * b];
                w2[b] = s;
            }
            memcpy(v, w2, sizeof(double) * rb);
            core += (i64)ra * d * rb;
        }
        return v[0];
    }
    case F_MPO:
        return mpo_eval(p, x);
    case F_CP: {
        /* CP-rank-K synthetic of SURVEY.md 8(d) (config 5): sum_k prod_t g[k][t][x_t];
         * p = [K, dmax, g (K x L x dmax, dmax fastest)] */
        int K = (int)p[0], dmax = (int)p[1];
        const double* g = p + 2;
        double acc = 0.0;
        for (int k = 0; k < K; ++k) {
            double prod = 1.0;
            for (int t = 0; t < L; ++t) prod = prod * g[((i64)k * L + t) * dmax + (x[t] - 1)];
            acc = acc + prod;
        }
        return acc;
    }
    }
    return NAN;
}

double orc_feval(int kind, const double* p, i64 np, const i32* localdims, int L, const i32* x) {
    orc_func f = {kind, L, localdims, p, np};
    return feval(&f, x);
}

#ifdef ORC_FAST
/* ------------------------------------------------------------------ fast mode
 * liboracle_fast.so (oracle/Makefile: -DORC_FAST -fopenmp, with cpu_rrlu_omp.c) exists for the
 * one config whose loop-for-loop restatement would take the CPU many hours: config 5 as stated
 * (12 legs of d = 32, CP rank 1024, maxbonddim 1024; Pi up to 32768^2). It changes three things
 * and nothing else:
 *  1. rrlu runs on cpu_rrlu_inplace_omp, bitwise equal to orc_rrlu_inplace
 *     (tests/test_oracle_kats.py::test_omp_baseline_bitwise_equals_oracle);
 *  2. the CP integrand is evaluated factorised at the bond: f(x) = sum_k EL[k, R] * ER[k, j] with
 *     EL = prod of g over the row legs (and the centre leg) in leg order, ER the same over the
 *     column legs, k ascending, one multiply and one add per term -- the same function, another
 *     association of its product (the product path evaluates it the same way, EL^T ER on fp64
 *     MFMA, so f is compared at tolerance, as for every transcendental/separable kind);
 *  3. setsitetensor! fills Pi1 (it updates maxsample, tensorci2.jl:610) and checks the pivot
 *     matrix is square, but skips the solve: in deterministic mode the solved tensors are never
 *     read -- the final sweep1site!(updatetensors) overwrites every site tensor
 *     (tensorci2.jl:683-716) before anything evaluates the tensor train.
 * The MatrixLUCI factors run their rows / columns in parallel (each entry's arithmetic unchanged). */
#include <omp.h>
int cpu_rrlu_inplace_omp(double* A, i64 m, i64 n, i64 lda, i64 maxrank, double reltol,
                         double abstol, int leftorth, i64* rowperm, i64* colperm, i64* npivot,
                         double* err, i64 pivot_limit);

typedef double v4d __attribute__((vector_size(32)));
enum { CP_MR = 8, CP_NR = 4, CP_KC = 256 };

/* E[k * ld + R] = prod of g[k][t0 + q][e_q - 1] over q (and the centre leg), in leg order */
static void cp_factors(const orc_func* f, const i32* T, i64 cnt_rows, int cnt, int M, i64 D,
                       int t0, double* E, i64 ld) {
    const double* p = f->p;
    const int L = f->L, K = (int)p[0], dmax = (int)p[1];
    const double* g0 = p + 2;
#pragma omp parallel for schedule(static)
    for (int k = 0; k < K; ++k) {
        const double* g = g0 + (i64)k * L * dmax;
        for (i64 R = 0; R < cnt_rows * D; ++R) {
            const i64 i = R % cnt_rows, c = R / cnt_rows;
            const i32* e = T + i * cnt;
            double prod = 1.0;
            for (int q = 0; q < cnt; ++q) prod = prod * g[(i64)(t0 + q) * dmax + (e[q] - 1)];
            if (M) prod = prod * g[(i64)(t0 + cnt) * dmax + c];
            E[(i64)k * ld + R] = prod;
        }
        for (i64 R = cnt_rows * D; R < ld; ++R) E[(i64)k * ld + R] = 0.0;
    }
}

/* out[R + mR j] = sum_k EL[k, R] ER[k, j], k ascending: a packed register-tile GEMM (CP_MR rows x
 * CP_NR columns per tile, all K terms of a tile summed in one pass in k order) */
static void cp_gemm(const double* EL, i64 mR, const double* ER, i64 n, int K, double* out) {
    const i64 nrb = (mR + CP_MR - 1) / CP_MR, ncb = (n + CP_NR - 1) / CP_NR;
    /* pack: Ap[rb][k][CP_MR], Bp[cb][k][CP_NR] (zero-padded at the edges) */
    double* Ap = (double*)aligned_alloc(64, sizeof(double) * (size_t)(nrb * K * CP_MR));
    double* Bp = (double*)aligned_alloc(64, sizeof(double) * (size_t)(ncb * K * CP_NR));
#pragma omp parallel for schedule(static)
    for (i64 rb = 0; rb < nrb; ++rb)
        for (int k = 0; k < K; ++k)
            for (int r = 0; r < CP_MR; ++r) {
                const i64 R = rb * CP_MR + r;
                Ap[(rb * K + k) * CP_MR + r] = R < mR ? EL[(i64)k * mR + R] : 0.0;
            }
#pragma omp parallel for schedule(static)
    for (i64 cb = 0; cb < ncb; ++cb)
        for (int k = 0; k < K; ++k)
            for (int c = 0; c < CP_NR; ++c) {
                const i64 j = cb * CP_NR + c;
                Bp[(cb * K + k) * CP_NR + c] = j < n ? ER[(i64)k * n + j] : 0.0;
            }
    /* a task = 16 column tiles; per row tile the K terms go in panels of CP_KC (the tile's A panel
     * stays in L1 while the task's B panels stream from L2), the running sums of the 16 tiles
     * carried in a small buffer between panels: every sum still adds its terms in k order */
    const i64 cbs = 16, ntask = (ncb + cbs - 1) / cbs;
#pragma omp parallel for schedule(dynamic, 1)
    for (i64 task = 0; task < ntask; ++task) {
        const i64 cb0 = task * cbs, cb1 = cb0 + cbs < ncb ? cb0 + cbs : ncb;
        v4d st[16][CP_NR][2];
        for (i64 rb = 0; rb < nrb; ++rb) {
            for (int kp = 0; kp < K; kp += CP_KC) {
                const int kc = K - kp < CP_KC ? K - kp : CP_KC;
                const double* a = Ap + (rb * K + kp) * CP_MR;
                for (i64 cb = cb0; cb < cb1; ++cb) {
                    const double* b = Bp + (cb * K + kp) * CP_NR;
                    v4d acc[CP_NR][2];
                    for (int c = 0; c < CP_NR; ++c) {
                        acc[c][0] = kp ? st[cb - cb0][c][0] : (v4d){0.0, 0.0, 0.0, 0.0};
                        acc[c][1] = kp ? st[cb - cb0][c][1] : (v4d){0.0, 0.0, 0.0, 0.0};
                    }
                    for (int k = 0; k < kc; ++k) {
                        v4d a0, a1;
                        memcpy(&a0, a + k * CP_MR, sizeof a0);
                        memcpy(&a1, a + k * CP_MR + 4, sizeof a1);
                        for (int c = 0; c < CP_NR; ++c) {
                            const double bv = b[k * CP_NR + c];
                            const v4d bb = {bv, bv, bv, bv};
                            acc[c][0] = acc[c][0] + a0 * bb;
                            acc[c][1] = acc[c][1] + a1 * bb;
                        }
                    }
                    for (int c = 0; c < CP_NR; ++c) {
                        st[cb - cb0][c][0] = acc[c][0];
                        st[cb - cb0][c][1] = acc[c][1];
                    }
                }
            }
            for (i64 cb = cb0; cb < cb1; ++cb)
                for (int c = 0; c < CP_NR; ++c) {
                    const i64 j = cb * CP_NR + c;
                    if (j >= n) break;
                    double v[CP_MR];
                    memcpy(v, &st[cb - cb0][c][0], sizeof(v4d));
                    memcpy(v + 4, &st[cb - cb0][c][1], sizeof(v4d));
                    for (int r = 0; r < CP_MR; ++r) {
                        const i64 R = rb * CP_MR + r;
                        if (R < mR) out[R + mR * j] = v[r];
                    }
                }
        }
    }
    free(Ap);
    free(Bp);
}

static void batcheval_cp_fast(const orc_func* f, const i32* I, i64 m, int nl, const i32* J, i64 n,
                              int nr, int M, double* out) {
    const int K = (int)f->p[0];
    const i64 D = M ? f->localdims[nl] : 1, mR = m * D;
    double* EL = (double*)malloc(sizeof(double) * (size_t)(K * mR + 1));
    double* ER = (double*)malloc(sizeof(double) * (size_t)(K * n + 1));
    double t0 = omp_get_wtime();
    cp_factors(f, I, m, nl, M, D, 0, EL, mR);
    cp_factors(f, J, n, nr, 0, 1, f->L - nr, ER, n);
    double t1 = omp_get_wtime();
    cp_gemm(EL, mR, ER, n, K, out);
    if (getenv("ORC_FAST_PROF"))
        fprintf(stderr, "cp %ld x %ld K=%d: factors %.3f s, gemm %.3f s\n", (long)mR, (long)n, K, t1 - t0,
                omp_get_wtime() - t1);
    free(EL);
    free(ER);
}
#endif

/* _batchevaluate_dispatch (batcheval.jl:131-175): result[i, c, j] = f([I_i..., c..., J_j...]),
 * loops i, c, j nested with j innermost. I: m x nl (row-major per entry), J: n x nr.
 * out is column-major (m, prod(d_c), n). Returns maxabs(init, out) via *maxabs (util.jl:34). */
static void batcheval(const orc_func* f, const i32* I, i64 m, int nl, const i32* J, i64 n, int nr,
                      int M, double* out, double* maxabs) {
#ifdef ORC_FAST
    if (f->kind == F_CP && m > 0 && n > 0) {
        batcheval_cp_fast(f, I, m, nl, J, n, nr, M, out);
        if (maxabs) {
            double mx = *maxabs;
            const i64 tot = m * (M ? f->localdims[nl] : 1) * n;
            for (i64 e = 0; e < tot; ++e) mx = jl_max(fabs(mx), fabs(out[e]));
            *maxabs = mx;
        }
        return;
    }
#endif
    int L = nl + M + nr;
    i32 x[512];
    i64 D = 1;
    for (int c = 0; c < M; ++c) D *= f->localdims[nl + c];
    double mx = maxabs ? *maxabs : 0.0;
    for (i64 i = 0; i < m; ++i) {
        for (i64 c = 0; c < D; ++c) {
            i64 cc = c;
            for (int t = 0; t < M; ++t) {
                int d = f->localdims[nl + t];
                x[nl + t] = (i32)(cc % d) + 1;
                cc /= d;
            }
            for (i64 j = 0; j < n; ++j) {
                for (int t = 0; t < nl; ++t) x[t] = I[i * nl + t];
                for (int t = 0; t < nr; ++t) x[nl + M + t] = J[j * nr + t];
                double v = feval(f, x);
                out[i + m * c + m * D * j] = v;
            }
        }
    }
    (void)L;
    if (maxabs) {
        i64 tot = m * D * n;
        for (i64 e = 0; e < tot; ++e) mx = jl_max(fabs(mx), fabs(out[e]));
        *maxabs = mx;
    }
}

int orc_batcheval(int kind, const double* p, i64 np, const i32* localdims, int L, const i32* I,
                  i64 m, int nl, const i32* J, i64 n, int nr, int M, double* out, double* maxabs) {
    if (nl + M + nr != L) return fail(ORC_ERR_ARG, "Invalid number of central indices");
    orc_func f = {kind, L, localdims, p, np};
    batcheval(&f, I, m, nl, J, n, nr, M, out, maxabs);
    return ORC_OK;
}

/* ---------------------------------------------------------------- rrLU */
/* submatrixargmax (matrixlu.jl:46-87): fkind 0 = identity, 1 = abs2. rows/cols are 0-based
 * lists. Column-major scan, strict '>', init typemin = -Inf: ties -> smallest column, then
 * smallest row; NaN never selected. */
int orc_submatrixargmax(const double* A, i64 lda, i64 nrowsA, i64 ncolsA, const i64* rows, i64 nr,
                        const i64* cols, i64 nc, int fkind, i64* mr, i64* mc) {
    if (nr <= 0) return fail(ORC_ERR_ARG, "rows must not be empty");
    if (nc <= 0) return fail(ORC_ERR_ARG, "cols must not be empty");
    for (i64 a = 0; a < nr; ++a)
        if (rows[a] < 0 || rows[a] >= nrowsA)
            return fail(ORC_ERR_ARG, "rows \xe2\x8a\x86 axes(A, 1) must be satified");
    for (i64 a = 0; a < nc; ++a)
        if (cols[a] < 0 || cols[a] >= ncolsA)
            return fail(ORC_ERR_ARG, "cols \xe2\x8a\x86 axes(A, 2) must be satified");
    double m = -INFINITY;
    i64 br = rows[0], bc = cols[0];
    for (i64 b = 0; b < nc; ++b) {
        i64 c = cols[b];
        for (i64 a = 0; a < nr; ++a) {
            i64 r = rows[a];
            double x = A[r + c * lda];
            double v = fkind ? x * x : x;
            int newm = v > m;
            if (newm) { m = v; br = r; bc = c; }
        }
    }
    *mr = br;
    *mc = bc;
    return ORC_OK;
}

/* trailing-block argmax used by _optimizerrlu! (matrixlu.jl:359, startindex form :133) */
static void argmax_trailing(const double* A, i64 lda, i64 m, i64 n, i64 k, i64* pr, i64* pc) {
    double best = -INFINITY;
    i64 br = k, bc = k;
    for (i64 c = k; c < n; ++c) {
        const double* col = A + c * lda;
        for (i64 r = k; r < m; ++r) {
            double v = col[r] * col[r];
            if (v > best) { best = v; br = r; bc = c; }
        }
    }
    *pr = br;
    *pc = bc;
}

/* addpivot! (matrixlu.jl:295-322) including swaprow!/swapcol! (:254-275) */
static void addpivot(double* A, i64 lda, i64 m, i64 n, i64 k, i64 p, i64 q, int leftorth,
                     i64* rowperm, i64* colperm) {
    i64 t;
    t = rowperm[k]; rowperm[k] = rowperm[p]; rowperm[p] = t;
    for (i64 j = 0; j < n; ++j) {
        double a = A[k + j * lda];
        A[k + j * lda] = A[p + j * lda];
        A[p + j * lda] = a;
    }
    t = colperm[k]; colperm[k] = colperm[q]; colperm[q] = t;
    for (i64 i = 0; i < m; ++i) {
        double a = A[i + k * lda];
        A[i + k * lda] = A[i + q * lda];
        A[i + q * lda] = a;
    }
    double piv = A[k + k * lda];
    if (leftorth) {
        for (i64 i = k + 1; i < m; ++i) A[i + k * lda] = A[i + k * lda] / piv;
    } else {
        for (i64 j = k + 1; j < n; ++j) A[k + j * lda] = A[k + j * lda] / piv;
    }
    const double* x = A + k * lda;
    for (i64 j = k + 1; j < n; ++j) {
        double y = A[k + j * lda];
        double* col = A + j * lda;
        for (i64 i = k + 1; i < m; ++i) {
            double prod = x[i] * y;
            col[i] = col[i] - prod;
        }
    }
}

/* _optimizerrlu! loop (matrixlu.jl:346-369) in place on A. Permutations 0-based.
 * pivot_limit >= 0 stops after that many pivots (bounded CPU-baseline sample only). */
int orc_rrlu_inplace(double* A, i64 m, i64 n, i64 lda, i64 maxrank, double reltol, double abstol,
                     int leftorth, i64* rowperm, i64* colperm, i64* npivot, double* err,
                     i64 pivot_limit) {
    for (i64 i = 0; i < m; ++i) rowperm[i] = i;
    for (i64 j = 0; j < n; ++j) colperm[j] = j;
    i64 mr = maxrank;
    if (mr > m) mr = m;
    if (mr > n) mr = n;
    double maxerror = 0.0, error = NAN;
    i64 np = 0;
    while (np < mr) {
        if (pivot_limit >= 0 && np >= pivot_limit) break;
        i64 k = np, p, q;
        argmax_trailing(A, lda, m, n, k, &p, &q);
        error = fabs(A[p + q * lda]);
        if ((fabs(error) < reltol * maxerror || fabs(error) < abstol) && np > 0) break;
        maxerror = jl_max(maxerror, error);
        addpivot(A, lda, m, n, k, p, q, leftorth, rowperm, colperm);
        np += 1;
    }
    i64 mn = m < n ? m : n;
    if (np >= mn) error = 0.0;
    *npivot = np;
    *err = error;
    return ORC_OK;
}

/* L = tril(A[:, 1:np]), U = triu(A[1:np, :]), NaN checks, unit diagonal (matrixlu.jl:372-388).
 * L: m x np (ld m), U: np x n (ld np). */
int orc_rrlu_extract(const double* A, i64 m, i64 n, i64 lda, i64 np, int leftorth, double* L,
                     double* U) {
    for (i64 c = 0; c < np; ++c)
        for (i64 r = 0; r < m; ++r) L[r + c * m] = (r >= c) ? A[r + c * lda] : 0.0;
    for (i64 c = 0; c < n; ++c)
        for (i64 r = 0; r < np; ++r) U[r + c * np] = (r <= c) ? A[r + c * lda] : 0.0;
    for (i64 e = 0; e < m * np; ++e)
        if (isnan(L[e])) return fail(ORC_ERR_NAN, "lu.L contains NaNs");
    for (i64 e = 0; e < np * n; ++e)
        if (isnan(U[e])) return fail(ORC_ERR_NAN, "lu.U contains NaNs");
    if (leftorth) {
        for (i64 c = 0; c < np; ++c) L[c + c * m] = 1.0;
    } else {
        for (i64 c = 0; c < np; ++c) U[c + c * np] = 1.0;
    }
    return ORC_OK;
}

typedef struct {
    i64 m, n, np;
    int leftorth;
    double error;
    i64* rowperm;
    i64* colperm;
    double* L;
    double* U;
} orc_lu;

static void lu_free(orc_lu* lu) {
    free(lu->rowperm); free(lu->colperm); free(lu->L); free(lu->U);
    memset(lu, 0, sizeof *lu);
}

/* rrlu(A) = rrlu!(copy(A)) (matrixlu.jl:455-463) */
static int rrlu_copy(const double* A, i64 m, i64 n, i64 maxrank, double reltol, double abstol,
                     int leftorth, orc_lu* lu) {
    memset(lu, 0, sizeof *lu);
    double* W = (double*)malloc(sizeof(double) * (size_t)(m * n > 0 ? m * n : 1));
    lu->rowperm = (i64*)malloc(sizeof(i64) * (size_t)(m > 0 ? m : 1));
    lu->colperm = (i64*)malloc(sizeof(i64) * (size_t)(n > 0 ? n : 1));
    if (!W || !lu->rowperm || !lu->colperm) return fail(ORC_ERR_ALLOC, "alloc");
#ifdef ORC_FAST
    /* first touch by the threads that update these columns (static contiguous column blocks, as
     * in cpu_rrlu_inplace_omp): on a multi-socket host the pages land on their NUMA node */
#pragma omp parallel for schedule(static)
    for (i64 j = 0; j < n; ++j) memcpy(W + j * m, A + j * m, sizeof(double) * (size_t)m);
#else
    memcpy(W, A, sizeof(double) * (size_t)(m * n));
#endif
    lu->m = m; lu->n = n; lu->leftorth = leftorth;
#ifdef ORC_FAST
    cpu_rrlu_inplace_omp(W, m, n, m, maxrank, reltol, abstol, leftorth, lu->rowperm, lu->colperm,
                         &lu->np, &lu->error, -1);
#else
    orc_rrlu_inplace(W, m, n, m, maxrank, reltol, abstol, leftorth, lu->rowperm, lu->colperm,
                     &lu->np, &lu->error, -1);
#endif
    lu->L = (double*)malloc(sizeof(double) * (size_t)(m * lu->np + 1));
    lu->U = (double*)malloc(sizeof(double) * (size_t)(lu->np * n + 1));
    int st = orc_rrlu_extract(W, m, n, m, lu->np, leftorth, lu->L, lu->U);
    free(W);
    return st;
}

/* pivoterrors (matrixlu.jl:799): [|diag|..., error]; diag from U if leftorth else L (:756) */
static void lu_pivoterrors(const orc_lu* lu, double* out) {
    for (i64 k = 0; k < lu->np; ++k)
        out[k] = lu->leftorth ? fabs(lu->U[k + k * lu->np]) : fabs(lu->L[k + k * lu->m]);
    out[lu->np] = lu->error;
}

/* MatrixLUCI left/right factors (matrixluci.jl:161-283). out column-major. */
static void luci_left(const orc_lu* lu, double* out /* m x np */) {
    i64 m = lu->m, np = lu->np;
    const double* L = lu->L;
    if (lu->leftorth) {
        /* colstimespivotinv: [I; L21 / LowerTriangular(L11)] then result[rowperm,:] = result */
        double* res = (double*)calloc((size_t)(m * np + 1), sizeof(double));
        for (i64 i = 0; i < np; ++i) res[i + i * m] = 1.0;
#ifdef ORC_FAST
#pragma omp parallel for schedule(dynamic, 64)
#endif
        for (i64 i = np; i < m; ++i) {
            for (i64 j = np - 1; j >= 0; --j) {
                double s = L[i + j * m];
                for (i64 t = j + 1; t < np; ++t) s = s - res[i + t * m] * L[t + j * m];
                res[i + j * m] = s / L[j + j * m];
            }
        }
        for (i64 i = 0; i < m; ++i)
            for (i64 j = 0; j < np; ++j) out[lu->rowperm[i] + j * m] = res[i + j * m];
        free(res);
    } else {
        /* colmatrix: left(lu) * right(lu, permute=false)[:, 1:np] */
        const double* U = lu->U;
#ifdef ORC_FAST
#pragma omp parallel for schedule(dynamic, 64)
#endif
        for (i64 i = 0; i < m; ++i)
            for (i64 j = 0; j < np; ++j) {
                double s = 0.0;
                for (i64 t = 0; t < np; ++t) s = s + L[i + t * m] * U[t + j * np];
                out[lu->rowperm[i] + j * m] = s;
            }
    }
}

static void luci_right(const orc_lu* lu, double* out /* np x n */) {
    i64 n = lu->n, np = lu->np, m = lu->m;
    const double* U = lu->U;
    if (lu->leftorth) {
        /* rowmatrix: left(lu, permute=false)[1:np, :] * right(lu) */
        const double* L = lu->L;
#ifdef ORC_FAST
#pragma omp parallel for schedule(dynamic, 64)
#endif
        for (i64 j = 0; j < n; ++j)
            for (i64 a = 0; a < np; ++a) {
                double s = 0.0;
                for (i64 t = 0; t < np; ++t) s = s + L[a + t * m] * U[t + j * np];
                out[a + lu->colperm[j] * np] = s;
            }
    } else {
        /* pivotinvtimesrows: [I, UpperTriangular(U11) \ U12], result[:, colperm] = result */
        double* res = (double*)calloc((size_t)(np * n + 1), sizeof(double));
        for (i64 i = 0; i < np; ++i) res[i + i * np] = 1.0;
#ifdef ORC_FAST
#pragma omp parallel for schedule(dynamic, 64)
#endif
        for (i64 c = np; c < n; ++c) {
            for (i64 a = np - 1; a >= 0; --a) {
                double s = U[a + c * np];
                for (i64 t = a + 1; t < np; ++t) s = s - U[a + t * np] * res[t + c * np];
                res[a + c * np] = s / U[a + a * np];
            }
        }
        for (i64 j = 0; j < n; ++j)
            for (i64 a = 0; a < np; ++a) out[a + lu->colperm[j] * np] = res[a + j * np];
        free(res);
    }
    (void)m;
}

/* Full rrlu + MatrixLUCI export for tests. rowperm/colperm 0-based, L m x maxrank (ld m),
 * U maxrank x n (ld maxrank) -- only the first np columns/rows are written. left m x maxrank,
 * right maxrank x n (ld maxrank); pass NULL to skip. */
int orc_rrlu(const double* A, i64 m, i64 n, i64 maxrank, double reltol, double abstol,
             int leftorth, i64* rowperm, i64* colperm, double* L, double* U, double* left,
             double* right, i64* npivot, double* lasterr, double* pivoterrs) {
    orc_lu lu;
    int st = rrlu_copy(A, m, n, maxrank, reltol, abstol, leftorth, &lu);
    if (st) { lu_free(&lu); return st; }
    i64 np = lu.np;
    *npivot = np;
    *lasterr = lu.error;
    memcpy(rowperm, lu.rowperm, sizeof(i64) * (size_t)m);
    memcpy(colperm, lu.colperm, sizeof(i64) * (size_t)n);
    if (L) memcpy(L, lu.L, sizeof(double) * (size_t)(m * np));
    if (U) memcpy(U, lu.U, sizeof(double) * (size_t)(np * n));
    if (pivoterrs) lu_pivoterrors(&lu, pivoterrs);
    if (left) luci_left(&lu, left);
    if (right) luci_right(&lu, right);
    lu_free(&lu);
    return ORC_OK;
}

/* ----------------------------------------------------- shared-divisor division check
 * Test support for the device's div_shared (tensorcrossinterpolation.jl_amd/csrc/tci_sweep_small.hip):
 * y = 1 / p once, then q = x y, r = fma(-p, q, x), q' = fma(r, y, q) must equal x / p bit for bit
 * (Markstein) for |x|, |p| in [2^-400, 2^400]. n random pairs (uniform exponents in a few ranges,
 * significands near all-ones / all-zeros); returns the number of mismatches. */
static uint64_t orc_xs(uint64_t* s) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }
static double orc_bits_dbl(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
i64 orc_div_shared_check(i64 n, uint64_t seed) {
    uint64_t s = seed ? seed : 88172645463325252ull;
    i64 bad = 0;
    for (i64 i = 0; i < n; ++i) {
        double x, p;
        const int mode = (int)(i % 4);
        uint64_t mx = orc_xs(&s) & 0xFFFFFFFFFFFFFull, mp = orc_xs(&s) & 0xFFFFFFFFFFFFFull;
        int ex, ep;
        if (mode >= 2) {  /* significands near all-ones or all-zeros */
            mp = (orc_xs(&s) & 1) ? 0xFFFFFFFFFFFFFull - (orc_xs(&s) & 0xFF) : (orc_xs(&s) & 0xFF);
            if (mode == 3) mx = (orc_xs(&s) & 1) ? 0xFFFFFFFFFFFFFull - (orc_xs(&s) & 0xFF) : (orc_xs(&s) & 0xFF);
        }
        const int span = mode == 1 ? 400 : 30;
        ex = (int)(orc_xs(&s) % (uint64_t)(2 * span + 1)) - span;
        ep = (int)(orc_xs(&s) % (uint64_t)(2 * span + 1)) - span;
        if (mode == 1) { ex = ex < -399 ? -399 : ex; ep = ep < -399 ? -399 : ep; }
        x = orc_bits_dbl(((uint64_t)(ex + 1023) << 52) | mx | ((orc_xs(&s) & 1) << 63));
        p = orc_bits_dbl(((uint64_t)(ep + 1023) << 52) | mp | ((orc_xs(&s) & 1) << 63));
        const double y = 1.0 / p;
        const double q = x * y;
        const double r = fma(-p, q, x);
        const double q2 = fma(r, y, q);
        const double t = x / p;
        if (memcmp(&q2, &t, 8)) ++bad;
    }
    return bad;
}

/* ----------------------------------------------------- partial-pivot solve
 * Tmat = transpose(transpose(P) \ transpose(Pi1)) (tensorci2.jl:626): LAPACK getrf/getrs on
 * P^T with partial pivoting (first maximal |a| in the column, like idamax). P: r x r,
 * Pi1: R x r, T out: R x r. */
int orc_sitetensor_solve(const double* P, i64 r, const double* Pi1, i64 R, double* T) {
    double* A = (double*)malloc(sizeof(double) * (size_t)(r * r + 1));
    i64* piv = (i64*)malloc(sizeof(i64) * (size_t)(r + 1));
    double* X = (double*)malloc(sizeof(double) * (size_t)(r * R + 1));
    if (!A || !piv || !X) return fail(ORC_ERR_ALLOC, "alloc");
    for (i64 i = 0; i < r; ++i)
        for (i64 j = 0; j < r; ++j) A[i + j * r] = P[j + i * r]; /* A = P^T */
    for (i64 k = 0; k < r; ++k) {
        i64 p = k;
        double best = fabs(A[k + k * r]);
        for (i64 i = k + 1; i < r; ++i)
            if (fabs(A[i + k * r]) > best) { best = fabs(A[i + k * r]); p = i; }
        piv[k] = p;
        if (p != k)
            for (i64 j = 0; j < r; ++j) {
                double t = A[k + j * r]; A[k + j * r] = A[p + j * r]; A[p + j * r] = t;
            }
        double d = A[k + k * r];
        for (i64 i = k + 1; i < r; ++i) A[i + k * r] = A[i + k * r] / d;
        for (i64 j = k + 1; j < r; ++j) {
            double y = A[k + j * r];
            for (i64 i = k + 1; i < r; ++i) A[i + j * r] = A[i + j * r] - A[i + k * r] * y;
        }
    }
    /* RHS B = Pi1^T (r x R) */
    for (i64 i = 0; i < r; ++i)
        for (i64 c = 0; c < R; ++c) X[i + c * r] = Pi1[c + i * R];
    for (i64 c = 0; c < R; ++c) {
        double* x = X + c * r;
        for (i64 k = 0; k < r; ++k)
            if (piv[k] != k) { double t = x[k]; x[k] = x[piv[k]]; x[piv[k]] = t; }
        for (i64 k = 0; k < r; ++k)
            for (i64 i = k + 1; i < r; ++i) x[i] = x[i] - A[i + k * r] * x[k];
        for (i64 k = r - 1; k >= 0; --k) {
            x[k] = x[k] / A[k + k * r];
            for (i64 i = 0; i < k; ++i) x[i] = x[i] - A[i + k * r] * x[k];
        }
    }
    for (i64 c = 0; c < R; ++c)
        for (i64 i = 0; i < r; ++i) T[c + i * R] = X[i + c * r];
    free(A); free(piv); free(X);
    return ORC_OK;
}

/* ------------------------------------------------------------ index sets */
typedef struct {
    int w;
    i64 n, cap;
    i32* d;
} iset_t;

static void iset_init(iset_t* s, int w) { s->w = w; s->n = 0; s->cap = 0; s->d = NULL; }
static void iset_free(iset_t* s) { free(s->d); s->d = NULL; s->n = s->cap = 0; }
static void iset_push(iset_t* s, const i32* e) {
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 8;
        s->d = (i32*)realloc(s->d, sizeof(i32) * (size_t)(s->cap * (s->w > 0 ? s->w : 1)));
    }
    if (s->w) memcpy(s->d + s->n * s->w, e, sizeof(i32) * (size_t)s->w);
    s->n += 1;
}
static void iset_copy(iset_t* dst, const iset_t* src) {
    iset_init(dst, src->w);
    for (i64 i = 0; i < src->n; ++i) iset_push(dst, src->d + i * src->w);
}

typedef struct {
    i64 cap;
    i64* slot; /* index + 1, 0 = empty */
} hset_t;
static uint64_t hash_e(const i32* e, int w) {
    uint64_t h = 1469598103934665603ull;
    for (int t = 0; t < w; ++t) { h ^= (uint32_t)e[t]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}
static void hset_init(hset_t* h, i64 n) {
    i64 cap = 16;
    while (cap < 2 * n + 2) cap *= 2;
    h->cap = cap;
    h->slot = (i64*)calloc((size_t)cap, sizeof(i64));
}
static void hset_free(hset_t* h) { free(h->slot); h->slot = NULL; }
/* pushunique! (util.jl:94) */
static void iset_pushunique(iset_t* s, const i32* e) {
    for (i64 i = 0; i < s->n; ++i)
        if (s->w == 0 || memcmp(s->d + i * s->w, e, sizeof(i32) * (size_t)s->w) == 0) return;
    iset_push(s, e);
}
/* Julia union(a, b): first-seen order, deduplicated */
static void iset_union(iset_t* out, const iset_t* a, const iset_t* b) {
    iset_init(out, a->w);
    hset_t h;
    hset_init(&h, a->n + (b ? b->n : 0));
    for (int pass = 0; pass < 2; ++pass) {
        const iset_t* s = pass ? b : a;
        if (!s) continue;
        for (i64 i = 0; i < s->n; ++i) {
            const i32* e = s->d + i * s->w;
            /* lookup against out (hash keyed on out's storage) */
            uint64_t pos = hash_e(e, out->w) & (uint64_t)(h.cap - 1);
            int found = 0;
            for (;;) {
                i64 v = h.slot[pos];
                if (v == 0) break;
                if (out->w == 0 ||
                    memcmp(out->d + (v - 1) * out->w, e, sizeof(i32) * (size_t)out->w) == 0) {
                    found = 1;
                    break;
                }
                pos = (pos + 1) & (uint64_t)(h.cap - 1);
            }
            if (!found) {
                iset_push(out, e);
                h.slot[pos] = out->n;
            }
        }
    }
    hset_free(&h);
}
/* kronecker(Iset, d) (tensorci2.jl:512-517): [is..., j], Iset fastest */
static void kron_right(iset_t* out, const iset_t* I, int d) {
    iset_init(out, I->w + 1);
    i32 e[512];
    for (int j = 1; j <= d; ++j)
        for (i64 i = 0; i < I->n; ++i) {
            if (I->w) memcpy(e, I->d + i * I->w, sizeof(i32) * (size_t)I->w);
            e[I->w] = j;
            iset_push(out, e);
        }
}
/* kronecker(d, Jset) (tensorci2.jl:524-529): [i, js...], i fastest */
static void kron_left(iset_t* out, int d, const iset_t* J) {
    iset_init(out, J->w + 1);
    i32 e[512];
    for (i64 j = 0; j < J->n; ++j)
        for (int i = 1; i <= d; ++i) {
            e[0] = i;
            if (J->w) memcpy(e + 1, J->d + j * J->w, sizeof(i32) * (size_t)J->w);
            iset_push(out, e);
        }
}
static void iset_select(iset_t* out, const iset_t* s, const i64* idx, i64 n) {
    iset_init(out, s->w);
    for (i64 i = 0; i < n; ++i) iset_push(out, s->d + idx[i] * s->w);
}

/* ------------------------------------------------------------ TensorCI2 */
typedef struct {
    int L;
    i32* localdims;
    orc_func f;
    double* params;
    iset_t* I;
    iset_t* J;
    iset_t* hI; /* Iset_history[end] / Jset_history[end]; only the last entry is ever read */
    iset_t* hJ;
    int has_hist;
    double** T;
    i64* Tn;
    double* pe; /* pivoterrors */
    i64 npe;
    double* bonderr;
    double maxsample;
} orc_tci;

static void tci_invalidate(orc_tci* t) {
    for (int p = 0; p < t->L; ++p) { free(t->T[p]); t->T[p] = NULL; t->Tn[p] = 0; }
}

/* addglobalpivots! (tensorci2.jl:335-357) */
int orc_tci_addglobalpivots(orc_tci* t, const i32* piv, int npiv) {
    int L = t->L;
    for (int a = 0; a < npiv; ++a) {
        const i32* pv = piv + (i64)a * L;
        for (int p = 0; p < L; ++p) {
            iset_pushunique(&t->I[p], pv);
            iset_pushunique(&t->J[p], pv + p + 1);
        }
    }
    if (npiv > 0) tci_invalidate(t);
    return ORC_OK;
}

/* TensorCI2{V}(f, localdims, initialpivots) (tensorci2.jl:105-116) */
orc_tci* orc_tci_new(int kind, const double* params, i64 nparams, const i32* localdims, int L,
                     const i32* initialpivots, int npiv, int* status) {
    *status = ORC_OK;
    if (L < 2) { *status = fail(ORC_ERR_ARG, "localdims should have at least 2 elements!"); return NULL; }
    orc_tci* t = (orc_tci*)calloc(1, sizeof(orc_tci));
    t->L = L;
    t->localdims = (i32*)malloc(sizeof(i32) * (size_t)L);
    memcpy(t->localdims, localdims, sizeof(i32) * (size_t)L);
    t->params = (double*)malloc(sizeof(double) * (size_t)(nparams + 1));
    if (nparams) memcpy(t->params, params, sizeof(double) * (size_t)nparams);
    t->f.kind = kind; t->f.L = L; t->f.localdims = t->localdims; t->f.p = t->params; t->f.np = nparams;
    t->I = (iset_t*)calloc((size_t)L, sizeof(iset_t));
    t->J = (iset_t*)calloc((size_t)L, sizeof(iset_t));
    t->hI = (iset_t*)calloc((size_t)L, sizeof(iset_t));
    t->hJ = (iset_t*)calloc((size_t)L, sizeof(iset_t));
    for (int p = 0; p < L; ++p) {
        iset_init(&t->I[p], p); iset_init(&t->J[p], L - 1 - p);
        iset_init(&t->hI[p], p); iset_init(&t->hJ[p], L - 1 - p);
    }
    t->T = (double**)calloc((size_t)L, sizeof(double*));
    t->Tn = (i64*)calloc((size_t)L, sizeof(i64));
    t->bonderr = (double*)calloc((size_t)(L - 1), sizeof(double));
    t->pe = NULL; t->npe = 0;
    orc_tci_addglobalpivots(t, initialpivots, npiv);
    double mx = -INFINITY;
    for (int a = 0; a < npiv; ++a) {
        double v = fabs(feval(&t->f, initialpivots + (i64)a * L));
        mx = (a == 0) ? v : jl_max(mx, v);
    }
    t->maxsample = mx;
    if (!(fabs(t->maxsample) > 0.0)) *status = fail(ORC_ERR_ZERO, "maxsamplevalue is zero!");
    tci_invalidate(t);
    return t;
}

void orc_tci_free(orc_tci* t) {
    if (!t) return;
    for (int p = 0; p < t->L; ++p) {
        iset_free(&t->I[p]); iset_free(&t->J[p]); iset_free(&t->hI[p]); iset_free(&t->hJ[p]);
        free(t->T[p]);
    }
    free(t->I); free(t->J); free(t->hI); free(t->hJ); free(t->T); free(t->Tn);
    free(t->bonderr); free(t->pe); free(t->localdims); free(t->params); free(t);
}

/* updatepivoterror! (tensorci2.jl:252-260) + updatebonderror! via updateerrors! (:281-289) */
static void tci_updateerrors(orc_tci* t, int p, const double* e, i64 ne) {
    t->bonderr[p] = e[ne - 1];
    i64 n = t->npe > ne ? t->npe : ne;
    double* out = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    for (i64 i = 0; i < n; ++i) {
        double a = i < t->npe ? t->pe[i] : 0.0;
        double b = i < ne ? e[i] : 0.0;
        out[i] = jl_max(a, b);
    }
    free(t->pe);
    t->pe = out;
    t->npe = n;
}
static void tci_flushpivoterror(orc_tci* t) { free(t->pe); t->pe = NULL; t->npe = 0; }

/* filltensor for Val(M), rows x cols; returns malloc'ed column-major (|I| * D, |J|) */
static double* filltensor(orc_tci* t, const iset_t* I, const iset_t* J, int M) {
    i64 D = 1;
    for (int c = 0; c < M; ++c) D *= t->localdims[I->w + c];
    double* out = (double*)malloc(sizeof(double) * (size_t)(I->n * D * J->n + 1));
    batcheval(&t->f, I->d, I->n, I->w, J->d, J->n, J->w, M, out, NULL);
    return out;
}
static void updatemaxsample(orc_tci* t, const double* a, i64 n) {
    double mx = t->maxsample;
    for (i64 e = 0; e < n; ++e) mx = jl_max(fabs(mx), fabs(a[e]));
    t->maxsample = mx;
}
static void set_T(orc_tci* t, int p, double* data, i64 n) {
    free(t->T[p]);
    t->T[p] = data;
    t->Tn[p] = n;
}

/* updatepivots! (tensorci2.jl:825-930), :full branch. p is the 0-based bond (sites p, p+1). */
static int tci_updatepivots_x(orc_tci* t, int p, int leftorth, double reltol, double abstol,
                              i64 maxbonddim, const iset_t* extraI, const iset_t* extraJ) {
    tci_invalidate(t);
    iset_t kI, kJ, Ic, Jc;
    kron_right(&kI, &t->I[p], t->localdims[p]);
    kron_left(&kJ, t->localdims[p + 1], &t->J[p + 1]);
    iset_union(&Ic, &kI, (extraI && extraI->n) ? extraI : NULL);
    iset_union(&Jc, &kJ, (extraJ && extraJ->n) ? extraJ : NULL);
    iset_free(&kI); iset_free(&kJ);
    i64 m = Ic.n, n = Jc.n;
    double* Pi = filltensor(t, &Ic, &Jc, 0);
    updatemaxsample(t, Pi, m * n);
    orc_lu lu;
    int st = rrlu_copy(Pi, m, n, maxbonddim, reltol, abstol, leftorth, &lu);
    free(Pi);
    if (st) { lu_free(&lu); iset_free(&Ic); iset_free(&Jc); return st; }
    iset_t nI, nJ;
    iset_select(&nI, &Ic, lu.rowperm, lu.np);
    iset_select(&nJ, &Jc, lu.colperm, lu.np);
    iset_free(&t->I[p + 1]); t->I[p + 1] = nI;
    iset_free(&t->J[p]); t->J[p] = nJ;
    int noextra = !(extraI && extraI->n) && !(extraJ && extraJ->n);
    if (noextra) {
        double* lf = (double*)malloc(sizeof(double) * (size_t)(m * lu.np + 1));
        double* rf = (double*)malloc(sizeof(double) * (size_t)(lu.np * n + 1));
        luci_left(&lu, lf);
        luci_right(&lu, rf);
        set_T(t, p, lf, m * lu.np);
        set_T(t, p + 1, rf, lu.np * n);
    }
    double* e = (double*)malloc(sizeof(double) * (size_t)(lu.np + 1));
    lu_pivoterrors(&lu, e);
    tci_updateerrors(t, p, e, lu.np + 1);
    free(e);
    lu_free(&lu);
    iset_free(&Ic); iset_free(&Jc);
    return ORC_OK;
}

int orc_tci_updatepivots(orc_tci* t, int p, int leftorth, double reltol, double abstol,
                         i64 maxbonddim) {
    if (p < 0 || p >= t->L - 1) return fail(ORC_ERR_ARG, "bond out of range");
    return tci_updatepivots_x(t, p, leftorth, reltol, abstol, maxbonddim, NULL, NULL);
}

/* setsitetensor!(tci, f, b) (tensorci2.jl:599-629) */
static int tci_setsitetensor(orc_tci* t, int p) {
    i64 nI = t->I[p].n, nJ = t->J[p].n, d = t->localdims[p];
    double* Pi1 = filltensor(t, &t->I[p], &t->J[p], 1);
    updatemaxsample(t, Pi1, nI * d * nJ);
    if (p == t->L - 1) {
        set_T(t, p, Pi1, nI * d * nJ);
        return ORC_OK;
    }
    i64 r1 = t->I[p + 1].n;
#ifdef ORC_FAST
    /* fast mode: the solved tensor is never read in deterministic mode (see "fast mode") */
    free(Pi1);
    if (r1 != nJ) {
        char msg[128];
        snprintf(msg, sizeof msg, "Pivot matrix at bond %d is not square!", p + 1);
        return fail(ORC_ERR_NONSQ, msg);
    }
    set_T(t, p, NULL, 0);
    return ORC_OK;
#endif
    double* P = filltensor(t, &t->I[p + 1], &t->J[p], 0);
    if (r1 != nJ) {
        free(P); free(Pi1);
        char msg[128];
        snprintf(msg, sizeof msg, "Pivot matrix at bond %d is not square!", p + 1);
        return fail(ORC_ERR_NONSQ, msg);
    }
    double* T = (double*)malloc(sizeof(double) * (size_t)(nI * d * r1 + 1));
    orc_sitetensor_solve(P, r1, Pi1, nI * d, T);
    free(P); free(Pi1);
    set_T(t, p, T, nI * d * r1);
    return ORC_OK;
}

/* fillsitetensors! (globalsearch.jl:202-208) */
int orc_tci_fillsitetensors(orc_tci* t) {
    for (int p = 0; p < t->L; ++p) {
        int st = tci_setsitetensor(t, p);
        if (st) return st;
    }
    return ORC_OK;
}

/* sweep2site! (tensorci2.jl:1195-1258). sweepstrategy: 0 = :backandforth, 1 = :forward */
int orc_tci_sweep2site(orc_tci* t, int niter, int iter1, double abstol, i64 maxbonddim,
                       int sweepstrategy, int strictlynested, int fillsitetensors) {
    tci_invalidate(t);
    int L = t->L;
    for (int iter = iter1; iter < iter1 + niter; ++iter) {
        iset_t* exI = NULL;
        iset_t* exJ = NULL;
        iset_t* sI = NULL;
        iset_t* sJ = NULL;
        if (!strictlynested && t->has_hist) {
            /* extraIset = Iset_history[end]: snapshot it before it is replaced below */
            sI = (iset_t*)calloc((size_t)L, sizeof(iset_t));
            sJ = (iset_t*)calloc((size_t)L, sizeof(iset_t));
            for (int p = 0; p < L; ++p) { iset_copy(&sI[p], &t->hI[p]); iset_copy(&sJ[p], &t->hJ[p]); }
            exI = sI; exJ = sJ;
        }
        for (int p = 0; p < L; ++p) {
            iset_free(&t->hI[p]); iset_free(&t->hJ[p]);
            iset_copy(&t->hI[p], &t->I[p]); iset_copy(&t->hJ[p], &t->J[p]);
        }
        t->has_hist = 1;
        tci_flushpivoterror(t);
        int fwd = (sweepstrategy == 1) || (sweepstrategy == 0 && (iter % 2 == 1));
        int st = ORC_OK;
        if (fwd) {
            for (int p = 0; p < L - 1 && !st; ++p)
                st = tci_updatepivots_x(t, p, 1, 1e-14, abstol, maxbonddim,
                                        exI ? &exI[p + 1] : NULL, exJ ? &exJ[p] : NULL);
        } else {
            for (int p = L - 2; p >= 0 && !st; --p)
                st = tci_updatepivots_x(t, p, 0, 1e-14, abstol, maxbonddim,
                                        exI ? &exI[p + 1] : NULL, exJ ? &exJ[p] : NULL);
        }
        if (sI) {
            for (int p = 0; p < L; ++p) { iset_free(&sI[p]); iset_free(&sJ[p]); }
            free(sI); free(sJ);
        }
        if (st) return st;
    }
    if (fillsitetensors) return orc_tci_fillsitetensors(t);
    return ORC_OK;
}

/* sweep1site! (tensorci2.jl:659-725) */
int orc_tci_sweep1site(orc_tci* t, int forward, double reltol, double abstol, i64 maxbonddim,
                       int updatetensors) {
    tci_flushpivoterror(t);
    tci_invalidate(t);
    int L = t->L;
    for (int s = 0; s < L - 1; ++s) {
        int p = forward ? s : (L - 1 - s); /* site index b-1 */
        iset_t Is, Js;
        if (forward) { kron_right(&Is, &t->I[p], t->localdims[p]); iset_copy(&Js, &t->J[p]); }
        else { iset_copy(&Is, &t->I[p]); kron_left(&Js, t->localdims[p], &t->J[p]); }
        double* Pi = filltensor(t, &t->I[p], &t->J[p], 1);
        i64 m = Is.n, n = Js.n;
        updatemaxsample(t, Pi, m * n);
        orc_lu lu;
        int st = rrlu_copy(Pi, m, n, maxbonddim, reltol, abstol, forward, &lu);
        free(Pi);
        if (st) { lu_free(&lu); iset_free(&Is); iset_free(&Js); return st; }
        iset_t nI, nJ;
        iset_select(&nI, &Is, lu.rowperm, lu.np);
        iset_select(&nJ, &Js, lu.colperm, lu.np);
        int pi = p + (forward ? 1 : 0), pj = p - (forward ? 0 : 1);
        iset_free(&t->I[pi]); t->I[pi] = nI;
        iset_free(&t->J[pj]); t->J[pj] = nJ;
        if (updatetensors) {
            if (forward) {
                double* lf = (double*)malloc(sizeof(double) * (size_t)(m * lu.np + 1));
                luci_left(&lu, lf);
                set_T(t, p, lf, m * lu.np);
            } else {
                double* rf = (double*)malloc(sizeof(double) * (size_t)(lu.np * n + 1));
                luci_right(&lu, rf);
                set_T(t, p, rf, lu.np * n);
            }
            for (i64 e = 0; e < t->Tn[p]; ++e)
                if (isnan(t->T[p][e])) {
                    lu_free(&lu); iset_free(&Is); iset_free(&Js);
                    char msg[64];
                    snprintf(msg, sizeof msg, "Error: NaN in tensor T[%d]", p + 1);
                    return fail(ORC_ERR_TNAN, msg);
                }
        }
        double* e = (double*)malloc(sizeof(double) * (size_t)(lu.np + 1));
        lu_pivoterrors(&lu, e);
        tci_updateerrors(t, forward ? p : p - 1, e, lu.np + 1);
        free(e);
        lu_free(&lu);
        iset_free(&Is); iset_free(&Js);
    }
    if (updatetensors) {
        int last = forward ? L - 1 : 0;
        double* lt = filltensor(t, &t->I[last], &t->J[last], 1);
        set_T(t, last, lt, t->I[last].n * t->localdims[last] * t->J[last].n);
    }
    return ORC_OK;
}

/* convergencecriterion (tensorci2.jl:947-966) */
int orc_convergencecriterion(const i64* ranks, const double* errors, const i64* ngp, int n,
                             double tolerance, i64 maxbonddim, int ncheckhistory,
                             int checkconvglobalpivot) {
    if (n < ncheckhistory) return 0;
    int all_err = 1, all_gp = 1, all_max = 1;
    i64 minr = INT64_MAX;
    for (int i = n - ncheckhistory; i < n; ++i) {
        if (!(errors[i] < tolerance)) all_err = 0;
        if (ngp[i] != 0) all_gp = 0;
        if (ranks[i] < minr) minr = ranks[i];
        if (!(ranks[i] >= maxbonddim)) all_max = 0;
    }
    /* all() over an empty history is true (ncheckhistory == 0) */
    i64 lastr = ncheckhistory > 0 ? ranks[n - 1] : minr;
    return (all_err && (checkconvglobalpivot ? all_gp : 1) && (ncheckhistory == 0 || minr == lastr)) || all_max;
}

static i64 tci_rank(const orc_tci* t) {
    i64 r = 0;
    for (int p = 0; p < t->L - 1; ++p) if (t->I[p + 1].n > r) r = t->I[p + 1].n;
    return r;
}
static double tci_maxbonderror(const orc_tci* t) {
    double m = t->bonderr[0];
    for (int p = 1; p < t->L - 1; ++p) m = jl_max(m, t->bonderr[p]);
    return m;
}

/* optimize! (tensorci2.jl:1018-1172), deterministic mode: the global pivot finder returns no
 * pivots (nsearchglobalpivot = 0, accepted by the guard at :1048). Returns the number of outer
 * iterations in *niter; ranks/errors must hold maxiter entries; errors are normalised like :1171. */
int orc_tci_optimize(orc_tci* t, double tolerance, i64 maxbonddim, int maxiter, int sweepstrategy,
                     int normalizeerror, int ncheckhistory, int strictlynested,
                     int checkconvglobalpivot, i64* ranks, double* errors, int* niter) {
    double tol = tolerance;
    if (maxbonddim >= INT64_MAX && tol <= 0)
        return fail(ORC_ERR_CONV, "Specify either tolerance > 0 or some maxbonddim; otherwise, the "
                                  "convergence criterion is not reachable!");
    i64* ngp = (i64*)calloc((size_t)(maxiter + 1), sizeof(i64));
    int it = 0;
    for (int iter = 1; iter <= maxiter; ++iter) {
        double errnorm = normalizeerror ? t->maxsample : 1.0;
        double abstol = tol * errnorm;
        int st = orc_tci_sweep2site(t, 2, 1, abstol, maxbonddim, sweepstrategy, strictlynested, 1);
        if (st) { free(ngp); return st; }
        errors[it] = tci_maxbonderror(t);
        ngp[it] = 0; /* finder(...) -> MultiIndex[] */
        ranks[it] = tci_rank(t);
        it += 1;
        if (orc_convergencecriterion(ranks, errors, ngp, it, abstol, maxbonddim, ncheckhistory,
                                     checkconvglobalpivot))
            break;
    }
    free(ngp);
    double errnorm = normalizeerror ? t->maxsample : 1.0;
    double abstol = tol * errnorm;
    int st = orc_tci_sweep1site(t, 1, 1e-14, abstol, maxbonddim, 1);
    if (st) return st;
    for (int p = 0; p < t->L - 1; ++p)
        if (t->I[p + 1].n != t->J[p].n) {
            char msg[128];
            snprintf(msg, sizeof msg, "Pivot matrix at bond %d is not square!", p + 1);
            return fail(ORC_ERR_NONSQ, msg);
        }
    for (int i = 0; i < it; ++i) errors[i] = errors[i] / errnorm;
    *niter = it;
    return ORC_OK;
}

/* ------------------------------------------------------------ checkpoints
 * The state a warm restart needs (SURVEY 5 "Checkpoint / resume": the reference resumes from
 * Iset/Jset, tensorci2.jl:123-137), plus what the next sweep2site! reads: the last history entry
 * (extra sets, :1212-1217), pivoterrors, bonderrors and maxsamplevalue. Site tensors are not
 * saved (every sweep recomputes them). Used to split long oracle runs (config 5 as stated). */
static int wr_iset(FILE* fp, const iset_t* s) {
    i64 h[2] = {s->n, s->w};
    if (fwrite(h, sizeof h, 1, fp) != 1) return 1;
    if (s->n * s->w > 0 && fwrite(s->d, sizeof(i32), (size_t)(s->n * s->w), fp) != (size_t)(s->n * s->w)) return 1;
    return 0;
}
static int rd_iset(FILE* fp, iset_t* s) {
    i64 h[2];
    if (fread(h, sizeof h, 1, fp) != 1 || h[1] != s->w) return 1;
    iset_free(s);
    iset_init(s, (int)h[1]);
    s->n = s->cap = h[0];
    s->d = (i32*)malloc(sizeof(i32) * (size_t)(h[0] * h[1] + 1));
    if (h[0] * h[1] > 0 && fread(s->d, sizeof(i32), (size_t)(h[0] * h[1]), fp) != (size_t)(h[0] * h[1])) return 1;
    return 0;
}

int orc_tci_save(const orc_tci* t, const char* path) {
    FILE* fp = fopen(path, "wb");
    if (!fp) return fail(ORC_ERR_ARG, "cannot open checkpoint for writing");
    int bad = 0;
    i64 hdr[4] = {0x54434932, t->L, t->has_hist, t->npe};
    bad |= fwrite(hdr, sizeof hdr, 1, fp) != 1;
    bad |= fwrite(&t->maxsample, sizeof(double), 1, fp) != 1;
    if (t->npe) bad |= fwrite(t->pe, sizeof(double), (size_t)t->npe, fp) != (size_t)t->npe;
    bad |= fwrite(t->bonderr, sizeof(double), (size_t)(t->L - 1), fp) != (size_t)(t->L - 1);
    for (int p = 0; p < t->L && !bad; ++p)
        bad |= wr_iset(fp, &t->I[p]) | wr_iset(fp, &t->J[p]) | wr_iset(fp, &t->hI[p]) | wr_iset(fp, &t->hJ[p]);
    bad |= fclose(fp) != 0;
    return bad ? fail(ORC_ERR_ARG, "checkpoint write failed") : ORC_OK;
}

/* t must come from orc_tci_new with the same integrand and localdims */
int orc_tci_load(orc_tci* t, const char* path) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return fail(ORC_ERR_ARG, "cannot open checkpoint");
    int bad = 0;
    i64 hdr[4];
    bad |= fread(hdr, sizeof hdr, 1, fp) != 1;
    if (!bad && (hdr[0] != 0x54434932 || hdr[1] != t->L)) bad = 1;
    if (!bad) {
        t->has_hist = (int)hdr[2];
        free(t->pe);
        t->npe = hdr[3];
        t->pe = (double*)malloc(sizeof(double) * (size_t)(t->npe + 1));
        bad |= fread(&t->maxsample, sizeof(double), 1, fp) != 1;
        if (t->npe) bad |= fread(t->pe, sizeof(double), (size_t)t->npe, fp) != (size_t)t->npe;
        bad |= fread(t->bonderr, sizeof(double), (size_t)(t->L - 1), fp) != (size_t)(t->L - 1);
        for (int p = 0; p < t->L && !bad; ++p)
            bad |= rd_iset(fp, &t->I[p]) | rd_iset(fp, &t->J[p]) | rd_iset(fp, &t->hI[p]) | rd_iset(fp, &t->hJ[p]);
    }
    fclose(fp);
    tci_invalidate(t);
    return bad ? fail(ORC_ERR_ARG, "checkpoint read failed") : ORC_OK;
}

/* -------------------------------------------------------------- accessors */
int orc_tci_L(const orc_tci* t) { return t->L; }
double orc_tci_maxsample(const orc_tci* t) { return t->maxsample; }
i64 orc_tci_iset_size(const orc_tci* t, int p) { return t->I[p].n; }
i64 orc_tci_jset_size(const orc_tci* t, int p) { return t->J[p].n; }
void orc_tci_iset_get(const orc_tci* t, int p, i32* out) {
    if (t->I[p].w) memcpy(out, t->I[p].d, sizeof(i32) * (size_t)(t->I[p].n * t->I[p].w));
}
void orc_tci_jset_get(const orc_tci* t, int p, i32* out) {
    if (t->J[p].w) memcpy(out, t->J[p].d, sizeof(i32) * (size_t)(t->J[p].n * t->J[p].w));
}
i64 orc_tci_pivoterrors(const orc_tci* t, double* out, i64 cap) {
    for (i64 i = 0; i < t->npe && i < cap; ++i) out[i] = t->pe[i];
    return t->npe;
}
void orc_tci_bonderrors(const orc_tci* t, double* out) {
    memcpy(out, t->bonderr, sizeof(double) * (size_t)(t->L - 1));
}
i64 orc_tci_sitetensor_size(const orc_tci* t, int p) { return t->Tn[p]; }
void orc_tci_sitetensor(const orc_tci* t, int p, double* out) {
    memcpy(out, t->T[p], sizeof(double) * (size_t)t->Tn[p]);
}
/* evaluate(tci, idx): product of T[:, i, :] over sites (abstracttensortrain.jl:328-342) */
int orc_tci_evaluate(const orc_tci* t, const i32* idx, double* out) {
    int L = t->L;
    for (int p = 0; p < L; ++p)
        if (!t->T[p]) return fail(ORC_ERR_ARG, "site tensors are not available");
    i64 ra = t->I[0].n; /* == 1 */
    double* v = (double*)malloc(sizeof(double) * 8);
    v[0] = 1.0;
    (void)ra;
    i64 cur = 1;
    for (int p = 0; p < L; ++p) {
        i64 a = t->I[p].n, d = t->localdims[p];
        i64 b = (p == L - 1) ? 1 : t->I[p + 1].n;
        double* w = (double*)malloc(sizeof(double) * (size_t)(b + 1));
        const double* T = t->T[p];
        for (i64 j = 0; j < b; ++j) {
            double s = 0.0;
            for (i64 i = 0; i < a; ++i) s = s + v[i] * T[i + a * (idx[p] - 1) + a * d * j];
            w[j] = s;
        }
        free(v);
        v = w;
        cur = b;
    }
    (void)cur;
    *out = v[0];
    free(v);
    return ORC_OK;
}

/* ============================================================ ComplexF64 rrLU
 * rrlu(A::Matrix{ComplexF64}) -- the same _optimizerrlu! / addpivot! loop (matrixlu.jl:295-322,
 * 346-396) on complex entries, stored interleaved (re, im) column-major like Julia's
 * ComplexF64 arrays. Julia Base arithmetic the loop relies on (base/complex.jl, not under
 * /root/reference; restated from its published algorithm, parity at the last-ulp level of the
 * division and of abs unpinned):
 *   abs2(z) = re*re + im*im;  z*w = (ac - bd, ad + bc) without fma;  a - b componentwise;
 *   z / w   = Baudin & Smith robust division (the ComplexF64 method of `/`);
 *   abs(z)  = hypot(re, im) (correctly rounded fma branch of Base.Math._hypot). */

static void jl_cdiv2(double a, double b, double c, double d, double r, double t, double* out) {
    if (r != 0) {
        double br = b * r;
        *out = (br != 0) ? (a + br) * t : a * t + (b * t) * r;
    } else {
        *out = (a + d * (b / c)) * t;
    }
}

static void jl_cdiv1(double a, double b, double c, double d, double* p, double* q) {
    double r = d / c;
    double t = 1.0 / (c + d * r);
    jl_cdiv2(a, b, c, d, r, t, p);
    jl_cdiv2(b, -a, c, d, r, t, q);
}

void orc_cdiv(double a, double b, double c, double d, double* re, double* im) {
    double absa = fabs(a), absb = fabs(b), ab = absa >= absb ? absa : absb;
    double absc = fabs(c), absd = fabs(d), cd = absc >= absd ? absc : absd;
    const double halfov = 0.5 * 1.7976931348623157e308;
    const double twounE = 2.2250738585072014e-308 * 2.0 / 2.220446049250313e-16;
    const double bs = 2.0 / (2.220446049250313e-16 * 2.220446049250313e-16);
    double s = 1.0, p, q;
    if (ab >= halfov) { a *= 0.5; b *= 0.5; s *= 2.0; }
    if (cd >= halfov) { c *= 0.5; d *= 0.5; s *= 0.5; }
    if (ab <= twounE) { a *= bs; b *= bs; s /= bs; }
    if (cd <= twounE) { c *= bs; d *= bs; s *= bs; }
    if (absd <= absc) {
        jl_cdiv1(a, b, c, d, &p, &q);
    } else {
        jl_cdiv1(b, a, d, c, &p, &q);
        q = -q;
    }
    *re = p * s;
    *im = q * s;
}

double orc_hypot(double x, double y) {
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
    double hsq = h * h, axsq = ax * ax;
    h -= (fma(-ay, ay, hsq - axsq) + fma(h, h, -hsq) - fma(ax, ax, -axsq)) / (2 * h);
    return h * scale;
}

/* _optimizerrlu! on ComplexF64 (matrixlu.jl:346-396); A interleaved m x n (ld m), copied.
 * rowperm/colperm 0-based; L m x np, U np x n (interleaved, written for the np found; capacity
 * maxrank); pivoterrs np + 1 values [abs.(diag(lu)); lu.error] (matrixlu.jl:799). */
int orc_rrlu_c128(const double* A0, i64 m, i64 n, i64 maxrank, double reltol, double abstol,
                  int leftorth, i64* rowperm, i64* colperm, double* L, double* U, i64* npivot,
                  double* lasterr, double* pivoterrs) {
    double* A = (double*)malloc(sizeof(double) * (size_t)(2 * m * n + 2));
    if (!A) return fail(ORC_ERR_ALLOC, "allocation failed");
    memcpy(A, A0, sizeof(double) * (size_t)(2 * m * n));
#define RE(i, j) A[2 * ((i) + (j) * m)]
#define IM(i, j) A[2 * ((i) + (j) * m) + 1]
    for (i64 i = 0; i < m; ++i) rowperm[i] = i;
    for (i64 j = 0; j < n; ++j) colperm[j] = j;
    i64 mr = maxrank < m ? maxrank : m;
    if (mr > n) mr = n;
    double maxerror = 0.0, error = NAN;
    i64 np = 0;
    while (np < mr) {
        i64 k = np, p = k, q = k;
        double best = -INFINITY;  /* submatrixargmax(abs2, A, k) (matrixlu.jl:46-87, 133-135) */
        for (i64 c = k; c < n; ++c)
            for (i64 r = k; r < m; ++r) {
                double v = RE(r, c) * RE(r, c) + IM(r, c) * IM(r, c);
                if (v > best) { best = v; p = r; q = c; }
            }
        error = orc_hypot(RE(p, q), IM(p, q));
        if ((error < reltol * maxerror || error < abstol) && np > 0) break;
        maxerror = jl_max(maxerror, error);
        /* addpivot!: swaprow!, swapcol!, normalise, rank-1 update (matrixlu.jl:295-322) */
        i64 t;
        t = rowperm[k]; rowperm[k] = rowperm[p]; rowperm[p] = t;
        for (i64 j = 0; j < n; ++j) {
            double a = RE(k, j), b = IM(k, j);
            RE(k, j) = RE(p, j); IM(k, j) = IM(p, j);
            RE(p, j) = a; IM(p, j) = b;
        }
        t = colperm[k]; colperm[k] = colperm[q]; colperm[q] = t;
        for (i64 i = 0; i < m; ++i) {
            double a = RE(i, k), b = IM(i, k);
            RE(i, k) = RE(i, q); IM(i, k) = IM(i, q);
            RE(i, q) = a; IM(i, q) = b;
        }
        const double pr = RE(k, k), pi = IM(k, k);
        if (leftorth) {
            for (i64 i = k + 1; i < m; ++i) orc_cdiv(RE(i, k), IM(i, k), pr, pi, &RE(i, k), &IM(i, k));
        } else {
            for (i64 j = k + 1; j < n; ++j) orc_cdiv(RE(k, j), IM(k, j), pr, pi, &RE(k, j), &IM(k, j));
        }
        for (i64 j = k + 1; j < n; ++j) {
            const double yr = RE(k, j), yi = IM(k, j);
            for (i64 i = k + 1; i < m; ++i) {
                const double xr = RE(i, k), xi = IM(i, k);
                const double zr = xr * yr - xi * yi, zi = xr * yi + xi * yr;
                RE(i, j) = RE(i, j) - zr;
                IM(i, j) = IM(i, j) - zi;
            }
        }
        np += 1;
    }
    if (np >= (m < n ? m : n)) error = 0.0;
    /* L = tril(A[:, 1:np]), U = triu(A[1:np, :]), NaN checks, unit diagonal (matrixlu.jl:372-388) */
    int nan = 0;
    for (i64 c = 0; c < np; ++c)
        for (i64 r = 0; r < m; ++r) {
            double a = r >= c ? RE(r, c) : 0.0, b = r >= c ? IM(r, c) : 0.0;
            nan |= isnan(a) || isnan(b);
            if (L) { L[2 * (r + c * m)] = a; L[2 * (r + c * m) + 1] = b; }
        }
    if (nan) { free(A); return fail(ORC_ERR_NAN, "lu.L contains NaNs"); }
    for (i64 c = 0; c < n; ++c)
        for (i64 r = 0; r < np; ++r) {
            double a = r <= c ? RE(r, c) : 0.0, b = r <= c ? IM(r, c) : 0.0;
            nan |= isnan(a) || isnan(b);
            if (U) { U[2 * (r + c * np)] = a; U[2 * (r + c * np) + 1] = b; }
        }
    if (nan) { free(A); return fail(ORC_ERR_NAN, "lu.U contains NaNs"); }
    for (i64 c = 0; c < np; ++c) {
        if (pivoterrs) pivoterrs[c] = orc_hypot(RE(c, c), IM(c, c));
        double* D = leftorth ? L : U;
        i64 off = leftorth ? 2 * (c + c * m) : 2 * (c + c * np);
        if (D) { D[off] = 1.0; D[off + 1] = 0.0; }
    }
    if (pivoterrs) pivoterrs[np] = error;
#undef RE
#undef IM
    *npivot = np;
    *lasterr = error;
    free(A);
    return ORC_OK;
}

/* MatrixLUCI{ComplexF64} left/right factors (matrixluci.jl:161-283) from orc_rrlu_c128's L / U,
 * the same loops as luci_left / luci_right above on complex entries (multiply without fma,
 * sequential sums, orc_cdiv for the divisions). left m x np, right np x n, interleaved;
 * rowidx / colidx: the np pivot rows / columns (0-based). */
int orc_luci_c128(const double* A, i64 m, i64 n, i64 maxrank, double reltol, double abstol,
                  int leftorth, i64* rowidx, i64* colidx, double* pivoterrs, double* left,
                  double* right, i64* npivot) {
    i64 mr = maxrank < m ? maxrank : m;
    if (mr > n) mr = n;
    if (mr < 0) mr = 0;
    i64* rp = (i64*)malloc(sizeof(i64) * (size_t)(m + 1));
    i64* cp = (i64*)malloc(sizeof(i64) * (size_t)(n + 1));
    double* L = (double*)malloc(sizeof(double) * (size_t)(2 * m * mr + 2));
    double* U = (double*)malloc(sizeof(double) * (size_t)(2 * mr * n + 2));
    if (!rp || !cp || !L || !U) {
        free(rp); free(cp); free(L); free(U);
        return fail(ORC_ERR_ALLOC, "allocation failed");
    }
    i64 np;
    double err;
    int st = orc_rrlu_c128(A, m, n, maxrank, reltol, abstol, leftorth, rp, cp, L, U, &np, &err,
                           pivoterrs);
    if (st) { free(rp); free(cp); free(L); free(U); return st; }
    *npivot = np;
    for (i64 k = 0; k < np; ++k) { rowidx[k] = rp[k]; colidx[k] = cp[k]; }
#define LR(i, j) L[2 * ((i) + (j) * m)]
#define LI(i, j) L[2 * ((i) + (j) * m) + 1]
#define UR(i, j) U[2 * ((i) + (j) * np)]
#define UI(i, j) U[2 * ((i) + (j) * np) + 1]
    if (left) {
        for (i64 i = 0; i < m; ++i) {
            double* o = left + 2 * rp[i];
            for (i64 j = np - 1; j >= 0; --j) {
                double sr = 0.0, si = 0.0;
                if (leftorth) {  /* [I; L21 / LowerTriangular(L11)] */
                    if (i < np) { sr = (i == j); si = 0.0; }
                    else {
                        sr = LR(i, j); si = LI(i, j);
                        for (i64 t = j + 1; t < np; ++t) {
                            const double xr = o[2 * (t * m)], xi = o[2 * (t * m) + 1];
                            sr = sr - (xr * LR(t, j) - xi * LI(t, j));
                            si = si - (xr * LI(t, j) + xi * LR(t, j));
                        }
                        orc_cdiv(sr, si, LR(j, j), LI(j, j), &sr, &si);
                    }
                } else {  /* colmatrix: L * U11 */
                    for (i64 t = 0; t < np; ++t) {
                        sr = sr + (LR(i, t) * UR(t, j) - LI(i, t) * UI(t, j));
                        si = si + (LR(i, t) * UI(t, j) + LI(i, t) * UR(t, j));
                    }
                }
                o[2 * (j * m)] = sr;
                o[2 * (j * m) + 1] = si;
            }
        }
    }
    if (right) {
        for (i64 c = 0; c < n; ++c) {
            double* o = right + 2 * np * cp[c];
            for (i64 a = np - 1; a >= 0; --a) {
                double sr = 0.0, si = 0.0;
                if (!leftorth) {  /* [I, UpperTriangular(U11) \ U12] */
                    if (c < np) { sr = (a == c); si = 0.0; }
                    else {
                        sr = UR(a, c); si = UI(a, c);
                        for (i64 t = a + 1; t < np; ++t) {
                            const double xr = o[2 * t], xi = o[2 * t + 1];
                            sr = sr - (UR(a, t) * xr - UI(a, t) * xi);
                            si = si - (UR(a, t) * xi + UI(a, t) * xr);
                        }
                        orc_cdiv(sr, si, UR(a, a), UI(a, a), &sr, &si);
                    }
                } else {  /* rowmatrix: L11 * U */
                    for (i64 t = 0; t < np; ++t) {
                        sr = sr + (LR(a, t) * UR(t, c) - LI(a, t) * UI(t, c));
                        si = si + (LR(a, t) * UI(t, c) + LI(a, t) * UR(t, c));
                    }
                }
                o[2 * a] = sr;
                o[2 * a + 1] = si;
            }
        }
    }
#undef LR
#undef LI
#undef UR
#undef UI
    free(rp); free(cp); free(L); free(U);
    return ORC_OK;
}
