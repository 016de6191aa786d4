/*
 * tci_hip.h -- C ABI of libtci_hip.so, the MI355X (gfx950) engine behind the TCI2 hot path of
 * TensorCrossInterpolation.jl (XiaoJiang-Phy fork of tensor4all v0.9.18).
 *
 * Plain pointers and sizes only; no torch/HIP types in any signature. A Julia shim binds these
 * with `ccall`; this repo's Python host (tci_amd) binds them with ctypes.
 *
 * Conventions
 *  - Matrices are column-major Float64, like Julia Matrix{Float64}.
 *  - Index sets (MultiIndex = Vector{Int}, abstracttensortrain.jl:33) are passed as int32 tables
 *    in row-major "entry" order: entry e occupies w consecutive values; values are 1-based.
 *  - Permutations and pivot row/column indices are returned 1-based (Julia convention).
 *  - `_h` entry points take host pointers (the library copies in and out, synchronous);
 *    `_d` entry points take device pointers on the context's device and leave results there.
 *  - Every call is synchronous with respect to the host for host outputs (stream synchronised
 *    before return). One tci_ctx per host thread; contexts are independent.
 *
 * Errors: 0 = success; otherwise one of TCI_ERR_*; tci_last_error(ctx) gives the message, which
 * matches the reference's exception text where one exists.
 */
#ifndef TCI_HIP_H
#define TCI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCI_OK 0
#define TCI_ERR_ARG 1    /* ArgumentError / DimensionMismatch (e.g. matrixlu.jl:58-67)         */
#define TCI_ERR_NAN 2    /* error("lu.L contains NaNs") / ("lu.U ...") (matrixlu.jl:376-381)    */
#define TCI_ERR_NONSQ 3  /* "Pivot matrix at bond $b is not square!" (tensorci2.jl:623)       */
#define TCI_ERR_DEVICE 4 /* HIP / RCCL failure                                                 */
#define TCI_ERR_NOMEM 5  /* device allocation failed                                           */
#define TCI_ERR_HOST 6   /* a host callback (tci_func_create_host) reported failure            */

/* Integrand catalog (DESIGN.md "Integrand catalog"); the reference's `f` is user Julia code,
 * a device kernel needs it as data. */
#define TCI_F_SUM 0      /* f(x) = sum(x)                               (test_batcheval.jl:19) */
#define TCI_F_LORENTZ 1  /* f(x) = p0 / (sum(x.^2) + 1)                 (README.md:21-29)      */
#define TCI_F_TABLE 2    /* f(x) = p[x] over a dense column-major tensor                       */
#define TCI_F_GAUSS 3    /* f(x) = exp(-(p0 * sum((x .- p1).^2)))        (BASELINE config 3)    */
#define TCI_F_GAUSSMIX 4 /* f(x) = sum_k w_k exp(-(a * sum((x .- c_k).^2)))                   */
#define TCI_F_QOSC 5     /* quantics x: exp(-p0 x) sin(p1 x^p2)         (test_tensorci2.jl:437) */
#define TCI_F_QEXP 6     /* quantics x: p0 exp(-p1 x) + p2 exp(-p3 x)   (test_tensorci2.jl:65)  */
#define TCI_F_TT 7       /* tensor-train evaluation (test_tensorci2.jl:477-502, TTCache as f)   */
#define TCI_F_CP 8       /* f(x) = sum_k prod_t g[k][t][x_t]: CP-rank-K synthetic */
#define TCI_F_MPO 9      /* Contraction(A, B) of two 4-leg tensor trains (contraction.jl:60-575)  */
#define TCI_F_HOST 10    /* the user's own f / BatchEvaluator, evaluated on the host by a callback
                            (tci_func_create_host; batcheval.jl:131-214, 247-308)               */
#define TCI_F_C128 11    /* a ComplexF64 integrand as sums of real ones, Re f = sum of parts, Im f
                            = sum of parts (tci_func_create_c128; Contraction{ComplexF64},
                            contraction.jl:60-152)                                              */
/* GAUSSMIX, CP and MPO are sums of K separable terms: Pi is assembled as a rank-K fp64 MFMA GEMM
 * (MPO: K = ra*rb at the cut, the factor rows are the left / right environments).
 * MPO params: [N, per site t (ra, d1, d2, ra', rb, d3, rb', offA, offB), cores]: A_t is
 * (ra, d1, d2, ra'), B_t is (rb, d2, d3, rb'), column-major at offA / offB past the 1 + 9N header;
 * localdims[t] = d1 * d3 (fused index s1 + d1 (s3 - 1), contraction.jl:226-237); boundary bonds 1;
 * every bond ra * rb <= 2048, every site rb*d2*ra' and ra*d2*rb' <= 8192 (TCI_ERR_ARG otherwise).
 * params: GAUSSMIX [K, a, centres (K x L, row-major), weights (K)];
 *         CP       [K, dmax, g (K x L x dmax, dmax fastest)] with dmax >= max(localdims). */

typedef struct tci_ctx tci_ctx;
typedef struct tci_func tci_func;
typedef struct tci_comm tci_comm;
typedef struct tci_cache tci_cache;
typedef struct tci_tci2 tci_tci2;
/* Host-side exchange hook of the column-sharded rrLU, for when no RCCL communicator is passed
 * (ranks sharing one GPU, or a Julia Distributed / MPI transport); called with the context stream
 * synchronised, d_send / d_recv device pointers of the calling context, `count` 8-byte words:
 *   op 0: all-gather -- d_recv[r * count + i] = rank r's d_send[i];
 *   op 1: element-wise max over the ranks of d_send[i] as uint64 into d_recv[i].
 * Returns 0 on success. A failure must be collective (every rank returns nonzero for the same
 * call), or the other ranks would wait in the next exchange. */
typedef int (*tci_exchange_fn)(void* user, int op, const void* d_send, void* d_recv, int64_t count);

/* ---------------------------------------------------------------- context */
int tci_ctx_create(int device, tci_ctx** out);
int tci_ctx_destroy(tci_ctx* ctx);
const char* tci_last_error(const tci_ctx* ctx);
/* Device stream the context launches on (a hipStream_t as an opaque pointer), e.g. for
 * hipEvent timing around _d calls. */
void* tci_ctx_stream(tci_ctx* ctx);
int tci_ctx_synchronize(tci_ctx* ctx);
/* Device time (ms, summed) and launch count of a kernel family since tci_set_timing(ctx, 1),
 * measured with hipEvents on the context stream: family 0 = rrLU pass that writes the Schur
 * update back, 2 = rrLU read-only pass (pending updates applied on the fly + argmax),
 * 1 = batch evaluation; 3 + P (P = 1..16) = the read-only passes that applied P pending updates
 * in the first shadow epoch after a write-back, 24 + P the same in the later shadow epochs of
 * the exact epoch (a breakdown of family 2); 20 = site-tensor solve (getrf + getrs of P^T),
 * 21 = MatrixLUCI factors, 22 = K3 GEMMs issued through tci_dgemm_d / tci_schur_update_d, 23 =
 * rrLU refresh passes (read-only passes that also rewrite the fp16 shadow, two-level epoch). */
int tci_last_kernel_stats(tci_ctx* ctx, int family, double* total_ms, int64_t* launches);
/* The same with the passes the timed launches covered (units): 41 / 42 = persistent launches of a
 * shadow epoch's read-only passes (first shadow epoch / later ones; tci_set_rrlu_persist), whose
 * units are passes, 43 = pass 0 (the exact pass after pivot 0 that writes the shadow of A; not in
 * family 2). Every other launch counts one unit. */
int tci_last_kernel_units(tci_ctx* ctx, int family, double* total_ms, int64_t* launches, int64_t* units);
/* enabled = 0: off; s >= 1: on, timing the rrLU pass of every s-th pivot (k % s == 0) and every
 * batch evaluation. Resets the statistics. */
int tci_set_timing(tci_ctx* ctx, int enabled);
/* Deferred-update depth of the rrLU (1..16; default 10, env TCI_RRLU_NB): up to nb rank-1
 * updates are applied on the fly by read-only passes, after which the shadow of the values is
 * rewritten -- by the search itself (a refresh) or, every `epochs`-th time, by a write-back of the
 * fp64 values. Results are bitwise identical for every nb and epochs. */
int tci_set_rrlu_flush(tci_ctx* ctx, int nb);
/* Shadow epochs per fp64 write-back (two-level epoch; 1..32 with nb * epochs <= 32;
 * 1 = write back every nb pivots; 0, the default, = by shape: 3 on trailing blocks of >= 2.4e7
 * elements, else 1; env TCI_RRLU_EPOCHS). tci_rrlu_epochs_for: the value an m x n rrLU will use. */
int tci_set_rrlu_epochs(tci_ctx* ctx, int epochs);
int tci_rrlu_epochs_for(tci_ctx* ctx, int64_t m, int64_t n);
/* Matrices with m*n <= 16384 and m + n <= 4096 are factorised by one workgroup holding the whole
 * matrix in LDS (one launch instead of one per pivot); enabled = 0 forces the pass pipeline.
 * Both paths give bitwise identical results. Default on (env TCI_RRLU_SMALL=0: off). */
int tci_set_rrlu_small(tci_ctx* ctx, int enabled);
/* Matrices with m*n <= 2^21 whose column blocks fit the LDS of one workgroup per CU are factorised
 * by a persistent grid holding the matrix on chip (one grid barrier per pivot);
 * enabled = 0 forces the pass pipeline. Bitwise identical results. Default on (env
 * TCI_RRLU_MID=0: off). */
int tci_set_rrlu_mid(tci_ctx* ctx, int enabled);
/* The read-only passes of a shadow epoch (the passes between two refreshes / write-backs of the
 * fp16 shadow; up to nb - 1 of them) run as ONE persistent launch whose resident grid hands each
 * pivot's commit to the next pass in place of a kernel boundary -- the same pass bodies, results
 * bitwise identical (replaces the per-pivot loop of _optimizerrlu!, matrixlu.jl:356-369). If the grid
 * is found not co-resident (another process holds CUs) the launch gives up after 0.5 s, the
 * factorisation resumes with per-pass launches and this context stops using the persistent form
 * (tci_rrlu_persist_faulted). Default OFF (measured slower than the per-pass launches, DESIGN.md K2;
 * env TCI_RRLU_PERSIST=1: on); enabled resets the flag.
 * enabled = 2 is a test mode: the persistent launch is used even where its grid exceeds one workgroup
 * per CU (TCI_PASS_GRIDX > 1), i.e. where it is NOT co-resident, and gives up after 2 ms, so that the
 * give-up-and-resume path runs. */
int tci_set_rrlu_persist(tci_ctx* ctx, int enabled);
/* 1 once a persistent launch of this context gave up (see tci_set_rrlu_persist), else 0. */
int tci_rrlu_persist_faulted(tci_ctx* ctx);
/* Per-pivot exchange of tci_rrlu_sharded_d (the candidate selection of _optimizerrlu!,
 * matrixlu.jl:356-369, across column shards): 1 = two collectives (all-gather of the 32-B
 * candidate records, then an element-wise max of the winning column as a broadcast), 2 = fused (ONE
 * all-gather of every rank's record together with its own candidate column), 0 = by size (fused
 * while (N - 1) x 8 (m + 36) B <= 4 MiB; the default; env TCI_SHARD_EXCHANGE). Identical results in
 * every mode. */
int tci_set_shard_exchange(tci_ctx* ctx, int mode);
/* The exchange the last tci_rrlu_sharded_d ran: 0 none (one rank, no communicator), 1, 2 as above. */
int tci_last_shard_exchange(tci_ctx* ctx);
/* Certified shadow search in the read-only passes of the pass pipeline: the write-back passes also
 * keep a shadow of the stale values -- fp16 scaled per write-back epoch (2 B/element; fp32 in
 * the TCI_SH_HALF=0 build) -- and a read-only pass streams it instead of the fp64 values, applies
 * the pending updates on the matrix cores (f16-split MFMA, fp32 accumulation), bounds the error,
 * and re-reads in fp64 only the elements that can hold the argmax. Bitwise identical results (same
 * argmax, same tie order as submatrixargmax, matrixlu.jl:46-87). Default on (env
 * TCI_RRLU_SHADOW=0: off). */
int tci_set_rrlu_shadow(tci_ctx* ctx, int enabled);
/* Bytes per element of that shadow in this build (2: fp16, 4: fp32). */
int tci_rrlu_shadow_bytes(void);
/* ComplexF64 rrLU: the same certified shadow search (fp16 planes of the real and imaginary parts,
 * pending updates on f16-split MFMA, exact fp64 re-reads). Bitwise identical
 * results. Default on (env TCI_C128_SH=0: off). */
int tci_set_c128_shadow(tci_ctx* ctx, int enabled);

/* fp64 MFMA forms of the MatrixLUCI factors (bit 1), the site-tensor getrf
 * (bit 2) and getrs (bit 4), the getrf's panels held in registers (bit 8; without it the
 * panels are factorised in LDS -- bitwise the same factors) and the getrf as one cooperative
 * launch for r <= 1024 (bit 16, with bits 2 and 8; without it: four launches per panel); default
 * 31 (env TCI_DENSE_MFMA). 0 restores the round-1 scalar kernels
 * (A/B). Factors / solutions agree to the parity tolerances either way. */
int tci_set_dense_mfma(tci_ctx* ctx, int mask);

/* ------------------------------------------------------------ integrands */
/* Uploads an integrand's parameters to the device once; localdims has L entries. */
int tci_func_create(tci_ctx* ctx, int kind, const double* params, int64_t nparams,
                    const int32_t* localdims, int32_t L, tci_func** out);
int tci_func_destroy(tci_func* f);

/* The user's own function as an integrand (the route of an arbitrary Julia closure or
 * BatchEvaluator, batcheval.jl:131-214, onto the device rrLU): the library calls
 *   fn(user, I, m, nl, J, n, nr, M, out, ldo)
 * on the calling host thread whenever it needs a batch -- I (m x nl) and J (n x nr) row-major
 * 1-based host tables, out a column-major (m * D) x n host buffer (ld ldo) to fill with
 * f([I_i..., c..., J_j...]) at out[i + m*c + ldo*j], exactly the array of
 * _batchevaluate_dispatch / (f::BatchEvaluator)(Iset, Jset, Val(M)). A nonzero return aborts the
 * calling entry with TCI_ERR_HOST. The batch is uploaded once into HBM and everything after it
 * (maxabs, rrLU, MatrixLUCI factors, site-tensor solve, the device memo) runs on the device: any
 * entry taking a tci_func accepts it (tci_update_pivots_h, tci_sitetensor_h, tci_tci2_sweep2site,
 * tci_batcheval_*, tci_cache_batcheval_*). */
typedef int (*tci_host_fn)(void* user, const int32_t* I, int64_t m, int32_t nl, const int32_t* J,
                           int64_t n, int32_t nr, int32_t M, double* out, int64_t ldo);
int tci_func_create_host(tci_ctx* ctx, tci_host_fn fn, void* user, const int32_t* localdims,
                         int32_t L, tci_func** out);

/* A ComplexF64 integrand from real ones: f(x) = sum_{i<nre} re[i](x) + im * sum_{i<nim} im[i](x)
 * (the sums in part order). Used for Contraction{ComplexF64} (contraction.jl:60-152): with both
 * complex MPOs realified (each entry a 2x2 real block, bonds doubled; A_re, A_im the real MPOs of
 * Re A, Im A), Re(A B) = A_re B_re + A_im (-B_im) and Im(A B) = A_im B_re + A_re B_im: four real
 * TCI_F_MPO parts, each an fp64 MFMA GEMM. The parts must outlive f and share its localdims. Only the ComplexF64
 * entries accept it (tci_batcheval_c128_h, tci_update_pivots_c128_h; the real ones return
 * TCI_ERR_ARG). */
int tci_func_create_c128(tci_ctx* ctx, const tci_func* const* re, int32_t nre,
                         const tci_func* const* im, int32_t nim, tci_func** out);

/* Batch evaluation with DEVICE-RESIDENT index tables and no host synchronisation (the column-sharded
 * evaluation's per-rank block): I (m x nl) and J (n x nr) device int32 tables (row-major
 * entries, 1-based), Pi into d_out (device, ld ldo) as tci_batcheval_d; the batch's max |value| is
 * folded into *d_maxbits, a device uint64 holding the bits of a running maximum (atomic max of the
 * non-negative doubles' bit patterns: NaN is the largest, as Julia's max propagates it) that the caller
 * zeroes when a maximum starts -- updatemaxsample! (tensorci2.jl:636-638) over many batches, reduced
 * over the ranks once with tci_comm_allreduce_max_u64_d. Stream-ordered on the context stream; catalog
 * integrands only (not TCI_F_HOST, TCI_F_C128). Replaces _batchevaluate_dispatch
 * (batcheval.jl:131-175) for a BatchEvaluator whose sets already live on the device. */
int tci_batcheval_dd(tci_ctx* ctx, const tci_func* f, const int32_t* d_I, int64_t m, int32_t nl, const int32_t* d_J,
                     int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo, uint64_t* d_maxbits);
/* As tci_batcheval_dd with HOST index tables: they are copied (pinned stage owned by this entry,
 * asynchronous upload) and the call returns without synchronising -- the column-sharded 2-site
 * update (ShardedBatchEvaluator) evaluates its block, runs tci_rrlu_sharded_d (which synchronises
 * at its end anyway) and only then reads *d_maxbits: one host synchronisation per bond instead of
 * two. I / J may be reused by the caller as soon as the call returns. */
int tci_batcheval_da(tci_ctx* ctx, const tci_func* f, const int32_t* I, int64_t m, int32_t nl, const int32_t* J,
                     int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo, uint64_t* d_maxbits);
/* ----------------------------------------------------------- batch eval
 * Replaces _batchevaluate_dispatch (batcheval.jl:131-175) plus maxabs (util.jl:34-43) as used by
 * updatemaxsample! (tensorci2.jl:636-638).
 * out[i + m*c + m*D*j] = f([I_i..., c..., J_j...]) for M = 0 or 1 centre legs (D = localdims[nl]
 * when M = 1). I: m x nl, J: n x nr (row-major entries, 1-based). *maxabs = max(|out|) with
 * Julia's NaN-propagating max. ldo = leading dimension of out (>= m*D). */
int tci_batcheval_h(tci_ctx* ctx, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                    const int32_t* J, int64_t n, int32_t nr, int32_t M, double* out, int64_t ldo,
                    double* maxabs);
int tci_batcheval_d(tci_ctx* ctx, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                    const int32_t* J, int64_t n, int32_t nr, int32_t M, double* d_out,
                    int64_t ldo, double* maxabs);

/* ------------------------------------------------------------------ rrLU
 * Replaces rrlu / rrlu! / _optimizerrlu! (matrixlu.jl:346-463) with identical arithmetic: full
 * pivoting by abs2 argmax (ties -> smallest column, then row; matrixlu.jl:46-87), the row and
 * column swaps of addpivot! (kept as position maps: the matrix itself never moves),
 * true-division normalisation and separate multiply/subtract rank-1 updates (deferred up to nb
 * pivots, applied on the fly in the reference's order: bitwise the same values).
 * Outputs mirror the rrLU struct (matrixlu.jl:200-207):
 *   rowperm[m], colperm[n]  (1-based),  L: m x maxrank (ld m), U: maxrank x n (ld ldu >= maxrank),
 *   only the first *npivot columns of L / rows of U are meaningful; *lasterror = lu.error.
 * Pass NULL for L/U to skip them. */
int tci_rrlu_h(tci_ctx* ctx, const double* A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
               double reltol, double abstol, int leftorth, int64_t* rowperm, int64_t* colperm,
               double* L, double* U, int64_t ldu, int64_t* npivot, double* lasterror);
/* rrlu! on a device matrix: factorises d_A (column-major, ld lda; lda even) using it as the work
 * matrix -- its contents are clobbered (stale trailing values), as the reference's A is after
 * _optimizerrlu! -- and returns to the host the permutations (NULL to skip), npivot, lu.error and
 * the np + 1 pivot errors (matrixlu.jl:799; NULL to skip). L and U stay in the context. */
int tci_rrlu_inplace_d(tci_ctx* ctx, double* d_A, int64_t m, int64_t n, int64_t lda,
                       int64_t maxrank, double reltol, double abstol, int leftorth,
                       int64_t* rowperm, int64_t* colperm, int64_t* npivot, double* lasterror,
                       double* pivoterrors);
/* rrlu(A) on device memory (matrixlu.jl:455-463: `rrlu!(copy(A))`): d_src (m x n, ld ldsrc) is
 * left untouched and d_W (ld ldw, even; 16-byte aligned; must not overlap d_src) receives the copy
 * and is used as the work matrix, as tci_rrlu_inplace_d. The copy is fused into the initial argmax
 * pass (it reads the input once and writes the work matrix as it searches) where the pass pipeline
 * runs; the one-launch small / mid paths copy first. Same outputs and results as copying d_src into
 * d_W and calling tci_rrlu_inplace_d. */
int tci_rrlu_copy_d(tci_ctx* ctx, const double* d_src, int64_t ldsrc, double* d_W, int64_t m, int64_t n,
                    int64_t ldw, int64_t maxrank, double reltol, double abstol, int leftorth,
                    int64_t* rowperm, int64_t* colperm, int64_t* npivot, double* lasterror,
                    double* pivoterrors);

/* rrlu(A::Matrix{ComplexF64}) (matrixlu.jl:455-463; the _optimizerrlu! loop :346-396 on complex
 * entries). A, L, U are ComplexF64 stored interleaved (re, im) column-major
 * (Julia's layout): A is 2*lda*n doubles, L m x maxrank (ld m), U maxrank x n (ld ldu >= maxrank,
 * counted in complex entries). pivoterrors: np + 1 values [abs.(diag(lu)); lu.error]
 * (matrixlu.jl:799), NULL to skip. Same permutation / error conventions as tci_rrlu_h. */
int tci_rrlu_c128_h(tci_ctx* ctx, const double* A, int64_t m, int64_t n, int64_t lda,
                    int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowperm,
                    int64_t* colperm, double* L, double* U, int64_t ldu, int64_t* npivot,
                    double* lasterror, double* pivoterrors);

/* rrlu! of a ComplexF64 device matrix (interleaved, ld lda >= m, 16-byte aligned), clobbered as
 * the work matrix; permutations (NULL to skip), npivot, lu.error and the np + 1 pivot errors
 * (NULL to skip) to the host, with the NaN checks of matrixlu.jl:376-381. */
int tci_rrlu_c128_inplace_d(tci_ctx* ctx, double* d_A, int64_t m, int64_t n, int64_t lda,
                            int64_t maxrank, double reltol, double abstol, int leftorth,
                            int64_t* rowperm, int64_t* colperm, int64_t* npivot,
                            double* lasterror, double* pivoterrors);

/* ------------------------------------------------------------ MatrixLUCI
 * Replaces MatrixLUCI(A; kw...) + left/right/pivoterrors (matrixluci.jl:55-57, 161-311):
 * leftorth: left = colstimespivotinv (TRSM), right = rowmatrix (GEMM);
 * otherwise left = colmatrix (GEMM), right = pivotinvtimesrows (TRSM).
 * left: m x np (ld m), right: np x n (ld np), rowidx/colidx: np pivot indices (1-based),
 * pivoterrors: np + 1 values (matrixlu.jl:799). Capacities: maxrank. */
int tci_luci_h(tci_ctx* ctx, const double* A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
               double reltol, double abstol, int leftorth, int64_t* rowidx, int64_t* colidx,
               double* pivoterrors, double* left, double* right, int64_t* npivot);

/* MatrixLUCI on a device matrix (e.g. a Pi all-gathered over RCCL by the sharded evaluation):
 * d_A (ld lda, even; 16-B aligned) is clobbered as rrlu!'s work matrix; outputs as tci_luci_h, on
 * the host. */
int tci_luci_inplace_d(tci_ctx* ctx, double* d_A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
                       double reltol, double abstol, int leftorth, int64_t* rowidx, int64_t* colidx,
                       double* pivoterrors, double* left, double* right, int64_t* npivot);

/* MatrixLUCI{ComplexF64} (matrixluci.jl:55-57, 161-311) on top of the ComplexF64 rrLU:
 * left m x np, right np x n, interleaved (re, im) column-major; otherwise as tci_luci_h. */
int tci_luci_c128_h(tci_ctx* ctx, const double* A, int64_t m, int64_t n, int64_t lda,
                    int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowidx,
                    int64_t* colidx, double* pivoterrors, double* left, double* right,
                    int64_t* npivot);

/* --------------------------------------------------------- 2-site update
 * Replaces the :full branch of updatepivots! (tensorci2.jl:842-928) with Pi kept on the device:
 * Pi = f(rows x cols) -> maxabs -> rrLU -> pivot rows/cols -> (optionally) MatrixLUCI factors.
 * rows: m x nl, cols: n x nr (row-major entries, 1-based, already the union/kronecker sets).
 * Outputs: rowidx/colidx (np entries, 1-based positions into rows/cols, in pivot order),
 * pivoterrors (np+1), *maxabs, and if want_factors: left (m x np), right (np x n).
 * The same entry serves sweep1site! (tensorci2.jl:679-709) with rows = kronecker(Iset, d). */
int tci_update_pivots_h(tci_ctx* ctx, const tci_func* f, const int32_t* rows, int64_t m,
                        int32_t nl, const int32_t* cols, int64_t n, int32_t nr, int64_t maxrank,
                        double reltol, double abstol, int leftorth, int want_factors,
                        int64_t* rowidx, int64_t* colidx, double* pivoterrors, int64_t* npivot,
                        double* maxabs, double* left, double* right);

/* Batch evaluation of the ComplexF64 evaluator (cre + i cim) * f (see below): out is the
 * (m * D) x n complex result, interleaved, ld m * D (NULL: only max|.| is returned). */
int tci_batcheval_c128_h(tci_ctx* ctx, const tci_func* f, double cre, double cim,
                         const int32_t* I, int64_t m, int32_t nl, const int32_t* J, int64_t n,
                         int32_t nr, int32_t M, double* out, double* maxabs);

/* The 2-site update for a ComplexF64 evaluator f_c(x) = (cre + i cim) * f(x) over a real device
 * integrand f (the complex Lorentzian of test_tensorci2.jl:246-249 is coeff * TCI_F_LORENTZ):
 * Pi on the device, max|Pi| (abs = hypot), complex rrLU, pivots, and with want_factors the
 * MatrixLUCI{ComplexF64} factors (left m x np, right np x n, interleaved). Otherwise as
 * tci_update_pivots_h. */
int tci_update_pivots_c128_h(tci_ctx* ctx, const tci_func* f, double cre, double cim,
                             const int32_t* rows, int64_t m, int32_t nl, const int32_t* cols,
                             int64_t n, int32_t nr, int64_t maxrank, double reltol, double abstol,
                             int leftorth, int want_factors, int64_t* rowidx, int64_t* colidx,
                             double* pivoterrors, int64_t* npivot, double* maxabs, double* left,
                             double* right);

/* ------------------------------------------------------ native sweep driver
 * The per-bond loop of sweep2site! (tensorci2.jl:1195-1258) behind one call: kronecker products
 * (:512-529), Julia's first-seen union with the previous sweep's sets unless strictly nested
 * (:1214-1216), the 2-site update of every bond (tci_update_pivots_h, no factors: fillsitetensors!
 * rebuilds them), updatemaxsample! and updateerrors! (:636-638, :281-289). The TCI2 state
 * (Isets, Jsets, the last sweep's sets, maxsamplevalue, bond and pivot errors) lives in a
 * tci_tci2 the host fills and reads back. Sets: which = 0 Iset[p] (width p), 1 Jset[p] (width
 * L-1-p), 2 / 3 the history's; entries row-major, 1-based. sweepstrategy: 0 backandforth,
 * 1 forward, 2 backward. */
int tci_tci2_create(tci_ctx* ctx, int32_t L, const int32_t* localdims, tci_tci2** out);
int tci_tci2_destroy(tci_tci2* tci);
int tci_tci2_set_set(tci_tci2* tci, int which, int32_t p, const int32_t* entries, int64_t count);
int tci_tci2_get_set(tci_tci2* tci, int which, int32_t p, int32_t* entries, int64_t capacity,
                     int64_t* count);
int tci_tci2_clear_history(tci_tci2* tci);
int tci_tci2_set_errors(tci_tci2* tci, double maxsample, const double* bonderrors,
                        const double* pivoterrors, int64_t npivoterrors);
int tci_tci2_errors(tci_tci2* tci, double* maxsample, double* bonderrors, double* pivoterrors,
                    int64_t capacity, int64_t* npivoterrors);
int tci_tci2_sweep2site(tci_tci2* tci, const tci_func* f, int32_t niter, int32_t iter1,
                        double abstol, int64_t maxbonddim, int32_t sweepstrategy,
                        int32_t strictlynested);
/* tci_tci2_sweep2site followed by fillsitetensors!'s maxsample update (see tci_tci2_fill_maxsample)
 * in the same device launch when the device-resident path runs; *filled = 0: the caller runs
 * its own fill loop. */
int tci_tci2_sweep2site_fill(tci_tci2* tci, const tci_func* f, int32_t niter, int32_t iter1,
                             double abstol, int64_t maxbonddim, int32_t sweepstrategy,
                             int32_t strictlynested, int* filled);
/* All sites of one bank in one call: counts[p] entries of set p, the sets concatenated in site
 * order (a width-0 set contributes no ints). get: packed may be NULL (counts only); capacity in
 * ints. */
int tci_tci2_set_sets(tci_tci2* tci, int which, const int64_t* counts, const int32_t* packed);
int tci_tci2_get_sets(tci_tci2* tci, int which, int64_t* counts, int32_t* packed, int64_t capacity);
/* fillsitetensors! with the solve unobservable (globalsearch.jl:202-208; tensorci2.jl:599-611):
 * updatemaxsample!(tci, Pi1) over every site, on the device in one launch for the staged catalog
 * kinds. *handled = 0: not done here (other kinds, a non-square pivot matrix, a site too large);
 * the caller runs its own loop (tci_sitetensor_h / a batch maxabs per site). */
int tci_tci2_fill_maxsample(tci_tci2* tci, const tci_func* f, int* handled);
/* fillsitetensors! as the reference runs it (globalsearch.jl:202-208; setsitetensor!,
 * tensorci2.jl:599-629): per site Pi1, updatemaxsample!, P = f(Iset[p+1] x Jset[p]) and the solve
 * T = transpose(transpose(P) \ transpose(Pi1)) (LAPACK getrf / getrs of P^T, partial pivoting, the
 * oracle's operation order), the last site T = Pi1 -- all sites in one device launch for the staged
 * catalog kinds (pivot matrices up to 64 x 64). Site p's tensor at tensors[offsets[2p]],
 * offsets[2p+1] doubles, column-major (len(Iset[p]) d) x len(Jset[p]); capacity in doubles.
 * *handled = 0: not done here (as tci_tci2_fill_maxsample, or a pivot matrix over 64); the caller
 * runs tci_sitetensor_h per site. */
int tci_tci2_fill_solve(tci_tci2* tci, const tci_func* f, double* tensors, int64_t capacity, int64_t* offsets,
                        int* handled);
/* optimize!(tci, f; tolerance, maxbonddim, maxiter, ncheckhistory, normalizeerror, strictlynested,
 * nsearchglobalpivot = 0, sweepstrategy = :backandforth, pivotsearch = :full) (tensorci2.jl:1018-1172)
 * for a TCI2 whose bonds fit the device-resident small sweep: every iteration (sweep2site! with
 * fillsitetensors! -- solved when solvefill -- then pivoterror / rank / convergencecriterion) runs as
 * a chain of launches that keeps the state on the device, then sweep1site!(forward, abstol =
 * tolerance * maxsample) with its site tensors (tensors / capacity / offsets as tci_tci2_sweep1site).
 * errors[i] / ranks[i]: iteration i + 1's pivoterror / rank, *niter of them (maxiter < 64).
 * *handled = 0: nothing done; otherwise the state is the one after *niter iterations and, when
 * *ended and *s1done, after the closing sweep too (*errnorm: the maxsample it normalised with). A
 * bond, fill or sweep the device cannot run ends the chain early (*ended = 0: the caller continues
 * the loop; *ended = 1, *s1done = 0: the caller runs the closing sweep). */
int tci_tci2_optimize_small(tci_tci2* t, const tci_func* f, double tolerance, int64_t maxbonddim, int32_t maxiter,
                            int32_t ncheckhistory, int32_t normalizeerror, int32_t strictlynested, int32_t solvefill,
                            double* tensors, int64_t capacity, int64_t* offsets, double* errors, int64_t* ranks,
                            int32_t* niter, int32_t* ended, int32_t* s1done, double* errnorm, int* handled);
/* tci_tci2_sweep2site followed by tci_tci2_fill_solve's work in the same device launch when the
 * device-resident path runs; *filled = 0: the caller runs its own fill loop. */
int tci_tci2_sweep2site_fillsolve(tci_tci2* tci, const tci_func* f, int32_t niter, int32_t iter1,
                                  double abstol, int64_t maxbonddim, int32_t sweepstrategy,
                                  int32_t strictlynested, double* tensors, int64_t capacity,
                                  int64_t* offsets, int* filled);
/* Replaces sweep1site!(tci, f, sweepdirection; reltol, abstol, maxbonddim, updatetensors)
 * (tensorci2.jl:659-725) for the staged catalog kinds when every bond fits the one-workgroup
 * rrLU: the whole sweep in one device launch (per bond kronecker product on the sweep's side, Pi,
 * updatemaxsample!, rrLU, the new sets, updateerrors!, and with updatetensors the MatrixLUCI
 * left (forward) / right (backward) factor as the bond's site tensor, then Pi1 of the last site).
 * Tensors: site p's at tensors[offsets[2p]], offsets[2p+1] doubles, column-major
 * (len(Iset[p]) d) x len(Jset[p]) (forward) or len(Iset[p]) x (d len(Jset[p])) (backward bonds);
 * capacity in doubles. *handled = 0 leaves the state untouched: the caller runs the sweep itself
 * (other kinds, a bond too large, a NaN: the host loop raises the reference's error). */
int tci_tci2_sweep1site(tci_tci2* tci, const tci_func* f, int32_t forward, double reltol, double abstol,
                        int64_t maxbonddim, int32_t updatetensors, double* tensors, int64_t capacity,
                        int64_t* offsets, int* handled);
/* Device-resident sweeps (tci_sweep_small.hip): while every bond's Pi fits the one-workgroup rrLU,
 * tci_tci2_sweep2site runs whole iterations in one kernel launch for the staged catalog kinds
 * (SUM, LORENTZ, TABLE, GAUSS, QOSC, QEXP), bitwise the per-bond loop; on by default (env
 * TCI_SWEEP_SMALL=0 disables). */
int tci_set_sweep_small(tci_ctx* ctx, int enabled);

/* ---------------------------------------------------- site-tensor solve
 * Replaces setsitetensor!(tci, f, b) (tensorci2.jl:599-629): Pi1 = f(Iset_b x d x Jset_b),
 * P = f(Iset_{b+1} x Jset_b), T = Pi1 * P^-1 (partial-pivot LU of P^T, like getrf/getrs).
 * If Inext is NULL (last site) T = Pi1. T: (|I_b| d) x |J_b| column-major. */
int tci_sitetensor_h(tci_ctx* ctx, const tci_func* f, const int32_t* Ib, int64_t nIb, int32_t wI,
                     const int32_t* Jb, int64_t nJb, int32_t wJ, const int32_t* Inext,
                     int64_t nInext, double* T, double* maxabs);

/* The solve of setsitetensor! alone (tensorci2.jl:620-627) on host matrices: T = Pi1 * P^-1,
 * P: r x r, Pi1 and T: R x r, column-major (ld r / R). Used when Pi1 and P come from an
 * evaluator other than a tci_func (e.g. the multi-GPU sharded evaluation). */
int tci_sitetensor_solve_h(tci_ctx* ctx, const double* P, int64_t r, const double* Pi1, int64_t R,
                           double* T);

/* The same solve on device buffers (P r x r is clobbered by its LU; Pi1 and T R x r, ld R): no
 * PCIe. Blocked right-looking getrf of P^T (panels factorised in LDS, partial pivoting as getrf)
 * and a blocked getrs, the trailing / off-diagonal updates on fp64 MFMA (K3). */
int tci_sitetensor_solve_d(tci_ctx* ctx, double* d_P, int64_t r, const double* d_Pi1, int64_t R,
                           double* d_T);

/* ------------------------------------------------ K3: fp64 MFMA GEMM / Schur update
 * The blocked Schur-complement update of a right-looking LU, C -= W * V (C m x n ld ldc, W m x k
 * ld ldw, V k x n ld ldv; device pointers), on v_mfma_f64_16x16x4f64 with the operands staged in
 * LDS -- the trailing update of the site-tensor getrf and the off-diagonal work of every blocked
 * triangular solve of this library (matrixluci.jl:194-241, tensorci2.jl:620-627 call LAPACK /
 * BLAS there; rrLU itself has no such update: exact full pivoting). */
int tci_schur_update_d(tci_ctx* ctx, double* d_C, int64_t m, int64_t n, int64_t ldc,
                       const double* d_W, int64_t ldw, const double* d_V, int64_t ldv, int64_t k);
/* C = beta * C + alpha * A * op(B); op(B) = B (k x n, ld ldb) or, transb != 0, B^T (B n x k). */
int tci_dgemm_d(tci_ctx* ctx, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* d_A, int64_t lda, const double* d_B, int64_t ldb, double beta,
                double* d_C, int64_t ldc);

/* evaluate(tt, idx) (abstracttensortrain.jl:328-342) of a tensor train at npts points, as the
 * global pivot search needs it (globalpivotfinder.jl:236): cores packed one after another, core
 * t being (bonddims[t], dims[t], bonddims[t+1]) column-major (the site tensors of a TensorCI2);
 * bonddims[0] = bonddims[L] = 1, bond dimensions <= 1024. X: npts x L row-major, 1-based. */
int tci_tt_evaluate_h(tci_ctx* ctx, int32_t L, const int32_t* dims, const int32_t* bonddims,
                      const double* cores, int64_t ncore, const int32_t* X, int64_t npts,
                      double* out);

/* ComplexF64 versions (interleaved re, im): the site-tensor solve T = Pi1 * P^-1
 * (tensorci2.jl:620-627; getrf of P^T with LAPACK's cabs1 partial pivoting) and the tensor-train
 * evaluation (abstracttensortrain.jl:328-342; ncore counts complex entries, X is validated). */
int tci_sitetensor_solve_c128_h(tci_ctx* ctx, const double* P, int64_t r, const double* Pi1,
                                int64_t R, double* T);
int tci_tt_evaluate_c128_h(tci_ctx* ctx, int32_t L, const int32_t* dims, const int32_t* bonddims,
                           const double* cores, int64_t ncore, const int32_t* X, int64_t npts,
                           double* out);

/* ------------------------------------------------- CachedFunction memo on the device
 * CachedFunction{Float64}(f, localdims) (cachedfunction.jl:53-135) over a device integrand: the
 * memo is a hash table in HBM keyed by key(x) = sum((x .- 1) .* coeffs), coeffs =
 * cumprod([1; localdims[1:end-1]]) (:197-199; index spaces below 2^62.5 keys, else TCI_ERR_ARG).
 * tci_cache_batcheval_d/h are tci_batcheval_d/h through the memo (the batch method, :255-302):
 * hits come from the table, the distinct misses of the batch are evaluated in one batch
 * evaluation of f and inserted; *nmiss = how many. The table grows (rehash) as needed. */
int tci_cache_create(tci_ctx* ctx, const int32_t* localdims, int32_t L, int64_t capacity, tci_cache** out);
int tci_cache_destroy(tci_cache* cache);
int tci_cache_clear(tci_cache* cache);                /* clearcache!(cf), :305-308 */
int tci_cache_size(tci_cache* cache, int64_t* n);     /* length of cacheddata(cf) */
/* cacheddata(cf) (:160-170) as (key, value) pairs: up to capacity written, *n = stored entries */
int tci_cache_dump_h(tci_cache* cache, int64_t* keys, double* vals, int64_t capacity, int64_t* n);
/* haskey(cf, x) / cf.cache[key] for npts points X (npts x L row-major, 1-based) without dumping the
 * table: found[q] = 1 and vals[q] = the memoised value when key(X[q]) is stored, else 0. */
int tci_cache_lookup_h(tci_cache* cache, const int32_t* X, int64_t npts, int32_t* found, double* vals);
int tci_cache_batcheval_d(tci_ctx* ctx, tci_cache* cache, const tci_func* f, const int32_t* I, int64_t m,
                          int32_t nl, const int32_t* J, int64_t n, int32_t nr, int32_t M, double* d_out,
                          int64_t ldo, double* maxabs, int64_t* nmiss);
int tci_cache_batcheval_h(tci_ctx* ctx, tci_cache* cache, const tci_func* f, const int32_t* I, int64_t m,
                          int32_t nl, const int32_t* J, int64_t n, int32_t nr, int32_t M, double* out,
                          int64_t ldo, double* maxabs, int64_t* nmiss);

/* ------------------------------------------------- multi-GPU: RCCL over xGMI
 * One process per GPU. Rank 0 makes the 128-byte unique id (tci_comm_unique_id; nbytes gets its
 * size), the host broadcasts it (torch.distributed / MPI / Julia Distributed), every rank
 * creates its communicator on its context's device. Collectives are enqueued on the context
 * stream (asynchronous: synchronise the context before reading results on the host). */
int tci_comm_unique_id(void* id, int64_t* nbytes);
int tci_comm_create(tci_ctx* ctx, int nranks, int rank, const void* id, tci_comm** out);
int tci_comm_destroy(tci_comm* comm);
int tci_comm_allgather_d(tci_comm* comm, const void* d_send, void* d_recv, int64_t bytes);
/* in-place max over ranks of count uint64 words (maxsample as the bit pattern of |x|: non-negative
 * doubles order like their bits, a NaN's bits exceed every finite |x|, Julia's NaN-propagating max) */
int tci_comm_allreduce_max_u64_d(tci_comm* comm, void* d_buf, int64_t count);

/* Column-sharded rrlu! (matrixlu.jl:346-396 with submatrixargmax :46-87 and addpivot! :254-322 split
 * across ranks): rank r holds global columns [c0, c0 + nloc) of the m x n matrix as
 * d_A (ld lda, even) columns 0..nloc-1; column nloc of d_A must exist and is scratch (the pivot
 * column is installed there on every rank). Per pivot every rank runs its pass on its columns, the
 * local winners (32 B each) are all-gathered, the rank owning the global winner contributes that
 * column through an element-wise uint64 max (8 (m + 16) B), both over RCCL when comm is given, else
 * exch, else nranks must be 1; every rank commits the same global winner in the reference's tie order:
 * permutations, npivot, lu.error and pivot errors are bitwise those of tci_rrlu_h on the full
 * matrix, on every rank (rowperm m, colperm n global, 1-based). d_A is clobbered. */
int tci_rrlu_sharded_d(tci_ctx* ctx, tci_comm* comm, tci_exchange_fn exch, void* user, int nranks,
                       double* d_A, int64_t m, int64_t nloc, int64_t lda, int64_t c0, int64_t n,
                       int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowperm,
                       int64_t* colperm, int64_t* npivot, double* lasterror, double* pivoterrors);
/* Factors of the last tci_rrlu_sharded_d on this context, position order as tci_rrlu_h: L (m x np,
 * ld m, identical on every rank; NULL to skip) and this rank's columns of U (np x n, ld ldu: only
 * the columns whose original index lies in [c0, c0 + nloc) are written; the caller combines the
 * ranks' disjoint columns). NaN checks of matrixlu.jl:376-381 on what this rank holds. */
int tci_rrlu_sharded_factors_h(tci_ctx* ctx, double* L, double* U, int64_t ldu);

/* ----------------------------------------------------- synthetic inputs
 * Fills d_A (m x n, ld lda) with U[0,1): splitmix64(seed * 0xD1B54A32D192ED03 + (i + m*j)) >> 11
 * times 2^-53 -- the same stream as the oracle's orc_fill_uniform. */
int tci_fill_uniform_d(tci_ctx* ctx, double* d_A, int64_t m, int64_t n, int64_t lda,
                       uint64_t seed);

/* The same stream from element index `offset` on: (i, j) gets splitmix64(seed * K + offset + i + m*j);
 * offset = m * c0 fills the column block [c0, c0 + n) of the m-row seed matrix (sharded inputs). */
int tci_fill_uniform_block_d(tci_ctx* ctx, double* d_A, int64_t m, int64_t n, int64_t lda,
                             uint64_t seed, uint64_t offset);

/* Diagnostic roofline calibration: average device time (ms) of a 16-B-per-lane stream read of
 * n doubles at d_a, and (if d_b) of a stream copy d_a -> d_b, over `reps` launches of `grid`
 * 256-thread workgroups (grid <= 0: 2048). */
int tci_diag_stream_d(tci_ctx* ctx, const double* d_a, double* d_b, int64_t n, int reps, int grid,
                      double* ms_read, double* ms_copy);

/* Diagnostic: measured fp64 MFMA throughput (TFLOP/s) of independent v_mfma_f64_16x16x4f64
 * chains on every SIMD -- the peak the separable-assembly GEMM is rated against. */
int tci_diag_mfma_f64(tci_ctx* ctx, double* tflops);
/* The same probe with 1, 2 or 4 waves per SIMD (one workgroup per CU); *ghz = clock64 cycles of
 * the loop / its wall time: the shader clock the chip held while issuing fp64 MFMA. */
int tci_diag_mfma_f64_ex(tci_ctx* ctx, int waves_per_simd, double* tflops, double* ghz);

/* ------------------------------------------------------------ device mem */
int tci_malloc_d(tci_ctx* ctx, void** p, int64_t bytes);
int tci_free_d(tci_ctx* ctx, void* p);
int tci_memcpy_h2d(tci_ctx* ctx, void* dst, const void* src, int64_t bytes);
/* device -> pageable host, synchronous; from 64 MB up in 32-MB chunks through two pinned slots (one
 * chunk's DMA in flight while host threads copy the previous one out). The site tensors and
 * MatrixLUCI factors of tci_sitetensor_h / tci_update_pivots_h come back the same way. */
int tci_memcpy_d2h(tci_ctx* ctx, void* dst, const void* src, int64_t bytes);
int tci_memcpy_d2d(tci_ctx* ctx, void* dst, const void* src, int64_t bytes);
/* bytes bytes of dst set to (unsigned char)value, stream-ordered on the context stream (no host
 * synchronisation; e.g. the device max word of tci_batcheval_da) */
int tci_memset_d(tci_ctx* ctx, void* dst, int value, int64_t bytes);
/* strided copy of `height` rows of `width` bytes (e.g. matrix columns between leading dimensions) */
int tci_memcpy2d_d2d(tci_ctx* ctx, void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                     int64_t height);

#ifdef __cplusplus
}
#endif
#endif /* TCI_HIP_H */
