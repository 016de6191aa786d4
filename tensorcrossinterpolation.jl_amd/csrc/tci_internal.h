// tci_internal.h -- shared declarations between the device code (tci_rrlu.hip, tci_device.hip)
// and the C-ABI host layer (tci_abi.cpp). Not part of the public ABI (include/tci_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tci {

constexpr int kMaxPend = 16;       // deferred rank-1 updates kept pending at most (ComplexF64 rrLU; the
                                   // register-resident x's of the real rrLU's k_pass2)
constexpr int kMaxPendR = 32;      // real rrLU: exact pending updates of a two-level epoch (X / Y slots;
                                   // beyond kMaxPend the x's live in LDS, k_pass_x)
constexpr int kRowsPerTile = 512;  // 256 lanes x double2
constexpr int kMaxCB = 16;         // rrLU pass: at most this many columns per tile (measured best)
constexpr int kMaxPassGrid = 2048; // rrLU pass: at most this many workgroups (8 per CU)

// Argmax candidate: abs2 value, the (current, pending-updated) value itself, its column and row
// *positions* (the reference's permuted coordinates: the tie-break keys) and its physical column
// and row. Sentinel: v = -1, positions = INT32_MAX.
struct Cand {
    double v;
    double val;
    int32_t cpos;
    int32_t rpos;
    int32_t pcol;
    int32_t prow;
};

// Device-resident rrLU state (mirrors rrLU.npivot / rrLU.error and the loop-local maxerror of
// _optimizerrlu!, matrixlu.jl:353-369). Written only by the selecting workgroup of a pass.
struct RrluState {
    int64_t np;      // pivots accepted so far
    int32_t done;    // stop test fired (matrixlu.jl:363-365)
    int32_t pad;
    double maxerror;
    double error;    // lu.error (last |A[p,q]| examined)
    int64_t p, q;    // accepted pivot: PHYSICAL row / column
    double pval;     // its current value
};

// Arguments of one rrLU pass (tci_rrlu.hip, k_pass).
struct PassArgs {
    double* A;
    int64_t lda;
    int m, n, k;
    double* X;  // pending x's, [physical row][ldx]
    int64_t ldx;
    double* Y;  // pending y's, [physical column][ldy]
    int64_t ldy;
    int32_t* rowpos;
    int32_t* colpos;
    RrluState* st;
    double* Lp;  // L columns in physical row order (m x maxrank, ld ldl)
    int64_t ldl;
    double* Up;  // U rows in physical column order (maxrank x n, ld ldu)
    int64_t ldu;
    int leftorth;
    Cand* cand;
    int cb;
    int rev;  // walk the tiles in descending memory order (alternated pass to pass, see k_pass)
    // pivot selection fused into the pass's tail (the last workgroup to finish): pivot selk
    // (< 0: none, e.g. after the last pivot)
    int selk;
    int64_t* rowphys;
    int64_t* colphys;
    double* pivvals;
    double reltol, abstol;
    unsigned* ticket;  // zero between passes
    // fp32 shadow of the stale values for the certified read-only passes (k_pass_sh), ld lds
    // (multiple of 4); null when the shadow search is off
    float* S;
    int64_t lds;
    // column-sharded rrLU (tci_rrlu_sharded_d): the pass tail writes its rank-local winner here
    // instead of committing pivot selk (null: commit as usual), its physical column made global by
    // adding pc_off (the rank's first global column; -1 when the rank has no candidate)
    Cand* lout = nullptr;
    int64_t pc_off = 0;
    // two-level epoch: the pass applies pe exact pending updates (the fp64 stale
    // values were last written back after pivot k - pe) and ps of them through the shadow (it was
    // last written -- by a write-back or a refresh -- after pivot k - ps); shadow epochs since the
    // last write-back are nbs pivots long. pe == ps: no refresh since the write-back.
    int pe = 0, ps = 0, nbs = 0;
    // rrlu's copy (matrixlu.jl:462) fused into the initial argmax pass: that pass reads the input
    // from Asrc (ld ldsrc) and writes it to A while it searches (null: A already holds the input)
    const double* Asrc = nullptr;
    int64_t ldsrc = 0;
};

// Selection fields of PassArgs as seen by the device.
struct SelArgs {
    int32_t* rowpos;
    int32_t* colpos;
    int64_t* rowphys;
    int64_t* colphys;
    double* pivvals;
    RrluState* st;
    unsigned* ticket;
    double reltol, abstol;
    int selk;
    Cand* lout;  // non-null: local winner only, no commit (column-sharded rrLU)
    int64_t pc_off;
};

// MPO-MPO contraction integrand (TCI_F_MPO): LDS limits of the environment kernel, in doubles
constexpr int kMpoEnv = 2048;  // ra * rb at every bond
constexpr int kMpoTmp = 8192;  // rb * d2 * ra' and ra * d2 * rb' at every site

// Device view of an integrand (tci_func).
struct FuncDev {
    int32_t kind;
    int32_t L;
    const int32_t* localdims;  // device
    const double* params;      // device
    int64_t nparams;
    const int64_t* strides;    // device, column-major strides for TCI_F_TABLE
    int32_t cpK;               // separable terms (TCI_F_GAUSSMIX, TCI_F_CP; TCI_F_MPO: max ra*rb), host copy
    int64_t ntab;              // TCI_F_LORENTZ: quotient table size (max sum of squares + 1), or 0
    int32_t mpoEnv, mpoTmp;    // TCI_F_MPO: LDS (doubles) of the environment kernel's two buffers
};

// ---- rrLU (tci_rrlu.hip)
int argmax_grid(int m, int n, int k, int cb, int max_grid);
// bytes per element of the rrLU passes' shadow (1: 8-bit codes, 2: fp16, both scaled per epoch;
// 4: fp32)
int shadow_elem_bytes();
bool shadow_two_level();
// the MFMA search's refresh stores reach the whole shadow (lds x n) through one 32-bit buffer
// offset: the two-level epoch needs lds * n * shadow_elem_bytes() <= 0xFFFFFFF0 bytes
inline bool refresh_fits(int64_t lds, int64_t n) { return lds * n * shadow_elem_bytes() <= (int64_t)0xFFFFFFF0; }
// pass after pivot k (k = -1: initial argmax) with P pending updates (slot P-1 = pivot k); its
// last workgroup selects pivot g.selk
// One 1024-thread workgroup per CU with wave-level dynamic column chunks (k_pass2).
// shadow: the initial and write-back passes also store the fp32 shadow g.S, and
// the read-only passes run the certified fp32 search (k_pass_sh; same results, ~half the bytes)
// ComplexF64 rrLU (tci_rrlu_c128.hip): candidate, device state, one step's arguments
struct CCand {
    double v;  // abs2
    int32_t col, row;
};
struct CState {
    int64_t np;
    int32_t done;
    int32_t nan;
    double maxerror;
    double err;
    double2 piv;
    int32_t p, q;  // accepted pivot (physical row / column)
};
struct CStepArgs {
    double2* A;
    int64_t ld;
    int m, n, t, mr, tiles_r, leftorth;
    double reltol, abstol;
    CState* st;
    CCand* cand;
    double2* colbuf;
    double2* rowbuf;
    int64_t* rowperm;
    int64_t* colperm;
    // deferred updates (k_crrlu_*_d): pending slots X[s * ldx + row], Y[s * ldy + col] (s < P),
    // P = pending count seen by reduce / swap, stash: 4 x kMaxPend entries of the swapped rows /
    // columns' slots, read by the swap kernel while its corner thread rewrites them
    double2* X;
    int64_t ldx;
    double2* Y;
    int64_t ldy;
    int P;
    double2* stash;
    // certified shadow search (k_crrlu_step_sh): fp16 planes of the stale values'
    // real / imaginary parts (ld lds, scaled per epoch), the pending x's / y's as f16-split MFMA
    // fragments (XA: 64 halves per row, YB: 2 x 64 per column) and |pivot t| per pivot
    uint16_t* SR;
    uint16_t* SI;
    int64_t lds;
    uint16_t* XA;
    uint16_t* YB;
    double* pmod;
    int sh;  // shadow search on: the swaps maintain the shadow and the fragments
};
int crrlu_grid(int m, int n, int t);
// the shadow search's step for pivot t with P pending (1 <= P <= kCShMaxP), then reduce + swap;
// stale = 1: exact step that also writes the shadow of the stale values (epoch 0)
constexpr int kCShMaxP = 10;
void launch_crrlu_step_sh(hipStream_t s, CStepArgs g, int P);
void launch_crrlu_step_stale_sh(hipStream_t s, CStepArgs g);
void debug_crrlu_check_sh(hipStream_t s, CStepArgs g, int P);
int crrlu_sh_grid(int m, int n, int t);
// the deferred-update pipeline: step<P, flush> (pending applied on the fly, written back when
// flush), then reduce + swap with the pending count P' (0 after a flush) of the step
void launch_crrlu_step_d(hipStream_t s, CStepArgs g, int P, bool flush);
void launch_crrlu_init(hipStream_t s, CState* st, int64_t* rowperm, int64_t* colperm, int m, int n);
void launch_crrlu_step(hipStream_t s, CStepArgs g);
void launch_crrlu_extract(hipStream_t s, const double2* A, int64_t ld, int m, int n, int np,
                          int leftorth, double2* L, double2* U, int64_t ldu, double* pe,
                          int* nanflag);

void launch_c128_scale(hipStream_t s, const double* re, int64_t ldr, int m, int n, double cre,
                       double cim, double2* out, int64_t ldo, unsigned long long* maxbits);
void launch_c128_accum(hipStream_t s, const double* re, int64_t ldr, int m, int n, int comp, double2* out,
                       int64_t ldo);
void launch_c128_finish(hipStream_t s, int m, int n, double cre, double cim, double2* out, int64_t ldo,
                        unsigned long long* maxbits);
void launch_csitetensor_solve(hipStream_t s, const double2* P, int r, const double2* Pi1, int R,
                              double2* T, double2* work, int* piv);
void launch_ctt_eval(hipStream_t s, const double2* cores, const int64_t* off, const int32_t* bd,
                     const int32_t* dims, int L, const int32_t* X, int npts, double2* out);
void launch_cluci_factors(hipStream_t s, const double2* L, const double2* U, int m, int n, int np,
                          int leftorth, const int64_t* rowperm, const int64_t* colperm,
                          double2* left, double2* right);
// kind: 0 read-only, 1 write-back (fp64 + shadow), 2 refresh (shadow only, from the MFMA search's
// values or, when its bound is not tight, from the exact ones); P = g.pe
void launch_pass(hipStream_t s, int P, bool flush, bool shadow, const PassArgs& g, int grid, int kind = -1);
// Persistent shadow epoch (k_pass_mf_epoch): the read-only passes k = g.k .. g.k + npass - 1 (shadow-
// pending counts g.ps .. g.ps + npass - 1 <= kEpochMaxP, g.pe > g.ps: EXT) in one launch of `grid`
// workgroups, which must all be resident at once (one per CU). sync: kEpochSlot zeroed words of this
// launch's own. A launch that finds its grid not co-resident sets st->done = 2 (tci_abi.cpp resumes).
#ifndef TCI_EPOCH_MAXP
#define TCI_EPOCH_MAXP 10
#endif
constexpr int kEpochMaxP = TCI_EPOCH_MAXP;
// The persistent epoch grid was measured slower than the per-pass launches and is
// compiled only with -DTCI_EPOCH_GRID=1 (make variant NAME=epoch VFLAGS=-DTCI_EPOCH_GRID=1); the
// default build has no k_pass_mf_epoch, epoch_fits() is false and tci_set_rrlu_persist(ctx, 1 | 2)
// is refused.
#ifndef TCI_EPOCH_GRID
#define TCI_EPOCH_GRID 0
#endif
constexpr bool kEpochGrid = TCI_EPOCH_GRID != 0;
constexpr int kEpochSlot = 64;  // unsigned words per launch (its ticket at 0; a 256-B line of its own)
void launch_pass_epoch(hipStream_t s, const PassArgs& g, int grid, int npass, int serp, unsigned* sync,
                       long long timeout);
// the persistent epoch launch's LDS maps hold this shape (n <= 32768, columns per workgroup bounded)
bool epoch_fits(int m, int n, int cb, int grid);
void launch_init_state(hipStream_t s, RrluState* st, int32_t* rowpos, int64_t* rowphys, int m,
                       int32_t* colpos, int64_t* colphys, int n);
// small matrices: the whole rrLU in one workgroup's LDS (same outputs as the pass pipeline:
// st, rowphys/colphys, pivvals, Lp (ld ldl, physical rows), Up (ld ldu, physical columns))
// Optionally also the NaN flags (*flag = 1: L, 2: U), the MatrixLUCI factors in their final
// layouts (left m x np, ld m; right np x n, ld np) and a copy of *maxin in *maxout. Null = skip.
// Any of them (and st, rowphys, colphys, pivvals) may point into mapped pinned host memory.
struct SmallOut {
    double* left;
    double* right;
    int* flag;
    const unsigned long long* maxin;
    unsigned long long* maxout;
};
bool rrlu_small_fits(int64_t m, int64_t n);
// mid-size matrices: persistent grid (one workgroup per CU, matrix in LDS), one grid
// barrier per pivot. colbuf: min(ncu, 256) x m doubles; count / fault: device words.
bool rrlu_mid_fits(int64_t m, int64_t n, int ncu);
hipError_t launch_rrlu_mid(hipStream_t s, int ncu, const double* A, int64_t lda, int m, int n, int mr,
                           double reltol, double abstol, int leftorth, RrluState* st, int64_t* rowphys,
                           int64_t* colphys, double* pivvals, double* Lp, int64_t ldl, double* Up,
                           int64_t ldu, Cand* cand, double* colbuf, unsigned* count, int* fault);
hipError_t launch_rrlu_small(hipStream_t s, const double* A, int64_t lda, int m, int n, int mr,
                             double reltol, double abstol, int leftorth, RrluState* st,
                             int64_t* rowphys, int64_t* colphys, double* pivvals, double* Lp,
                             int64_t ldl, double* Up, int64_t ldu, SmallOut out);
// L (m x np, ld ldl) / U (np x n, ld ldu) in position order from the physical-order factors;
// either output may be null (NaN check only). flag |= 1 (NaN in L), 2 (NaN in U).
void launch_extract(hipStream_t s, const double* Lp, int64_t ldlp, const double* Up, int64_t ldup,
                    const double* pivvals, const int64_t* rowphys, const int64_t* colphys, int m,
                    int n, int np, int leftorth, double* L, int64_t ldl, double* U, int64_t ldu,
                    int* flag);

// ---- column-sharded rrLU (tci_rrlu.hip). Rank r holds the global columns [c0, c0 + nloc) as its
// local physical columns 0..nloc-1 plus a ghost column nloc: the column of the last committed
// pivot, installed on every rank so that the unchanged passes derive x_k from it. Per pivot, the
// candidate first: each rank's pass publishes its local winner (lout: a 32-B Cand
// with the GLOBAL physical column); the N records are all-gathered (exchange op 0); k_shard_pick
// reduces them in rank order to the same winner everywhere (abs2, then column position, then row
// position -- submatrixargmax's order) and the ONE rank owning the winning column writes its pending
// y's and stale values into a kShardCol(m)-word buffer, the others zeros; an element-wise max of
// those words as uint64 over the ranks (exchange op 1) leaves the winner's bits everywhere (every
// bit pattern, -0.0 and NaN payloads included, is >= 0 as uint64); k_shard_commit commits the pivot
// to the replicated row / global column maps and installs the ghost. Per pivot 32 B x N + 8 (m +
// kMaxPendR) B cross the ranks, not N x 8 m. One rank: no exchange, the commit reads the column in
// place.
// The fused form (one collective per pivot): every rank all-gathers its record
// AND its own candidate column, kCandWords + shard_col(m) words per rank (k_shard_pack), and
// k_shard_commit takes the winner's column from the winner's slot -- N x 8 (m + kMaxPendR + 4) B
// received per rank instead of two collective latencies.
inline int64_t shard_col(int64_t m) { return m + kMaxPendR; }
constexpr int kCandWords = (int)(sizeof(Cand) / 8);
static_assert(sizeof(Cand) % 8 == 0, "candidate records are whole uint64 words");
void launch_shard_pack(hipStream_t s, const Cand* own_rec, const double* A, int64_t lda, int m, const double* Y,
                       int64_t ldy, int64_t c0, int nloc, uint64_t* send);
void launch_shard_init(hipStream_t s, int32_t* colpos_loc, int nloc, int64_t c0);
void launch_shard_pick(hipStream_t s, const Cand* recv, int nranks, const double* A, int64_t lda, int m,
                       const double* Y, int64_t ldy, int64_t c0, int nloc, uint64_t* colsend);
// recv: rank r's record at recv + r * rstride words. colrecv null and fused 0 (one rank): the
// winner's column and pending y's are read from this rank's A / Y; fused 1: from the winner's slot
void launch_shard_commit(hipStream_t s, const uint64_t* recv, int64_t rstride, int nranks, const uint64_t* colrecv,
                         int fused, int m, int k, RrluState* st, double reltol, double abstol, int32_t* rowpos,
                         int32_t* colpos_g, int64_t* rowphys, int64_t* colphys_g, double* pivvals,
                         int32_t* colpos_loc, int64_t c0, int nloc, double* A, int64_t lda, double* Y,
                         int64_t ldy);
// extraction of a sharded rank's part: U columns whose physical column is in [c0, c0 + nloc)
void launch_extract_shard(hipStream_t s, const double* Lp, int64_t ldlp, const double* Up, int64_t ldup,
                          const double* pivvals, const int64_t* rowphys, const int64_t* colphys, int m,
                          int n, int np, int leftorth, double* L, int64_t ldl, double* U, int64_t ldu,
                          int* flag, int64_t c0, int nloc);

// ---- CachedFunction device memo (tci_cache.hip)
struct CacheProbeArgs {
    unsigned long long* keys;
    double* vals;
    unsigned* state;
    int64_t cap;
    const int64_t* kI;
    const int64_t* kJ;
    int64_t ccoef;
    int64_t m, mR, n;
    double* out;
    int64_t ldo;
    int64_t* miss;
    int64_t* dup;
    unsigned long long* counts;
};
void launch_cache_partial_keys(hipStream_t s, const int32_t* T, int cnt, int w, const int64_t* coeff, int t0,
                               int64_t* out);
void launch_cache_probe(hipStream_t s, const CacheProbeArgs& a);
void launch_cache_gather_points(hipStream_t s, const int64_t* miss, int64_t nmiss, const int32_t* I, int nl,
                                const int32_t* J, int nr, int M, int64_t m, int64_t mR, int32_t* X);
void launch_cache_fill(hipStream_t s, const int64_t* miss, int64_t nmiss, const double* v, double* vals,
                       unsigned* state, int64_t mR, double* out, int64_t ldo);
void launch_cache_dups(hipStream_t s, const CacheProbeArgs& a, int64_t ndup);
void launch_cache_unclaim(hipStream_t s, const int64_t* miss, int64_t nmiss, unsigned long long* keys,
                          unsigned* state);
void launch_cache_lookup(hipStream_t s, const int32_t* X, int64_t npts, int L, const int64_t* coeff,
                         const unsigned long long* keys, const double* vals, const unsigned* state, int64_t cap,
                         int32_t* found, double* out);
void launch_cache_maxabs(hipStream_t s, const double* out, int64_t mR, int64_t n, int64_t ldo,
                         unsigned long long* maxbits);
void launch_cache_rehash(hipStream_t s, const unsigned long long* ok, const double* ov, int64_t ocap,
                         unsigned long long* nk, double* nv, unsigned* ns, int64_t ncap);

// ---- factors, batch evaluation, solve (tci_device.hip)
// MatrixLUCI factors from position-order L (m x np) / U (np x n); L rows >= np (leftorth) or U
// columns >= np (otherwise) are overwritten by the triangular solve.
// dense: bit mask of the fp64 MFMA forms (tci_dense.hip) to use, kDense* below; 0 = the
// round-1 scalar GEMMs / LDS TRSMs / single-workgroup getrf (kept for A/B)
constexpr int kDenseLuci = 1, kDenseGetrf = 2, kDenseGetrs = 4, kDenseGetrfReg = 8, kDenseGetrfCoop = 16,
              kDenseAll = 31;
void launch_luci_factors(hipStream_t s, double* L, int64_t ldl, double* U, int64_t ldu, int m,
                         int n, int np, int leftorth, const int64_t* rowperm,
                         const int64_t* colperm, double* left, double* right, int dense);
void launch_fill_uniform(hipStream_t s, double* A, int64_t m, int64_t n, int64_t lda, uint64_t seed,
                         uint64_t offset = 0);
void launch_stream_read(hipStream_t s, const double* a, int64_t n, unsigned long long* out, int grid);
void launch_stream_copy(hipStream_t s, const double* a, double* b, int64_t n, int grid);

// batch evaluation: I (m x nl) and J (n x nr) device int32 tables, row-major entries.
// scratch must hold batcheval_scratch_bytes() bytes. maxbits: device uint64, zeroed.
// D = prod of the M centre local dims (1 when M == 0).
void launch_batcheval(hipStream_t s, const FuncDev& f, const int32_t* I, int m, int nl,
                      const int32_t* J, int n, int nr, int M, int D, double* out, int64_t ldo,
                      unsigned long long* maxbits, void* scratch);
int64_t batcheval_scratch_bytes(const FuncDev& f, int m, int D, int n);

// ---- fp64 MFMA dense algebra (tci_dense.hip)
// Out = beta C + alpha A op(B) (op(B) = B, or with tb B(t, j) = B[j + t ldb]); Out null: in place
// in C; rmap / cmap (nullable) scatter result (i, j) to Out[rmap[i] + cmap[j] ldo].
// maxbits (nullable): atomicMax of the |result| bit patterns (the fused maxabs of batch evaluation)
void launch_dgemm(hipStream_t s, bool tb, int m, int n, int k, double alpha, const double* A,
                  int64_t lda, const double* B, int64_t ldb, double beta, const double* C,
                  int64_t ldc, double* Out, int64_t ldo, const int64_t* rmap, const int64_t* cmap,
                  unsigned long long* maxbits = nullptr);
// probe: waves_per_simd in {1, 2, 4}, one workgroup per CU; cycles[grid]: clock64 cycles of the loop
void launch_mfma_probe2(hipStream_t s, int waves_per_simd, int grid, int iters, double* sink,
                        long long* cycles);

// diagnostic fp64 MFMA throughput probe: grid x 256 threads, iters x 8 x v_mfma_f64_16x16x4 per wave
void launch_mfma_f64_probe(hipStream_t s, int grid, int iters, double* sink);

// tensor-train values at npts points (X: npts x L, 1-based); rmax = max bond dimension (<= 1024)
void launch_tt_eval(hipStream_t s, const double* cores, const int64_t* off, const int32_t* rdim,
                    const int32_t* dims, int L, const int32_t* X, int npts, double* out, int rmax);

// site-tensor solve: T (R x r) = Pi1 (R x r) * P^-1; P overwritten by its LU (partial pivot of P^T)
// piv: 2 r ints
bool getrf_coop_fits(int r);
void launch_sitetensor_solve(hipStream_t s, double* P, int r, double* Pi1, int R, double* T,
                             int* piv, int dense);

// ---- device-resident small sweep (tci_sweep_small.hip)
constexpr int kSwMaxL = 64;      // tensor-train length the kernel takes
constexpr int kSwPE = 136;       // pivot errors per iteration (np <= 128 on the small path, + lu.error)
constexpr int kSwCatCap = 4096;  // kronecker + extra entries of one combined set before the union
// Host <-> kernel I/O (mapped host memory), byte offsets: int64 header[16] (0 status: 0 done,
// 1 resume at (it, q), 2 / 3 NaN in L / U at bond [7]; 1 it, 2 q, 3 has_history, 4 extra banks
// valid, 5 npe, 6 maxsample bits, 7 bond, 8 fill status (-1 not run, 0 done, 4 non-square pivot
// matrix at bond [9], 5 a site too large for it), 9 bond), int64 counts[6 L] (banks: Iset, Jset, history I / J, extra I / J;
// a width-0 set's count is its number of empty entries), double bonderrors[L], double
// pivoterrors[kSwPE], then the sets bank by bank, site by site, entries row-major.
struct SwIO {
    size_t counts, bonderr, pe, sets;
};
__host__ __device__ inline SwIO sw_io(int L) {
    SwIO o;
    o.counts = 16 * 8;
    o.bonderr = o.counts + (size_t)6 * L * 8;
    o.pe = o.bonderr + (size_t)L * 8;
    o.sets = o.pe + (size_t)kSwPE * 8;
    return o;
}
struct SweepSmallArgs {
    FuncDev f;
    int L;
    int32_t* ws;           // set banks: bank b, site p at ws + cap (b L (L-1) / 2 + widths of sites < p)
    int64_t cap;           // entries per set slot
    const char* inbuf;     // device copy of the input image (SwIO)
    char* out;             // mapped host output image (SwIO)
    int niter, iter1, strategy, strictlynested;
    double abstol;
    int64_t maxbonddim;
    int mode;              // 0: sweep2site! iterations; 1: fillsitetensors!'s maxsample update only;
                           // 2: sweep1site! (s1fwd, s1tens, reltol below)
    int fill;              // mode 0: the maxsample update after the iterations too (header [8] / [9])
    int fsolve = 0;        // modes 0 (fill) / 1: also setsitetensor!'s solve, the tensors into tens / tcap
    int32_t* fmap = nullptr;  // modes 0 (fill) / 1: the per-site work of the fill is left to k_fill_sites
                              // (one workgroup per site): [0] ok flag, then per site (bank of Iset[s],
                              // bank of Jset[s], nI, nJ); the tensors' table entries written here
    int s1fwd, s1tens;     // mode 2: forward sweep; site tensors (MatrixLUCI factors) wanted
    double reltol;         // mode 2: the rrLU's reltol
    double* tens;          // mode 2 / fsolve: [site] (offset, count) int64 pairs, then the tensors (header [10]: used)
    int64_t tcap;          // mode 2 / fsolve: doubles available after the 2 L table entries
    int lu_wave = 1;       // bonds with m, n <= 32: the one-wave rrLU (sw_lu_wave; env TCI_SW_LUWAVE=0: off)
    int lazy_union = 1;    // mode 0: the union without materialising the kronecker products (env TCI_SW_LAZYU=0: off)
    // Chained optimize! (tci_sweep_small_optimize): opt_it > 0, this launch is optimize! iteration
    // opt_it (its abstol = opt_tol * maxsample, or opt_tol without normalizeerror); opt_it < 0, the
    // closing sweep1site! (mode 2). ctl (device): [0] stop (0 running, 1 the loop ended -- converged or
    // maxiter --, 2 iteration ctl[1] could not run on the device), [1] that iteration, [2] / [3] the
    // closing sweep's errornormalization / abstol bits, [8 + i] / [8 + kSwOptMax + i] iteration i's
    // pivot error bits / rank. A launch after the stop does nothing. fmax_in: the previous iteration's
    // fill maxima, folded into maxsample first.
    unsigned long long* ctl = nullptr;
    const unsigned long long* fmax_in = nullptr;
    int opt_it = 0, opt_maxiter = 0, opt_ncheck = 3, opt_norm = 1;
    double opt_tol = 0.0;
    const char* img_sel[2] = {nullptr, nullptr};  // the closing sweep: iteration i's image is img_sel[i & 1]
};
constexpr int kSwOptMax = 64;  // optimize! iterations a chain takes
// sweep1site! on the device (mode 2): the host's request and where the site tensors go
struct SwSweep1 {
    int forward, tensors;  // (a fill with the solve: forward unused, tensors = 1)
    double reltol;
    int64_t tcap;      // doubles of tensor data the caller can take
    int64_t* table;    // [site] (offset, count) into data, 2 L entries (host)
    double* data;      // host
};
bool sweep_small_kind(int kind);
size_t sweep_small_lds_bytes();
hipError_t launch_sweep_small(hipStream_t s, const SweepSmallArgs& a);
// fillsitetensors! after k_sweep_small (modes 0 with fill / 1): every site's Pi1 (max |Pi1| into
// fmax[s] as |v| bits, Julia's NaN-propagating max) and, with a.fsolve, P and T = Pi1 P^-1 into the
// table entries k_sweep_small wrote -- one workgroup per site, all sites at once
hipError_t launch_fill_sites(hipStream_t s, const SweepSmallArgs& a, unsigned long long* fmax);

}  // namespace tci
