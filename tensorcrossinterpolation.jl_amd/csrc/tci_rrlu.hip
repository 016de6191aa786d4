// tci_rrlu.hip -- exact full-pivoting rank-revealing LU (matrixlu.jl:46-87, 254-322, 346-396) on
// gfx950, with deferred rank-1 updates and logical row/column swaps.
//
// The reference does, per pivot k: argmax of abs2 over the trailing block, swaprow!(k,p),
// swapcol!(k,q), normalise, and A[i,j] -= x[i]*y[j] over the trailing block (24 B/element/pivot
// on the CPU: a read pass + a read/write pass).
//
// Here the matrix never moves. The reference's swaps only permute positions, so they are kept as
// maps: rowpos[i] / colpos[j] give the current position of physical row i / column j, rowphys /
// colphys the inverse (= rowpermutation / colpermutation, since physical = original index). The
// trailing block is the set of physical rows/columns whose position is > k, and the argmax key of
// an element is (colpos[j], rowpos[i]): exactly the reference's column-major scan order over the
// permuted matrix (ties -> smallest column position, then row position).
//
// Rank-1 updates are deferred: the trailing values live "stale" in HBM and up to P <= kMaxPend
// pending updates x_s (per physical row) and y_s (per physical column) are applied on the fly,
// in the reference's order and rounding (separate multiply and subtract), by every pass:
//   v = stale[i,j]; for s in pending: v = v - x_s[i]*y_s[j]        (bit-identical values)
// A pass only reads the block (8 B/element) except every nb-th, which writes the values back
// (16 B/element) and empties the pending list. Physical indexing means the pending vectors need
// no swapping. The new pivot's x_k (its column, normalised if leftorth) and y_k (its row,
// normalised otherwise) are computed inside the pass by each workgroup for its own tile, and
// written once (by designated workgroups) as the k-th column of L / row of U, kept in physical
// order until extraction.
//
// Per pivot: select (1 workgroup: winner, stop test, map update) -> pass (<= 2048 workgroups).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "tci_internal.h"
#include "tci_smalllu.h"

#ifndef TCI_PASS2_U
#define TCI_PASS2_U 4  // k_pass2: columns per chunk (two chunks in flight per lane)
#endif
#ifndef TCI_SH_HALF
#define TCI_SH_HALF 1  // shadow of the stale values in fp16, scaled per write-back epoch (0: fp32)
#endif
#ifndef TCI_PASS_SH_U
#define TCI_PASS_SH_U 2  // k_pass_sh: columns per chunk (kShRL rows of the shadow loaded per column)
#endif
#ifndef TCI_SH_MFMA
#define TCI_SH_MFMA TCI_SH_HALF  // fp16 shadow: pending updates applied on the matrix cores (k_pass_mf)
#endif
#ifndef TCI_SH_NT
#define TCI_SH_NT 0  // write-back pass: fp16 shadow stores non-temporal
#endif
#ifndef TCI_SH_TIGHT
#define TCI_SH_TIGHT 7  // shadow search only while its error bound is below 2^-TCI_SH_TIGHT |pivot k|
#endif
#ifndef TCI_FLUSH_NTL
#define TCI_FLUSH_NTL 1  // write-back pass: fp64 loads non-temporal (the shadow stays cached for the next pass)
#endif
#ifndef TCI_FLUSH_NT
#define TCI_FLUSH_NT 1  // write-back pass: fp64 stores non-temporal (the next pass reads the shadow, not them)
#endif

namespace tci {

static constexpr int32_t kBig = 0x7fffffff;

// Shadow element: fp16 (2 B) or fp32 (4 B). The fp16 shadow holds s * v with a power-of-two scale
// s per epoch (the pivots between two write-backs): the stale trailing values of an epoch are
// bounded by B (below), and s = 2^(13 - ilogb B) maps them below 2^14 < 65504. The scale is a
// pure function of the committed pivot values, so the pass that writes the shadow and the passes
// that read it derive the same s. 0 (search off) when B is outside [2^-100, 2^100] or not finite.
constexpr bool kShHalf = TCI_SH_HALF != 0;
// TCI_SH_U8: the narrow shadow in 8 bits instead of fp16 -- q = rint(s v) in [-127, 127] stored as
// the offset-binary byte q + 128, with s = 127 / B per epoch (B the epoch's stale bound, below):
// 1 B per element per read-only pass instead of 2. Read by the MFMA search only (the byte widened
// into the fp32 accumulator, the offset -128 carried by one extra split slot of the MFMA, x = 1
// against y = -128); error bound and certificate in sh_cert.
#ifndef TCI_SH_U8
#define TCI_SH_U8 1
#endif
constexpr bool kShU8 = TCI_SH_U8 != 0;
#if TCI_SH_U8
static_assert(TCI_SH_HALF && TCI_SH_MFMA, "the 8-bit shadow is read by the MFMA search only");
static_assert(!TCI_EPOCH_GRID, "the persistent epoch grid reads the fp16 shadow only");
typedef uint8_t shT;
#elif TCI_SH_HALF
typedef _Float16 shT;
#else
typedef float shT;
#endif
#ifndef TCI_SH_TIGHT_U8
#define TCI_SH_TIGHT_U8 4  // 8-bit shadow: search only while its error bound is below 2^-TCI_SH_TIGHT_U8 |pivot k|
#endif
constexpr int kShTight = kShU8 ? TCI_SH_TIGHT_U8 : TCI_SH_TIGHT;

// s = 2^(13 - ilogb B) maps the stale values below 2^14 and leaves one bit of headroom for the
// pending updates: the certificate needs max |pivot_s| s <= 2^15 (the y's are split into fp16), i.e.
// pivots up to 2 B. (Round 4 used 2^(14 - ilogb B): the first shadow epoch after pass 0, where B is
// |pivot 0| = max |A| and the Schur complement's pivots of a random matrix grow past it, then failed
// its certificate at every pass and ran the exact body -- 8 of every factorisation's passes.)
constexpr int kShExp = 13;
__device__ __forceinline__ double sh_scale(double B) {
    if (!kShHalf) return 1.0;
    if (!(B >= 0x1p-100 && B <= 0x1p100)) return 0.0;
    if constexpr (kShU8) return 127.0 / B;  // (the same fp64 quotient in every pass: deterministic)
    return ldexp(1.0, kShExp - ilogb(B));
}
// upper bound of 1 / sh_scale(B) (exact for the power-of-two fp16 scale)
__device__ __forceinline__ double sh_rscale(double B) {
    if constexpr (kShU8) return B * (1.0 / 127.0) * (1.0 + 0x1p-40);
    return ldexp(1.0, ilogb(B) - kShExp);
}
// the 8-bit code of a scaled value f = s v: clamp to [-127, 127], round to nearest even (the add
// of 1.5 2^23 + 128 leaves rint(f) + 128 in the low byte of the sum's bits; exact for |f| <= 127).
// A NaN clamps to an end of the range (an exact examination then finds the NaN, never selected).
__device__ __forceinline__ uint32_t sh_u8(float f) {
    f = __builtin_fminf(__builtin_fmaxf(f, -127.0f), 127.0f);
    return __float_as_uint(f + 12583040.0f) & 0xFFu;
}
constexpr uint32_t kShU8Zero = 0x80u;  // the code of 0

// Bound on the stale trailing values of the epoch whose first pending pivot is t0. t0 = 0: the
// stale values are A itself, bounded by |pivot 0| (the maximum of A). Otherwise they are the
// Schur complement after pivot t0 - 1: a - x y with |a| <= |pivot t0-1| (the argmax) and
// |x y| <= |pivot t0-1| (one factor normalised by it, the other bounded by it), so <= 2 |pivot t0-1|.
__device__ __forceinline__ double sh_bound(const double* pv, int t0) {
    return t0 == 0 ? fabs(pv[0]) : 2.0 * fabs(pv[t0 - 1]);
}


// (v1,c1,r1) beats (v2,c2,r2): larger abs2, then smaller column position, then smaller row
// position -- the order in which the reference's column-major scan with strict '>' meets them.
__device__ __forceinline__ bool cand_better(double v1, int c1, int r1, double v2, int c2, int r2) {
    return (v1 > v2) || (v1 == v2 && (c1 < c2 || (c1 == c2 && r1 < r2)));
}

struct CandR {  // register form of Cand
    double v, val;
    int cpos, rpos, pc, pr;
};

__device__ __forceinline__ void cand_take(CandR& a, const CandR& b) {
    if (cand_better(b.v, b.cpos, b.rpos, a.v, a.cpos, a.rpos)) a = b;
}

// Wave argmax of the candidates on DPP lane moves (VALU; ds_bpermute shuffles of all six fields
// cost ~2 us per wave on the pass's critical path): (abs2, column position, row position, lane)
// is reduced within rows of 16 lanes (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror), then across the four rows by readlane; the winning lane's fields are read last.
// Candidate abs2 values are never NaN (the passes only take a2 >= best).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

template <int CTRL>
__device__ __forceinline__ void dpp_take_cand(double& bv, unsigned& bc, unsigned& br, unsigned& bl) {
    const uint64_t b = (uint64_t)__double_as_longlong(bv);
    const uint64_t o = ((uint64_t)dpp_u32<CTRL>((unsigned)(b >> 32)) << 32) | dpp_u32<CTRL>((unsigned)b);
    const double ov = __longlong_as_double((long long)o);
    const unsigned oc = dpp_u32<CTRL>(bc), orr = dpp_u32<CTRL>(br), ol = dpp_u32<CTRL>(bl);
    const bool better = (ov > bv) || (ov == bv && (oc < bc || (oc == bc && orr < br)));
    bv = better ? ov : bv;
    bc = better ? oc : bc;
    br = better ? orr : br;
    bl = better ? ol : bl;
}

__device__ __forceinline__ double readlane_dbl(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// every lane ends with the wave's winner
__device__ __forceinline__ void wave_reduce_cand(CandR& c) {
    double bv = c.v;
    unsigned bc = (unsigned)c.cpos, br = (unsigned)c.rpos, bl = threadIdx.x & 63;
    dpp_take_cand<0xb1>(bv, bc, br, bl);
    dpp_take_cand<0x4e>(bv, bc, br, bl);
    dpp_take_cand<0x141>(bv, bc, br, bl);
    dpp_take_cand<0x140>(bv, bc, br, bl);
    double v = readlane_dbl(bv, 0);
    unsigned cc = (unsigned)__builtin_amdgcn_readlane((int)bc, 0);
    unsigned rr = (unsigned)__builtin_amdgcn_readlane((int)br, 0);
    unsigned ln = (unsigned)__builtin_amdgcn_readlane((int)bl, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double ov = readlane_dbl(bv, r);
        const unsigned oc = (unsigned)__builtin_amdgcn_readlane((int)bc, r);
        const unsigned orr = (unsigned)__builtin_amdgcn_readlane((int)br, r);
        const unsigned ol = (unsigned)__builtin_amdgcn_readlane((int)bl, r);
        const bool better = (ov > v) || (ov == v && (oc < cc || (oc == cc && orr < rr)));
        v = better ? ov : v;
        cc = better ? oc : cc;
        rr = better ? orr : rr;
        ln = better ? ol : ln;
    }
    const int w = (int)ln;
    c.v = v;
    c.cpos = (int)cc;
    c.rpos = (int)rr;
    c.val = readlane_dbl(c.val, w);
    c.pc = __builtin_amdgcn_readlane(c.pc, w);
    c.pr = __builtin_amdgcn_readlane(c.pr, w);
}

// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8). The passes map a logical
// index to (row tile, column set) row tile fastest, so with the raw blockIdx an XCD would only
// ever see the row tiles congruent to it mod 8 -- the same offsets in every column, i.e. the same
// subset of memory channels and its own L2 slice pattern (measured: even XCDs ended their
// streaming 2-4 us after odd ones). Giving every XCD a contiguous range of logical indices spreads
// all row tiles over every XCD.
#ifndef TCI_XCD_SPREAD
#define TCI_XCD_SPREAD 1
#endif
__device__ __forceinline__ int xcd_spread(int b, int G) {
    if (!TCI_XCD_SPREAD || (G & 7)) return b;
    return (b & 7) * (G >> 3) + (b >> 3);
}

__device__ __forceinline__ CandR cand_none() { return CandR{-1.0, 0.0, kBig, kBig, 0, 0}; }

// Block reduction; wave 0 ends with the winner.
template <int NT>
__device__ __forceinline__ void block_reduce_cand(CandR& c) {
    __shared__ CandR sc[NT / 64];
    wave_reduce_cand(c);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) sc[w] = c;
    __syncthreads();
    if (w == 0) {
        c = (l < NT / 64) ? sc[l] : cand_none();
        wave_reduce_cand(c);
    }
}

// ------------------------------------------------------------------ pass
// Runs after pivot k has been selected (k = -1: the initial argmax, no pending update). The
// physical matrix is cut into row tiles of 512 rows (256 lanes x double2, 16-B accesses; lda
// even) and column tiles of cb columns. Workgroup w owns row tile w % tiles_r and the column
// tiles q, q + nq, ... (q = w / tiles_r): its rows' pending x's -- and pivot k's x_k, which it derives --
// stay in registers while it walks the chunk, one column tile (and its y's, staged in LDS) at a
// time. Elements outside the trailing block are skipped (columns: uniformly; rows: masked).
// P = pending updates including pivot k's own:
//   x_k[i] = (stale[i,b] - sum_{s<P-1} x_s[i] y_s[b]) (/ piv if leftorth)
//   y_k[j] = (stale[a,j] - sum_{s<P-1} x_s[a] y_s[j]) (/ piv otherwise)
// with (a, b) the pivot's physical row/column. Pending vectors are slot-major, X[s*ldx + i] and
// Y[s*ldy + j], so every access to them is coalesced. Workgroups with q = 0 store x_k (slot P-1
// and L column k), those of row tile 0 store y_k (slot P-1 and U row k).
// Serpentine: with rev set the bands are walked backwards, so a pass starts on the bytes the
// previous pass touched last (still in the 256 MiB Infinity Cache).
//
// Tail: the workgroups publish their candidates (sc1 stores, then one agent-scope atomic add each;
// MI355X_MICROARCH.md hand-off table, first row) and the one whose add comes last reduces them and
// commits pivot sel.selk -- the selection needs no launch of its own. rowpos / colpos / st change
// only there, after every other workgroup has finished reading them.
template <bool COH = false>
__device__ void commit_pivot(int k, const CandR& best, RrluState* st, double reltol, double abstol,
                             int32_t* rowpos, int32_t* colpos, int64_t* rowphys, int64_t* colphys,
                             double* pivvals, int64_t rk = -1, int64_t ck = -1, bool has_mxe = false,
                             double mxe = 0.0);

__device__ __forceinline__ void store_cand_sc1(Cand* dst, const CandR& c) {
    uint64_t* d = reinterpret_cast<uint64_t*>(dst);
    const uint64_t w0 = (uint64_t)__double_as_longlong(c.v);
    const uint64_t w1 = (uint64_t)__double_as_longlong(c.val);
    const uint64_t w2 = (uint64_t)(uint32_t)c.cpos | ((uint64_t)(uint32_t)c.rpos << 32);
    const uint64_t w3 = (uint64_t)(uint32_t)c.pc | ((uint64_t)(uint32_t)c.pr << 32);
    __hip_atomic_store(d + 0, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d + 1, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d + 2, w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(d + 3, w3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ CandR load_cand_sc1(const Cand* src) {
    const uint64_t* s = reinterpret_cast<const uint64_t*>(src);
    const uint64_t w0 = __hip_atomic_load(s + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t w1 = __hip_atomic_load(s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t w2 = __hip_atomic_load(s + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t w3 = __hip_atomic_load(s + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return CandR{__longlong_as_double((long long)w0), __longlong_as_double((long long)w1),
                 (int)(uint32_t)w2, (int)(uint32_t)(w2 >> 32), (int)(uint32_t)w3,
                 (int)(uint32_t)(w3 >> 32)};
}

// Phase profile of one pass (build with -DTCI_PASS_PROF=K): every workgroup stamps entry, end of
// start-up, end of staging, end of streaming and its ticket (100 MHz wall clock); the last one
// prints the spread at pivot selections K and K + 1, including the gap since the previous pass's
// commit.
#ifndef TCI_PASS_PROF
#define TCI_PASS_PROF 0
#endif
#if TCI_PASS_PROF
__device__ unsigned long long g_pprof[kMaxPassGrid * 8 + 8];
__device__ unsigned long long g_pprof_x[kMaxPassGrid * 4];  // thread 0's prologue sub-phases (k_pass_mf)
__shared__ unsigned g_exam_lds;  // exact examinations of this workgroup (k_pass_mf)
__device__ unsigned g_cert_fails;  // read-only / refresh passes whose certificate failed (exact body ran)
#define PPROF(i) (pt[i] = wall_clock64())
#define PPROFX(i)                                                                                   \
    do {                                                                                            \
        if (threadIdx.x == 0)                                                                       \
            __hip_atomic_store(&g_pprof_x[blockIdx.x * 4 + (i)], wall_clock64(), __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_AGENT);                                           \
    } while (0)
#else
#define PPROF(i) ((void)pt)
#define PPROFX(i) ((void)0)
#endif

#ifndef TCI_PASS_ONEP
#define TCI_PASS_ONEP 0  // 1: every EXT read-only pass launches one instance, k_pass_mf<kEpochMaxP, true, false, true>
#endif

#ifndef TCI_TICKET_XCD
#define TCI_TICKET_XCD 0  // pass tail: 1 = per-XCD-class counters + a top counter (measured 2.7 us slower per pass than one counter)
#endif

// Pass tail: block reduction of the workgroups' candidates, then the hand-off to the last one
// (sc1 stores + agent-scope ticket), which reduces all of them and commits pivot sel.selk.
template <int NT>
__device__ __forceinline__ void pass_tail(CandR best, const SelArgs& sel, Cand* __restrict__ cand,
                                          unsigned long long (&pt)[8], int m, int P, int flush) {
    RrluState* st = sel.st;
    (void)m;
    (void)P;
    (void)flush;
    block_reduce_cand<NT>(best);
    if (sel.selk < 0) return;
    __shared__ int last_s;
#if TCI_TICKET_XCD
    // Two-level hand-off (MI355X_MICROARCH.md price list, fanin: shard the counter per XCD): the
    // workgroups of one blockIdx % 8 class (one XCD under the round-robin dispatch; speed only)
    // count on their own line, the last of each class reduces the class's candidates and publishes
    // one, and the last of the <= 8 class leaders reduces those and commits. Each level is the
    // hand-off table's first row (sc1 stores, vmcnt(0), one agent-scope counter, the last adder
    // reads). The reduction order does not matter: cand_better is a strict total order.
    const int ncls = min((int)gridDim.x, 8);
    const int cls = (int)blockIdx.x & 7;
    const int csize = ((int)gridDim.x - cls + 7) >> 3;  // blocks b < grid with b % 8 == cls
    unsigned* ctick = sel.ticket + 16 * (1 + cls);      // own 64-B line
    if (threadIdx.x == 0) {
#if TCI_PASS_PROF
        for (int i = 0; i < 4; ++i)
            __hip_atomic_store(&g_pprof[blockIdx.x * 8 + i], pt[i], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
#endif
        store_cand_sc1(cand + blockIdx.x, best);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(ctick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = (old == (unsigned)csize - 1);
    }
    __syncthreads();
    if (!last_s) return;
    {
        constexpr int CPC = kMaxPassGrid / 8 / NT > 0 ? kMaxPassGrid / 8 / NT : 1;
        CandR cs[CPC];
#pragma unroll
        for (int u = 0; u < CPC; ++u) {
            const int i = threadIdx.x + u * NT;
            cs[u] = i < csize ? load_cand_sc1(cand + cls + 8 * i) : cand_none();
        }
        CandR wc = cs[0];
#pragma unroll
        for (int u = 1; u < CPC; ++u) cand_take(wc, cs[u]);
        __syncthreads();  // block_reduce_cand's LDS slots are reused
        block_reduce_cand<NT>(wc);
        if (threadIdx.x == 0) {
            __hip_atomic_store(ctick, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            store_cand_sc1(cand + kMaxPassGrid + cls, wc);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned old = __hip_atomic_fetch_add(sel.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_s = (old == (unsigned)ncls - 1);
            PPROF(4);
        }
        __syncthreads();
        if (!last_s) return;
    }
    int64_t rk = -1, ck = -1;
    double mxe = 0.0;
    if (threadIdx.x == 0) {
        rk = sel.rowphys[sel.selk];
        ck = sel.colphys[sel.selk];
        mxe = st->maxerror;
    }
    CandR w = threadIdx.x < ncls ? load_cand_sc1(cand + kMaxPassGrid + threadIdx.x) : cand_none();
    __syncthreads();
    block_reduce_cand<NT>(w);
#else
    if (threadIdx.x == 0) {
#if TCI_PASS_PROF
        for (int i = 0; i < 8; ++i)
            if (i < 4 || i >= 6)
                __hip_atomic_store(&g_pprof[blockIdx.x * 8 + i], pt[i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&g_pprof[blockIdx.x * 8 + 5], (unsigned long long)g_exam_lds, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        g_exam_lds = 0;
#endif
        store_cand_sc1(cand + blockIdx.x, best);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old =
            __hip_atomic_fetch_add(sel.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last_s = (old == gridDim.x - 1);
        PPROF(4);
    }
    __syncthreads();
    if (!last_s) return;
    // the physical row / column at position selk (swapped by the commit) and the running maximum
    // pivot error (the stop test): requested with the candidates, not after them
    int64_t rk = -1, ck = -1;
    double mxe = 0.0;
    CandR w;
    constexpr int kWaveCand = 8;  // candidates per lane when wave 0 alone reduces
    if ((int)gridDim.x <= 64 * kWaveCand) {
        // wave 0 alone: every lane's candidates in flight at once, one wave reduction, no barrier
        // (the other waves of the committing workgroup are done)
        if (threadIdx.x >= 64) return;
        if (threadIdx.x == 0) {
            rk = sel.rowphys[sel.selk];
            ck = sel.colphys[sel.selk];
            mxe = st->maxerror;
        }
        CandR cs[kWaveCand];
#pragma unroll
        for (int u = 0; u < kWaveCand; ++u) {
            const int i = threadIdx.x + u * 64;
            cs[u] = i < (int)gridDim.x ? load_cand_sc1(cand + i) : cand_none();
        }
        w = cs[0];
#pragma unroll
        for (int u = 1; u < kWaveCand; ++u) cand_take(w, cs[u]);
        wave_reduce_cand(w);
    } else {
        // all of this thread's candidate loads in flight at once (grid <= kMaxPassGrid)
        constexpr int CPT = kMaxPassGrid / NT;
        if (threadIdx.x == 0) {
            rk = sel.rowphys[sel.selk];
            ck = sel.colphys[sel.selk];
            mxe = st->maxerror;
        }
        CandR cs[CPT];
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int i = threadIdx.x + u * NT;
            cs[u] = i < (int)gridDim.x ? load_cand_sc1(cand + i) : cand_none();
        }
        w = cs[0];
#pragma unroll
        for (int u = 1; u < CPT; ++u) cand_take(w, cs[u]);
        __syncthreads();  // block_reduce_cand's LDS slots are reused
        block_reduce_cand<NT>(w);
    }
#endif
    if (threadIdx.x == 0) {
        __hip_atomic_store(sel.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sel.lout) {  // column-sharded: this rank's winner, committed after the exchange
            *sel.lout = Cand{w.v, w.val, w.cpos, w.rpos, w.v >= 0.0 ? (int32_t)(w.pc + sel.pc_off) : -1, w.pr};
            return;
        }
        commit_pivot(sel.selk, w, st, sel.reltol, sel.abstol, sel.rowpos, sel.colpos, sel.rowphys,
                     sel.colphys, sel.pivvals, rk, ck, true, mxe);
#if TCI_PASS_PROF
        __threadfence();
        PPROF(5);
        unsigned long long* gp = g_pprof;
        const unsigned long long prev5 = gp[kMaxPassGrid * 8];
        gp[kMaxPassGrid * 8] = pt[5];
#ifdef TCI_EXAM_CENSUS
        {  // every pass: the grid's exact examinations (k_pass_mf; 0 for the exact bodies) and the
           // running count of certificate failures -- one line per pass
            unsigned long long tot = 0;
            if (!flush)
                for (int i = 0; i < (int)gridDim.x; ++i)
                    tot += __hip_atomic_load(&gp[i * 8 + 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            printf("[census k=%d P=%d flush=%d grid=%d] exams %llu cert_fails %u\n", sel.selk, P, flush, (int)gridDim.x,
                   tot, __hip_atomic_load(&g_cert_fails, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
#endif
        if (sel.selk == TCI_PASS_PROF || sel.selk == TCI_PASS_PROF + 1) {
            unsigned long long t0min = ~0ull, t0max = 0, t3max = 0, t3min = ~0ull;
            double s01 = 0, s12 = 0, s23 = 0, s06 = 0, s61 = 0, s17 = 0, s72 = 0;
            // stream-end times (from the first entry) averaged by XCD (blockIdx % 8) and by
            // dispatch round (blockIdx / 256)
            unsigned long long ex[8] = {}, eq[8] = {};
            int nx[8] = {}, nr[8] = {};
            for (int i = 0; i < (int)gridDim.x; ++i) {
                unsigned long long t[4];
                for (int z = 0; z < 4; ++z)
                    t[z] = __hip_atomic_load(&gp[i * 8 + z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ex[i % 8] += t[3];
                nx[i % 8]++;
                eq[min(i / 256, 7)] += t[3];
                nr[min(i / 256, 7)]++;
                t0min = min(t0min, t[0]);
                t0max = max(t0max, t[0]);
                t3min = min(t3min, t[3]);
                t3max = max(t3max, t[3]);
                s01 += (double)(t[1] - t[0]);
                s12 += (double)(t[2] - t[1]);
                s23 += (double)(t[3] - t[2]);
                const unsigned long long t6 = __hip_atomic_load(&gp[i * 8 + 6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long t7 = __hip_atomic_load(&gp[i * 8 + 7], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (t6 && t7) {  // thread 0's sub-phases (k_pass_mf only)
                    s06 += (double)(t6 - t[0]);
                    s61 += (double)(t[1] - t6);
                    s17 += (double)(t7 - t[1]);
                    s72 += (double)(t[2] - t7);
                }
            }
            const double us = 0.01, G = (double)gridDim.x;  // 100 MHz ticks

            printf("[pass k=%d P=%d flush=%d grid=%d] gap-since-prev-commit %.2f us | entry spread %.2f | "
                   "avg startup %.2f staging %.2f stream %.2f | first/last stream end %.2f/%.2f | "
                   "ticket->last %.2f | reduce+commit %.2f | total %.2f\n",
                   sel.selk, P, flush, (int)gridDim.x, (double)(t0min - prev5) * us,
                   (double)(t0max - t0min) * us, s01 / G * us, s12 / G * us, s23 / G * us,
                   (double)(t3min - t0min) * us, (double)(t3max - t0min) * us,
                   (double)(pt[4] - t3max) * us, (double)(pt[5] - pt[4]) * us,
                   (double)(pt[5] - t0min) * us);
            {  // the four workgroups that ended streaming last: id, row tile, stream end, examinations
                int top[4] = {-1, -1, -1, -1};
                for (int z = 0; z < 4; ++z) {
                    unsigned long long bestt = 0;
                    for (int i = 0; i < (int)gridDim.x; ++i) {
                        if (i == top[0] || i == top[1] || i == top[2]) continue;
                        const unsigned long long t3 = __hip_atomic_load(&gp[i * 8 + 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (t3 >= bestt) { bestt = t3; top[z] = i; }
                    }
                }
                const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile;
                for (int z = 0; z < 4; ++z) {
                    const int i = top[z];
                    const int wid = xcd_spread(i, (int)gridDim.x);
                    printf("  [k=%d] late wg %d (row tile %d, q %d): stream end %.2f, staged at %.2f, %llu exact examinations\n",
                           sel.selk, i, wid % tiles_r, wid / tiles_r,
                           (double)(__hip_atomic_load(&gp[i * 8 + 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - t0min) * us,
                           (double)(__hip_atomic_load(&gp[i * 8 + 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - t0min) * us,
                           __hip_atomic_load(&gp[i * 8 + 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                }
                unsigned long long tot = 0;
                for (int i = 0; i < (int)gridDim.x; ++i) tot += __hip_atomic_load(&gp[i * 8 + 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                printf("  [k=%d] exact examinations over the grid: %llu\n", sel.selk, tot);
            }
            printf("  [k=%d] thread 0: entry->pivot known %.2f | ->end of startup %.2f | ->y's staged %.2f | ->streaming %.2f\n",
                   sel.selk, s06 / G * us, s61 / G * us, s17 / G * us, s72 / G * us);
            {  // k_pass_mf prologue sub-phases of thread 0 (0 when the kernel has none)
                double x0 = 0, x1 = 0, x2 = 0, x3 = 0;
                int nxs = 0;
                for (int i = 0; i < (int)gridDim.x; ++i) {
                    unsigned long long t0 = __hip_atomic_load(&gp[i * 8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned long long q[4];
                    for (int z = 0; z < 4; ++z)
                        q[z] = __hip_atomic_load(&g_pprof_x[i * 4 + z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (q[0] < t0 || q[3] < q[0]) continue;  // a stale stamp of another kernel
                    x0 += (double)(q[0] - t0);
                    x1 += (double)(q[1] - q[0]);
                    x2 += (double)(q[2] - q[1]);
                    x3 += (double)(q[3] - q[2]);
                    ++nxs;
                }
                if (nxs)
                    printf("  [k=%d] thread 0 prologue (%d wgs): entry->pivot in hand %.2f | ->prefetches issued %.2f | "
                           "->certificate %.2f | ->x/y chain inputs issued %.2f\n",
                           sel.selk, nxs, x0 / nxs * us, x1 / nxs * us, x2 / nxs * us, x3 / nxs * us);
            }
            printf("  [k=%d] end by XCD: %.1f %.1f %.1f %.1f %.1f %.1f %.1f %.1f | by round: %.1f %.1f %.1f %.1f\n",
                   sel.selk, (ex[0] / nx[0] - t0min) * us, (ex[1] / nx[1] - t0min) * us,
                   (ex[2] / nx[2] - t0min) * us, (ex[3] / nx[3] - t0min) * us,
                   (ex[4] / nx[4] - t0min) * us, (ex[5] / nx[5] - t0min) * us,
                   (ex[6] / nx[6] - t0min) * us, (ex[7] / nx[7] - t0min) * us,
                   nr[0] ? (eq[0] / nr[0] - t0min) * us : 0.0, nr[1] ? (eq[1] / nr[1] - t0min) * us : 0.0,
                   nr[2] ? (eq[2] / nr[2] - t0min) * us : 0.0, nr[3] ? (eq[3] / nr[3] - t0min) * us : 0.0);
        }
#endif
    }
}

// ------------------------------------------------------------------ pass, one workgroup per CU
// The same pass (same values, same candidate order) with the work balanced inside each CU. With
// four 256-thread workgroups per CU the oldest one finishes its fixed share first (measured: the
// four dispatch rounds ended 64 / 70 / 79 / 89 us into a 100 us pass) and the CU idles on the last.
// Here a CU runs ONE 1024-thread workgroup: its 512-row tile is cut into 4 row slices of 128 rows
// (one wave each, x's in registers) and every slice is served by 4 waves, which take U-column
// chunks of the workgroup's columns from a per-slice LDS counter -- the faster waves take more.
// Start-up: the first two chunks of every wave are assigned statically and requested before
// anything else; every load that does not need the pivot (maps, pending x's and y's) goes out
// before the pivot is read.
constexpr int kP2Threads = 1024;
constexpr int kP2Slices = kRowsPerTile / 128;              // 128-row slices of a tile
constexpr int kP2Reps = kP2Threads / 64 / kP2Slices;        // waves per slice
constexpr int kP2StageCols = 512;                           // columns staged at once
static_assert(kP2StageCols <= kP2Threads, "one staged column per thread");
#ifndef TCI_SH_RL
#define TCI_SH_RL 4  // shadow search: rows per lane (4: 16-B fp32 loads, 4P registers of x's; 2: 8-B, 2P)
#endif
constexpr int kShRL = TCI_SH_RL;
static_assert(kShRL == 2 || kShRL == 4, "rows per lane");
constexpr int kShSliceRows = 64 * kShRL;                    // shadow search: rows per slice
constexpr int kShSlices = kRowsPerTile / kShSliceRows;
constexpr int kShReps = kP2Threads / 64 / kShSlices;        // waves per slice
static_assert(kShSlices <= kP2Slices, "one LDS chunk counter per slice");

// Kernel view of PassArgs.
struct PassK {
    double* A;
    int64_t lda;
    int m, n, k;
    double* X;
    int64_t ldx;
    double* Y;
    int64_t ldy;
    double* Lp;
    int64_t ldl;
    double* Up;
    int64_t ldu;
    int leftorth;
    Cand* cand;
    int cb;
    int rev;
    float* S;  // fp32 shadow of the stale values (ld lds), or null
    int64_t lds;
    int pe, ps, nbs;  // two-level epoch: exact / shadow pending counts, shadow epoch length
    const double* Asrc;  // initial pass only: the input to copy into A while searching (or null)
    int64_t ldsrc;
};

// LDS of a one-workgroup-per-CU pass: the staged columns' y's [local column][slot] in fp64 (and
// fp32 for the shadow search), their positions, the per-slice chunk counters and the shadow
// search's threshold (float bits; non-negative floats order like their bits).
template <int PP>
struct P2Lds {
    double ys[kP2StageCols * PP];
    float yf[kP2StageCols * PP];
    int cpos[kP2StageCols];
    int cnt[kP2Slices];
    unsigned tau;
    double xk[kRowsPerTile];  // shadow search: x_k of the tile's rows (exact examinations)
};

// Raw buffer stores (the MFMA search's refresh stores): an out-of-range offset is dropped, so a
// chunk issues a fixed number of stores with no branch around them. (Measured in round 4: the
// same treatment of the write-back passes' loads and stores made their waits precise but did not
// make them faster -- 325 us either way; their single-row 8-B stores issued unconditionally cost
// 60 us per deep write-back -- so those keep their branches.)
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
constexpr int kBufOOB = 0x7ffffff0;  // a buffer offset past every num_records: dropped / reads 0
// a raw buffer resource over `bytes` bytes at p (gfx9 dword 3: 0x00020000)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}

// Loads and stores of the data one pass hands to the next (pending X / Y slots, the position maps,
// the pivot values and the state). Between launches the kernel boundary makes them visible; inside
// the persistent epoch kernel (k_pass_mf_epoch) they are handed over without fences, as
// MI355X_MICROARCH.md's hand-off table, first row: every store of them `sc1`, drained before the
// pass's ticket (or, for the commit, before the generation flag), and every load of them a
// `global_load ... sc1` after the consumer's poll has matched. COH = false: plain accesses.
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <bool COH, typename T>
__device__ __forceinline__ T ldc(const T* p) {
    if constexpr (COH)
        return __hip_atomic_load((gptr<T>)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        return *p;
}
template <bool COH, typename T>
__device__ __forceinline__ void stc(T* p, T v) {
    if constexpr (COH)
        __hip_atomic_store((gptr<T>)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// Body of the exact pass (k_pass2). SH: also store the fp32 shadow S of the values this pass
// leaves as the new stale ones (write-back passes) or reads unmodified (the initial pass, P = 0).
// Returns false when the factorisation has already stopped.
template <int P, bool FLUSH, bool SH, bool COH = false>
__device__ __forceinline__ bool pass2_body(const PassK& g, const SelArgs& sel,
                                           P2Lds<(P > 0 ? P : 1)>& L, CandR& best,
                                           unsigned long long (&pt)[8]) {
    RrluState* st = sel.st;
    const int32_t* rowpos = sel.rowpos;
    const int32_t* colpos = sel.colpos;
    double* __restrict__ A = g.A;
    const int64_t lda = g.lda;
    const int m = g.m, n = g.n, k = g.k, cb = g.cb, rev = g.rev, leftorth = g.leftorth;
    double* __restrict__ X = g.X;
    double* __restrict__ Y = g.Y;
    const int64_t ldx = g.ldx, ldy = g.ldy;
    constexpr int U = TCI_PASS2_U;
    static_assert(U <= 8 && 8 % U == 0, "U must divide every column-tile width");
    constexpr int PP = P > 0 ? P : 1;
    double* ys = L.ys;
    int* cpos_s = L.cpos;
    int* cnt = L.cnt;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slice = wave % kP2Slices, rep = wave / kP2Slices;
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile;
    const int tiles_c = (n + cb - 1) / cb;
    const int nq = gridDim.x / tiles_r;
    const int wid = xcd_spread(blockIdx.x, gridDim.x);
    const int tr = wid % tiles_r;
    const int q = rev ? nq - 1 - wid / tiles_r : wid / tiles_r;
    const int ntc = q < tiles_c ? (tiles_c - 1 - q) / nq + 1 : 0;
    const int G = kP2StageCols / cb;
    const int r0 = tr * kRowsPerTile + slice * 128 + 2 * lane;
    const bool rowok = r0 < m, pair = r0 + 1 < m;
    double* const base = A + (rowok ? r0 : 0);  // rows past m read row 0 (never used)
    // the initial pass with rrlu's copy fused: it reads the input (ld ldsrc) and stores every value
    // it reads into A (uniform; the copy's read of the input is this pass's own read)
    const bool cpy = P == 0 && g.Asrc != nullptr;
    const double* const sbase = cpy ? g.Asrc + (rowok ? r0 : 0) : base;
    const int64_t slda = cpy ? g.ldsrc : lda;
    auto chunk_col = [&](int g0, int h) -> int {
        const int it = g0 + (h * U) / cb;
        return (q + (rev ? ntc - 1 - it : it) * nq) * cb + (h * U) % cb;
    };
    auto load_chunk = [&](int g0, int h, double2 (&v)[U]) {
        const int j = chunk_col(g0, h);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double2* pa = reinterpret_cast<const double2*>(sbase + (int64_t)min(j + u, n - 1) * slda);
            if constexpr (FLUSH && TCI_FLUSH_NTL) {
                typedef double dv2 __attribute__((ext_vector_type(2)));
                const dv2 w = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(pa));
                v[u] = double2{w.x, w.y};
            } else {
                v[u] = *pa;
            }
        }
    };
    auto stage_col = [&](int g0) -> int {  // the column this thread stages in group g0 (or -1)
        const int gn = min(G, ntc - g0);
        const int lc = threadIdx.x;
        if (lc >= gn * cb) return -1;
        const int it = g0 + lc / cb;
        return (q + (rev ? ntc - 1 - it : it) * nq) * cb + lc % cb;
    };
    // loads that need no pivot: this thread's rows' positions and pending x's, its staged column's
    // position, then the first two chunks of the matrix
    const int rp0 = rowok ? rowpos[r0] : -1;
    const int rp1 = pair ? rowpos[r0 + 1] : -1;
    double x0[PP], x1[PP];
    if constexpr (P > 1) {
#pragma unroll
        for (int s = 0; s < P - 1; ++s) {
            const double2 u = *reinterpret_cast<const double2*>(X + (int64_t)s * ldx + (rowok ? r0 : 0));
            x0[s] = u.x;
            x1[s] = u.y;
        }
    }
    int jst = ntc > 0 ? stage_col(0) : -1;
    int cpst = (jst >= 0 && jst < n) ? colpos[jst] : -1;
    double2 va[U], vb[U];
    const int nch0 = ntc > 0 ? min(G, ntc) * cb / U : 0;
    if (rep < nch0) load_chunk(0, rep, va);
    if (rep + kP2Reps < nch0) load_chunk(0, rep + kP2Reps, vb);
    if (st->done) return false;
    int a = 0, b = 0;
    double piv = 1.0;
    if (P > 0) {
        a = (int)st->p;
        b = (int)st->q;
        piv = st->pval;
    }
    const bool in0 = rp0 > k, in1 = rp1 > k;
    const bool active = in0 || in1;
    // fp16 shadow scale: of the epoch this write-back starts (first pending pivot k + 1), or of
    // epoch 0 when pass 0 writes the shadow of A
    [[maybe_unused]] const double shs =
        (SH && kShHalf && P > 0) ? sh_scale(sh_bound(sel.pivvals, FLUSH ? k + 1 : 0)) : 1.0;
    if constexpr (P > 0) {
        // x_k of this thread's rows (pivot k's column, pending updates applied)
        const double2 cb2 = *reinterpret_cast<const double2*>(A + (rowok ? r0 : 0) + (int64_t)b * lda);
        double xk0 = cb2.x, xk1 = cb2.y;
#pragma unroll
        for (int s = 0; s < P - 1; ++s) {
            const double yv = Y[(int64_t)s * ldy + b];
            xk0 = __dsub_rn(xk0, __dmul_rn(x0[s], yv));
            xk1 = __dsub_rn(xk1, __dmul_rn(x1[s], yv));
        }
        if (leftorth) {
            xk0 = xk0 / piv;
            xk1 = xk1 / piv;
        }
        x0[P - 1] = xk0;
        x1[P - 1] = xk1;
        if (q == 0 && rep == 0) {
            double* xs = X + (int64_t)(P - 1) * ldx;
            if (in0) {
                stc<COH>(xs + r0, xk0);
                g.Lp[r0 + (int64_t)k * g.ldl] = xk0;
            }
            if (in1) {
                stc<COH>(xs + r0 + 1, xk1);
                g.Lp[r0 + 1 + (int64_t)k * g.ldl] = xk1;
            }
        }
    }
    PPROF(1);
    // wave-uniform: the slice has rows in the trailing block (the passes that write the fp16
    // shadow visit every row: non-trailing rows get shadow 0)
    const bool wact = (SH && kShHalf && P > 0) || __any(active);
    for (int g0 = 0; g0 < ntc; g0 += G) {
        const int gn = min(G, ntc - g0);
        const int nch = gn * cb / U;
        if (g0 > 0) {
            jst = stage_col(g0);
            cpst = (jst >= 0 && jst < n) ? colpos[jst] : -1;
            if (wact) {
                if (rep < nch) load_chunk(g0, rep, va);
                if (rep + kP2Reps < nch) load_chunk(g0, rep + kP2Reps, vb);
            }
            __syncthreads();  // previous group's readers are done with ys / cpos_s / cnt
        }
        if (jst >= 0) {
            const int lc = threadIdx.x;
            cpos_s[lc] = cpst;  // -1 past the last column: skipped like a pivoted one
            if (P > 0 && cpst > k) {
                double yk = A[a + (int64_t)jst * lda];
#pragma unroll
                for (int s = 0; s < P - 1; ++s) {
                    const double ysv = Y[(int64_t)s * ldy + jst];
                    ys[lc * PP + s] = ysv;
                    yk = __dsub_rn(yk, __dmul_rn(X[(int64_t)s * ldx + a], ysv));
                }
                if (!leftorth) yk = yk / piv;
                ys[lc * PP + P - 1] = yk;
                if (tr == 0) {
                    stc<COH>(Y + (int64_t)(P - 1) * ldy + jst, yk);
                    g.Up[k + (int64_t)jst * g.ldu] = yk;
                }
            }
        }
        if (threadIdx.x < kP2Slices) cnt[threadIdx.x] = 2 * kP2Reps;
        __syncthreads();
        if (g0 == 0) PPROF(2);
        if (!wact) continue;
        auto column = [&](double2 v, int lc, int j) {
            const int cp = cpos_s[lc];
            if (cp <= k) return;
            if (P == 0 && cpy && rowok) {  // (columns past n: cp = -1, returned above)
                double* pw = base + (int64_t)j * lda;
                if (pair)
                    *reinterpret_cast<double2*>(pw) = v;
                else
                    pw[0] = v.x;
            }
            if constexpr (SH && kShHalf && !FLUSH && P > 0) {
                // pass 0 of an fp16 shadow: the shadow of the stale values (A itself), whose bound
                // |pivot 0| is known only now. Every row: the epoch starts at pivot 0, so pivot
                // 0's own row counts as pivoted during it (see k_pass_mf)
                if (rowok && kShU8) {
                    uint8_t* ps = reinterpret_cast<uint8_t*>(g.S) + r0 + (int64_t)j * g.lds;
                    const uint32_t c0 = sh_u8((float)(v.x * shs));
                    if (pair)
                        *reinterpret_cast<uint16_t*>(ps) = (uint16_t)(c0 | sh_u8((float)(v.y * shs)) << 8);
                    else
                        ps[0] = (uint8_t)c0;
                } else if (rowok) {
                    _Float16* ps = reinterpret_cast<_Float16*>(g.S) + r0 + (int64_t)j * g.lds;
                    const _Float16 h0 = (_Float16)(float)(v.x * shs);
                    if (pair) {
                        typedef _Float16 h2v __attribute__((ext_vector_type(2)));
                        *reinterpret_cast<h2v*>(ps) = h2v{h0, (_Float16)(float)(v.y * shs)};
                    } else {
                        ps[0] = h0;
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const double y = ys[lc * PP + s];
                v.x = __dsub_rn(v.x, __dmul_rn(x0[s], y));
                v.y = __dsub_rn(v.y, __dmul_rn(x1[s], y));
            }
            // write back trailing rows only: a row outside the block keeps its stale value, which
            // matters for pivot k's own row -- other workgroups read its stale values while
            // staging y_k, concurrently with this store (a second staging group can start after
            // the owner of that row has stored the group's columns)
            if (FLUSH && (in0 || in1)) {
                double2* pa = reinterpret_cast<double2*>(base + (int64_t)j * lda);
                if (!in1) {
                    pa->x = v.x;
                } else if (!in0) {
                    pa->y = v.y;
                } else if (TCI_FLUSH_NT) {
                    typedef double dv2 __attribute__((ext_vector_type(2)));
                    dv2 w = {v.x, v.y};
                    __builtin_nontemporal_store(w, reinterpret_cast<dv2*>(pa));
                } else {
                    *pa = v;
                }
            }
            if constexpr (SH && kShU8 && FLUSH) {
                if (rowok) {  // rows outside the trailing block: 0 (the MFMA search masks by data)
                    uint8_t* ps = reinterpret_cast<uint8_t*>(g.S) + r0 + (int64_t)j * g.lds;
                    const uint32_t c0 = in0 ? sh_u8((float)(v.x * shs)) : kShU8Zero;
                    if (pair)
                        *reinterpret_cast<uint16_t*>(ps) =
                            (uint16_t)(c0 | (in1 ? sh_u8((float)(v.y * shs)) : kShU8Zero) << 8);
                    else
                        ps[0] = (uint8_t)c0;
                }
            } else if constexpr (SH && kShHalf && FLUSH) {
                if (rowok) {  // rows outside the trailing block: 0 (the MFMA search masks by data)
                    _Float16* ps = reinterpret_cast<_Float16*>(g.S) + r0 + (int64_t)j * g.lds;
                    const _Float16 h0 = in0 ? (_Float16)(float)(v.x * shs) : (_Float16)0.0f;
                    if (pair) {
                        typedef _Float16 h2v __attribute__((ext_vector_type(2)));
                        const h2v hw = h2v{h0, in1 ? (_Float16)(float)(v.y * shs) : (_Float16)0.0f};
                        if (TCI_SH_NT)
                            __builtin_nontemporal_store(hw, reinterpret_cast<h2v*>(ps));
                        else
                            *reinterpret_cast<h2v*>(ps) = hw;
                    } else {
                        ps[0] = h0;
                    }
                }
            } else if constexpr (SH && !kShHalf) {
                if ((FLUSH || P == 0) && rowok) {
                    float* ps = g.S + r0 + (int64_t)j * g.lds;
                    if (pair)
                        *reinterpret_cast<float2*>(ps) = make_float2((float)v.x, (float)v.y);
                    else
                        ps[0] = (float)v.x;
                }
            }
            const double a0 = __dmul_rn(v.x, v.x), a1 = __dmul_rn(v.y, v.y);
            if ((in0 && a0 >= best.v) || (in1 && a1 >= best.v)) {
                if (in0) cand_take(best, CandR{a0, v.x, cp, rp0, j, r0});
                if (in1) cand_take(best, CandR{a1, v.y, cp, rp1, j, r0 + 1});
            }
        };
        auto process = [&](int h, const double2 (&v)[U]) {
            const int j = chunk_col(g0, h);
#pragma unroll
            for (int u = 0; u < U; ++u) column(v[u], h * U + u, j + u);
        };
        auto grab = [&]() -> int {
            int h = 0;
            if (lane == 0) h = atomicAdd(&cnt[slice], 1);
            return __shfl(h, 0);
        };
        // h0's values in va, h1's in vb; every grab returns a larger index than both
        int h0 = rep, h1 = rep + kP2Reps;
        while (h0 < nch) {
            process(h0, va);
            h0 = grab();
            if (h0 < nch) load_chunk(g0, h0, va);
            if (h1 >= nch) break;
            process(h1, vb);
            h1 = grab();
            if (h1 < nch) load_chunk(g0, h1, vb);
        }
    }
    return true;
}

template <int P, bool FLUSH, bool SH>
__global__ __launch_bounds__(kP2Threads) void k_pass2(PassK g, SelArgs sel) {
    __shared__ P2Lds<(P > 0 ? P : 1)> L;
    [[maybe_unused]] unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    PPROF(0);
    CandR best = cand_none();
    if (!pass2_body<P, FLUSH, SH>(g, sel, L, best, pt)) return;
    PPROF(3);
    pass_tail<kP2Threads>(best, sel, g.cand, pt, g.m, P, (int)FLUSH);
}

// ------------------------------------------------------------------ shadow search
// A read-only pass must find the exact argmax of abs2 over the updated trailing block, but it
// does not need every exact value: it needs a certificate. The write-back passes (and the
// initial one) also store S = fl32(stale value) (4 B/element). A read-only pass then streams S
// instead of the fp64 values and applies the P pending updates in fp32 (FMA) with fp32 copies of
// x_s and y_s. With M_f = |pivot k-P+1| (every stale trailing value is bounded by it: that pivot
// was the argmax over the block the last write-back left) and |x_s[i] y_s[j]| <= |pivot_s| (full
// pivoting), the fp32 value w of every trailing element is within
//     eps = (P + 3) 2^-23 (M_f + 2 sum_s |pivot_s|) + (P + 2) 2^-124
// of the exact fp64 value v the reference computes (error analysis in DESIGN.md: conversions,
// one rounding per FMA, subnormal flushes, plus the fp64 chain's own roundings, with a 2x margin).
// Every lane keeps the maximum |w| of each chunk it streams; c - eps is a proven lower bound on
// the block's max |v|, and the workgroup shares the best such bound (tau, LDS). A chunk whose
// c + eps falls below tau cannot hold the argmax -- nor any element tied with it in abs2 (the
// comparison keeps a 2^-20 relative margin for the fp32 roundings of c, eps and tau) -- and is
// skipped; the others (the running maxima, a handful per workgroup) are re-read in fp64 and
// examined exactly, in the reference's operation order, with the reference's tie order. The
// workgroup's candidate is therefore exactly what the exact pass produces, and the pass reads
// ~4 B/element instead of 8. NaN elements (never selected by the reference) stay NaN in fp32 and
// drop out of the maxima. When the bound is not tight (eps >= 2^-10 |pivot k|, a rapidly decaying
// block) or fp32 could overflow, the kernel runs the exact body instead (uniform decision).
template <int P>
__device__ __forceinline__ bool pass_sh_body(const PassK& g, const SelArgs& sel, P2Lds<P>& L,
                                             CandR& best, float eps, double shs,
                                             unsigned long long (&pt)[8]) {
    RrluState* st = sel.st;
    const int32_t* colpos = sel.colpos;
    const int m = g.m, n = g.n, k = g.k, cb = g.cb, rev = g.rev;
    const int64_t lda = g.lda, ldx = g.ldx, ldy = g.ldy, lds = g.lds;
    constexpr int U = TCI_PASS_SH_U;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int slice = wave % kShSlices, rep = wave / kShSlices;
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile;
    const int tiles_c = (n + cb - 1) / cb;
    const int nq = gridDim.x / tiles_r;
    const int wid = xcd_spread(blockIdx.x, gridDim.x);
    const int tr = wid % tiles_r;
    const int q = rev ? nq - 1 - wid / tiles_r : wid / tiles_r;
    const int ntc = q < tiles_c ? (tiles_c - 1 - q) / nq + 1 : 0;
    const int G = kP2StageCols / cb;
    // kShRL rows per lane: 8-B (16-B) fp32 loads (lda, ldx and lds are multiples of 4, r0 of kShRL,
    // so the rows of a lane with r0 < m are inside the column)
    constexpr int RL = kShRL, RH = RL / 2;
    typedef float fvec __attribute__((ext_vector_type(RL)));
    typedef shT svec __attribute__((ext_vector_type(RL)));
    const int r0 = tr * kRowsPerTile + slice * kShSliceRows + RL * lane;
    const int rb = r0 < m ? r0 : 0;
    const shT* const sbase = reinterpret_cast<const shT*>(g.S) + rb;
    const int cbs = __builtin_ctz(cb);  // cb is 8 or 16
    auto chunk_col = [&](int g0, int h) -> int {
        const int it = g0 + ((h * U) >> cbs);
        return ((q + (rev ? ntc - 1 - it : it) * nq) << cbs) + ((h * U) & (cb - 1));
    };
    auto load_chunk = [&](int g0, int h, svec (&v)[U]) {
        const int j = chunk_col(g0, h);
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = *reinterpret_cast<const svec*>(sbase + (int64_t)min(j + u, n - 1) * lds);
    };
    auto stage_col = [&](int g0) -> int {
        const int gn = min(G, ntc - g0);
        const int lc = threadIdx.x;
        if (lc >= gn * cb) return -1;
        const int it = g0 + (lc >> cbs);
        return ((q + (rev ? ntc - 1 - it : it) * nq) << cbs) + (lc & (cb - 1));
    };
    int rp[RL];
#pragma unroll
    for (int t = 0; t < RL; ++t) rp[t] = r0 + t < m ? sel.rowpos[r0 + t] : -1;
    const int lrow = slice * kShSliceRows + RL * lane;  // the lane's first row within the tile
    int jst = ntc > 0 ? stage_col(0) : -1;
    int cpst = (jst >= 0 && jst < n) ? colpos[jst] : -1;
    svec va[U], vb[U];
    const int nch0 = ntc > 0 ? min(G, ntc) * cb / U : 0;
    if (rep < nch0) load_chunk(0, rep, va);
    if (rep + kShReps < nch0) load_chunk(0, rep + kShReps, vb);
    if (st->done) return false;
    const int a = (int)st->p, b = (int)st->q;
    const double piv = st->pval;
    // the pivot-row element of this thread's first staged column: requested together with the
    // pivot column below (one memory round trip for both instead of two in sequence)
    const double ypr0 = g.A[a + (int64_t)((jst >= 0 && jst < n) ? jst : 0) * lda];
    unsigned inm = 0;  // bit t: row r0 + t is in the trailing block
#pragma unroll
    for (int t = 0; t < RL; ++t) inm |= (rp[t] > k ? 1u : 0u) << t;
    const bool active = inm != 0;
    // pending x's in fp32; x_k exact (fp64, kept for the exact examinations) and in fp32
    typedef float f2v __attribute__((ext_vector_type(2)));  // packed pairs: v_pk_fma_f32
    f2v xf[P][RH];  // row pairs (0, 1) [, (2, 3)] of the lane
    {
        double xk[RL];
#pragma unroll
        for (int hh = 0; hh < RH; ++hh) {
            const double2 c0 = *reinterpret_cast<const double2*>(g.A + rb + 2 * hh + (int64_t)b * lda);
            xk[2 * hh] = c0.x;
            xk[2 * hh + 1] = c0.y;
        }
#pragma unroll
        for (int s = 0; s < P - 1; ++s) {
            double xs[RL];
#pragma unroll
            for (int hh = 0; hh < RH; ++hh) {
                const double2 u0 = *reinterpret_cast<const double2*>(g.X + (int64_t)s * ldx + rb + 2 * hh);
                xs[2 * hh] = u0.x;
                xs[2 * hh + 1] = u0.y;
                xf[s][hh] = f2v{(float)u0.x, (float)u0.y};
            }
            const double yv = g.Y[(int64_t)s * ldy + b];
#pragma unroll
            for (int t = 0; t < RL; ++t) xk[t] = __dsub_rn(xk[t], __dmul_rn(xs[t], yv));
        }
#pragma unroll
        for (int t = 0; t < RL; ++t)
            if (g.leftorth) xk[t] = xk[t] / piv;
#pragma unroll
        for (int hh = 0; hh < RH; ++hh) xf[P - 1][hh] = f2v{(float)xk[2 * hh], (float)xk[2 * hh + 1]};
        if (rep == 0) {
#pragma unroll
            for (int t = 0; t < RL; ++t) L.xk[lrow + t] = xk[t];
            if (q == 0) {
#pragma unroll
                for (int t = 0; t < RL; ++t)
                    if (inm >> t & 1) {
                        g.X[(int64_t)(P - 1) * ldx + r0 + t] = xk[t];
                        g.Lp[r0 + t + (int64_t)k * g.ldl] = xk[t];
                    }
            }
        }
    }
    PPROF(1);
    const bool wact = __any(active);
    const float margin = 0x1p-20f;
    float tau = 0.0f;  // this lane's view of the workgroup's lower bound on the max |v|
    // chunk h's maximum |w| over the lane's trailing-block elements
    auto approx = [&](int h, const svec (&v)[U]) -> float {
        float cm[RL];
#pragma unroll
        for (int t = 0; t < RL; ++t) cm[t] = 0.0f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int lc = h * U + u;
            if (L.cpos[lc] <= k) continue;  // wave-uniform
            const fvec vf = __builtin_convertvector(v[u], fvec);
            f2v w[RH];
#pragma unroll
            for (int hh = 0; hh < RH; ++hh) w[hh] = f2v{vf[2 * hh], vf[2 * hh + 1]};
#pragma unroll
            for (int s = 0; s < P; ++s) {
                const float y = L.yf[lc * P + s];
                const f2v yy = {y, y};
#pragma unroll
                for (int hh = 0; hh < RH; ++hh) w[hh] = __builtin_elementwise_fma(-xf[s][hh], yy, w[hh]);
            }
#pragma unroll
            for (int hh = 0; hh < RH; ++hh) {
                cm[2 * hh] = fmaxf(cm[2 * hh], fabsf(w[hh].x));
                cm[2 * hh + 1] = fmaxf(cm[2 * hh + 1], fabsf(w[hh].y));
            }
        }
        float c = 0.0f;
#pragma unroll
        for (int t = 0; t < RL; ++t)
            if (inm >> t & 1) c = fmaxf(c, cm[t]);
        return c;
    };
    // exact examination of chunks e0 / e1 (< 0: none; the lane's rows), as the exact pass
    // does it. One call site and rolled loops: it runs for a handful of chunks per workgroup.
    auto examine = [&](int g0, int e0, int e1) {
#pragma unroll 1
        for (int z = 0; z < 2; ++z) {
            const int h = z ? e1 : e0;
            if (h < 0) continue;
            // addresses recomputed here from an opaque copy of the row index: otherwise they are
            // shared with the start-up code's and kept live (in registers) across the whole pass
            int rbx = rb;
            asm volatile("" : "+v"(rbx));
            const int j0 = chunk_col(g0, h);
#pragma unroll 1
            for (int u = 0; u < U; ++u) {
                const int lc = h * U + u;
                const int cp = L.cpos[lc];
                if (cp <= k) continue;
                const int j = j0 + u;
                const double* pa = g.A + rbx + (int64_t)j * lda;
                double v[RL];
#pragma unroll
                for (int hh = 0; hh < RH; ++hh) {
                    const double2 p0 = *reinterpret_cast<const double2*>(pa + 2 * hh);
                    v[2 * hh] = p0.x;
                    v[2 * hh + 1] = p0.y;
                }
#pragma unroll 1
                for (int s = 0; s < P - 1; ++s) {
                    const double y = L.ys[lc * P + s];
#pragma unroll
                    for (int hh = 0; hh < RH; ++hh) {
                        const double2 u0 = *reinterpret_cast<const double2*>(g.X + (int64_t)s * ldx + rbx + 2 * hh);
                        v[2 * hh] = __dsub_rn(v[2 * hh], __dmul_rn(u0.x, y));
                        v[2 * hh + 1] = __dsub_rn(v[2 * hh + 1], __dmul_rn(u0.y, y));
                    }
                }
                const double yk = L.ys[lc * P + P - 1];
#pragma unroll 1
                for (int t = 0; t < RL; ++t) {
                    if (!(inm >> t & 1)) continue;
                    const double vt = __dsub_rn(v[t], __dmul_rn(L.xk[lrow + t], yk));
                    const double a2 = __dmul_rn(vt, vt);
                    if (a2 >= best.v) cand_take(best, CandR{a2, vt, cp, sel.rowpos[r0 + t], j, r0 + t});
                }
            }
        }
    };
    // fold chunk maximum c into the bounds; true when the chunk must be examined exactly
    auto test = [&](float c) -> bool {
        const float lb = fmaxf(c - eps, 0.0f);
        const float ts = __uint_as_float(__hip_atomic_load(&L.tau, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        tau = fmaxf(tau, ts);
        if (lb > tau) {
            tau = lb;
            atomicMax(&L.tau, __float_as_uint(lb));
        }
        return c + eps >= tau - tau * margin;
    };
    for (int g0 = 0; g0 < ntc; g0 += G) {
        const int gn = min(G, ntc - g0);
        const int nch = gn * cb / U;
        if (g0 > 0) {
            jst = stage_col(g0);
            cpst = (jst >= 0 && jst < n) ? colpos[jst] : -1;
            if (wact) {
                if (rep < nch) load_chunk(g0, rep, va);
                if (rep + kShReps < nch) load_chunk(g0, rep + kShReps, vb);
            }
            __syncthreads();
        }
        if (jst >= 0) {
            int lc = threadIdx.x;
            asm volatile("" : "+v"(lc));  // staging addresses: not hoisted out of the group loop
            L.cpos[lc] = cpst;
            if (cpst > k) {
                double yk = g0 == 0 ? ypr0 : g.A[a + (int64_t)jst * lda];
#pragma unroll
                for (int s = 0; s < P - 1; ++s) {
                    const double ysv = g.Y[(int64_t)s * ldy + jst];
                    L.ys[lc * P + s] = ysv;
                    L.yf[lc * P + s] = (float)(ysv * shs);  // in the shadow's scale (exact: 2^e)
                    yk = __dsub_rn(yk, __dmul_rn(g.X[(int64_t)s * ldx + a], ysv));
                }
                if (!g.leftorth) yk = yk / piv;
                L.ys[lc * P + P - 1] = yk;
                L.yf[lc * P + P - 1] = (float)(yk * shs);
                if (tr == 0) {
                    g.Y[(int64_t)(P - 1) * ldy + jst] = yk;
                    g.Up[k + (int64_t)jst * g.ldu] = yk;
                }
            }
        }
        if (threadIdx.x < kShSlices) L.cnt[threadIdx.x] = 2 * kShReps;
        if (g0 == 0 && threadIdx.x == 0) L.tau = 0u;
        __syncthreads();
        if (g0 == 0) PPROF(2);
        auto grab = [&]() -> int {
            int h = 0;
            if (lane == 0) h = atomicAdd(&L.cnt[slice], 1);
            return __shfl(h, 0);
        };
        int h0 = rep, h1 = rep + kShReps;
        int ex0 = -1, ex1 = -1;  // chunks to examine exactly
        if (g0 == 0) {
            // seed: the first two chunks of every wave set the workgroup's bound before any exact
            // examination, so only chunks near the workgroup's maximum are ever re-read
            float c0 = -1.0f, c1 = -1.0f;
            const int e0 = h0, e1 = h1;
            if (wact) {
                if (h0 < nch) {
                    c0 = approx(h0, va);
                    h0 = grab();
                    if (h0 < nch) load_chunk(g0, h0, va);
                }
                if (h1 < nch) {
                    c1 = approx(h1, vb);
                    h1 = grab();
                    if (h1 < nch) load_chunk(g0, h1, vb);
                }
                float lb = fmaxf(fmaxf(c0, c1) - eps, 0.0f);
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) lb = fmaxf(lb, __shfl_xor(lb, off));
                if (lane == 0) atomicMax(&L.tau, __float_as_uint(lb));
            }
            __syncthreads();
            if (!wact) continue;
            tau = __uint_as_float(L.tau);
            if (c0 >= 0.0f && c0 + eps >= tau - tau * margin) ex0 = e0;
            if (c1 >= 0.0f && c1 + eps >= tau - tau * margin) ex1 = e1;
        } else if (!wact) {
            continue;
        }
        // h0's values in va, h1's in vb; every grab returns a larger index than both
        for (;;) {
            if (ex0 >= 0 || ex1 >= 0) examine(g0, ex0, ex1);
            ex0 = ex1 = -1;
            if (h0 >= nch) break;
            {
                const float c = approx(h0, va);
                const int e = h0;
                h0 = grab();
                if (h0 < nch) load_chunk(g0, h0, va);
                if (test(c)) ex0 = e;
            }
            if (h1 < nch) {
                const float c = approx(h1, vb);
                const int e = h1;
                h1 = grab();
                if (h1 < nch) load_chunk(g0, h1, vb);
                if (test(c)) ex1 = e;
            }
        }
    }
    return true;
}

template <int P>
__global__ __launch_bounds__(kP2Threads) void k_pass_sh(PassK g, SelArgs sel) {
    __shared__ P2Lds<P> L;
    [[maybe_unused]] unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    PPROF(0);
    // error bound of the fp32 search over pending pivots k-P+1 .. k (uniform)
    const double* pv = sel.pivvals;
    const int t0 = g.k - P + 1;  // first pending pivot; the shadow holds the stale values after t0 - 1
    const double Mf = fabs(pv[t0]);
    double sumM = 0.0;
#pragma unroll
    for (int s = 0; s < P; ++s) sumM += fabs(pv[t0 + s]);
    const double mag = Mf + 2.0 * sumM;
    // fp16 shadow: everything below runs in the shadow's scale shs (a power of two), and the
    // stored value adds one fp16 rounding of s v (|v| <= Mf): 2^-11 relative via fp32 (double
    // rounding covered by the 2^-10 margin) or half an fp16 subnormal ulp, 2^-25
    const double shs = sh_scale(sh_bound(pv, t0));
    double epsd = (double)(P + 3) * 0x1p-23 * mag * shs + (double)(P + 2) * 0x1p-124;
    if (kShHalf) epsd += 0x1p-11 * (1.0 + 0x1p-10) * Mf * shs + 0x1p-25;
    const bool shok = shs > 0.0 && mag < 0x1p100 &&
                      epsd < ldexp(fabs(pv[g.k]) * shs, -(kShHalf ? TCI_SH_TIGHT : 10));
    CandR best = cand_none();
    bool go;
    if (shok)
        go = pass_sh_body<P>(g, sel, L, best, (float)(epsd * (1.0 + 0x1p-20)), shs, pt);
    else
        go = pass2_body<P, false, false>(g, sel, L, best, pt);
    if (!go) return;
    PPROF(3);
    pass_tail<kP2Threads>(best, sel, g.cand, pt, g.m, P, 0);
}

// ------------------------------------------------------------------ shadow search on MFMA
// The read-only pass of k_pass_sh spends one fp32 FMA per element per pending update on the VALU
// (measured ~2.5 us per pending update per pass at 8192^2), which is what bounded nb. Here the P
// pending updates are one small GEMM per 16 x 16 tile on the matrix cores:
//     W = S - X Y,   v_mfma_f32_16x16x32_f16, C = the fp16 shadow tile converted to fp32,
// with X (16 rows x 3P) and Y (3P x 16 columns) the f16 two-term splits of the pending x's and
// y's (x = xh + xl, y = yh + yl: slots (xh, yh), (xh, yl), (xl, yh) per update; the dropped xl yl
// and the splits' own roundings are ~2^-21 |x y|). Products of f16 are exact in fp32; the MFMA
// accumulates in fp32. One of x, y carries the shadow's scale, so both operands stay below 2^15.
//
// Geometry: a wave owns a 64-row slice (4 MFMA blocks) of its workgroup's 512-row tile, 2 waves
// per slice take 16-column chunks from the slice's LDS counter. Lane l loads 16 consecutive fp16
// rows (32 B) of the chunk's column l & 15; MFMA block b takes rows 16 (l >> 4) + 4 b + t of the
// slice -- i.e. block b's D row i is slice row 16 (i >> 2) + 4 b + (i & 3), and the A fragment
// (x's, registers for the whole pass) follows the same map.
//
// Row masking by data: rows pivoted before the epoch hold shadow 0 (the write-backs store 0 for
// non-trailing rows) and x = 0, so W = 0; a row pivoted during the epoch at step t gets x_s for
// s < t, x_t = 1 (leftorth; the pivot's own x) or pivot t (otherwise) and 0 after, so W is the
// shadow image of its value after update t -- exactly 0 in the reference's arithmetic, |W| <= eps
// here (the row was trailing for every update applied). Neither can raise a chunk's lower bound
// above the true maximum. Rows past m: shadow rows [m, lds) are zero (memset once), x = 0; lanes
// past lds load nothing. Columns are one per lane: a non-trailing column's lane reports no
// maximum.
//
// Error bound (scaled units; |v| <= Mf the stale bound of the epoch, sumM = sum |pivot_s|):
//   fp16 storage of s v:             2^-11 (1 + 2^-9) s Mf + 2^-25
//   f16 splits and dropped xl yl:    2^-19 s sumM + P 2^-24 (subnormal halves)
//   fp32 accumulation, <= 3P + 2 roundings of partial sums <= s (Mf + 2 sumM):  (3P + 4) 2^-23 s mag
// (twice the rounding counts as margin), evaluated below as eps.
constexpr int kMfRows = 64;                            // rows per wave slice
constexpr int kMfBlk = kMfRows / 16;                   // MFMA row blocks per slice
constexpr int kMfSlices = kRowsPerTile / kMfRows;      // slices per tile
constexpr int kMfReps = kP2Threads / 64 / kMfSlices;   // waves per slice
static_assert(kMfBlk == 4, "a lane's 16 loaded rows are 4 blocks of 4");

// P <= 10 pending updates: 3P <= 30 split slots, one MFMA (K = 32) per tile; P <= 15 (the
// deepest read pass at kMaxPend = 16): 3P <= 45 slots, two MFMAs (K = 64). Deep passes keep only
// y_k per staged column in LDS (examinations read the pending y's from Y) so that the 64-slot
// fragments fit.
constexpr int kMfMaxP = 15;
constexpr int kMfExCap = 128;                         // deferred examinations per wave
#ifndef TCI_EXB
#define TCI_EXB 4
#endif
constexpr int kExB = TCI_EXB;  // final examinations with pending y's in memory: updates in flight
static_assert(3 * kMfMaxP <= 64 && kMfMaxP < kMaxPend, "two MFMA K-steps per tile");

template <int P, bool EXT = false>
struct MfGeom {
    static constexpr bool deep = P > 10;
    static constexpr int KS = deep ? 64 : 32;         // split slots per row / column
    static constexpr int KSP = KS + 8;                // LDS stride in halves (spreads banks)
    // exact y's kept per staged column: all P, or (deep search, or an exact epoch longer than the
    // shadow epoch: EXT) only y_k -- the examinations then read the pending y's from Y
    static constexpr bool ymem = deep || EXT;
    static constexpr int YS = ymem ? 1 : P;
};

// v - x_0 y_0 - x_1 y_1 - ... (cnt terms, in order; separate multiply and subtract, the
// reference's arithmetic) with strided x / y loads, kB of each in flight at a time
template <int kB>
__device__ __forceinline__ double pend_apply(double v, const double* __restrict__ xp, int64_t xst,
                                             const double* __restrict__ yp, int64_t yst, int cnt) {
    for (int s0 = 0; s0 < cnt; s0 += kB) {
        double xv[kB], yv[kB];
#pragma unroll
        for (int i = 0; i < kB; ++i)
            if (s0 + i < cnt) {
                xv[i] = xp[(int64_t)(s0 + i) * xst];
                yv[i] = yp[(int64_t)(s0 + i) * yst];
            }
#pragma unroll
        for (int i = 0; i < kB; ++i)
            if (s0 + i < cnt) v = __dsub_rn(v, __dmul_rn(xv[i], yv[i]));
    }
    return v;
}

// Two-level epoch chains, v - p_0 u_0 - p_1 u_1 - ... (cnt <= kMaxPendR - 1 terms, in order;
// separate multiply and subtract): p_s = xp[s xst] per thread, the first kPendPre of them loaded
// early (PendPre: requested before the pivot is read), the rest in one batch after those are
// applied (all at once would cost 62 VGPRs: spills); u_s wave-uniform, lane s of upl. IEEE
// multiplication commutes, so p u is the reference's x y bit for bit.
constexpr int kPendPre = 16;
static_assert(kMaxPendR - 1 <= 2 * kPendPre, "two batches");
struct PendPre {
    double v[kPendPre];
};
// Loads unconditional (slots < kMaxPendR always exist), masked after: a load inside `i < cnt`
// became a branch each, and the other role's branch then began with a wait for all of them.
template <bool COH = false>
__device__ __forceinline__ void pend_pre(PendPre& p, const double* __restrict__ xp, int64_t xst, int cnt) {
    static_assert(kPendPre <= kMaxPendR, "prefetched slots exist");
#pragma unroll
    for (int i = 0; i < kPendPre; ++i) p.v[i] = ldc<COH>(xp + (int64_t)i * xst);
#pragma unroll
    for (int i = 0; i < kPendPre; ++i)
        if (i >= cnt) p.v[i] = 0.0;
}
template <bool COH = false>
__device__ __forceinline__ double pend_chain(double v, const PendPre& p, const double* __restrict__ xp,
                                             int64_t xst, double upl, int cnt) {
#pragma unroll
    for (int i = 0; i < kPendPre; ++i)
        if (i < cnt) v = __dsub_rn(v, __dmul_rn(p.v[i], readlane_dbl(upl, i)));
    if (cnt > kPendPre) {
        double r[kMaxPendR - 1 - kPendPre];
#pragma unroll
        for (int i = 0; i < kMaxPendR - 1 - kPendPre; ++i) r[i] = ldc<COH>(xp + (int64_t)(kPendPre + i) * xst);
#pragma unroll
        for (int i = 0; i < kMaxPendR - 1 - kPendPre; ++i)
            if (kPendPre + i < cnt) v = __dsub_rn(v, __dmul_rn(r[i], readlane_dbl(upl, kPendPre + i)));
    }
    return v;
}

template <int P, bool EXT = false>
struct P2MfLds {
    using Gm = MfGeom<P, EXT>;
    double ys[kP2StageCols * Gm::YS];                 // exact y's of the staged columns (examinations)
    _Float16 yb[kP2StageCols * Gm::KSP];              // their B fragments (y splits)
    int cpos[kP2StageCols];
    int cnt[kMfSlices];
    unsigned tau;
    double xk[kRowsPerTile];                          // x_k of the tile's rows
    // the tile's rows' A fragments are read into registers before the first examination list
    // entry is written (a barrier lies between), so the two share the space
    union {
        _Float16 xa[kRowsPerTile * Gm::KSP];          // -x splits
        struct {
            unsigned ex[kP2Threads / 64 * kMfExCap];  // per-wave lists of blocks to examine exactly
            float exm[kP2Threads / 64 * kMfExCap];    // their approximate maxima
        } e;
    } u;
};

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
// a lane's 16 shadow rows of one column: two h8v (fp16) or one u32x4v (8-bit codes)
typedef std::conditional<kShU8, u32x4v, h8v>::type ShVec;
constexpr int kShVecs = kShU8 ? 1 : 2;

__device__ __forceinline__ void f16_split(double v, _Float16& hi, _Float16& lo) {
    hi = (_Float16)(float)v;
    lo = (_Float16)(float)(v - (double)hi);
}

// Two-level epoch: EXT -- the exact epoch is longer than the shadow epoch: the pass
// applies the P shadow-pending updates on the matrix cores, but x_k, y_k and the exact
// examinations apply all PE = g.pe exact-pending ones (the shadow epoch's slots are the last P of
// them). RF -- a refresh: the pass also writes the shadow of the values it computes (W, updated
// through pivot k, scaled for the epoch that starts at k + 1; rows outside the trailing block 0),
// so the next shadow epoch starts without a write-back of the fp64 values.
// The certificate of a shadow-search pass after pivot k (two-level epoch): the
// current shadow epoch started at t0 = k - PS + 1, the exact epoch at te = k - PE + 1, and every
// shadow epoch in [te, t0) (nbs pivots each) ended with a refresh. In absolute units, with
// |v| <= Mf the epoch's stale bound, d the error of its shadow against the exact stale values
// (0 after a write-back or an exact refresh, else the bound of the refresh pass's W) and
// sumM = sum |pivot_s| over its pending updates:
//   d + 2^-11 (1 + 2^-9) (Mf + d) + 2^-25 / s     fp16 storage (s the epoch's scale)
//     + 2^-19 sumM + P 2^-24 / s                   f16 splits, dropped xl yl
//     + (3P + 4) 2^-23 (Mf + d + 2 sumM)           fp32 accumulation
// The search runs while that is below 2^-TCI_SH_TIGHT |pivot k| (else the exact body, uniform).
// Each pass re-derives the decisions of the refreshes before it from the pivot values with this
// same function, so every pass agrees with what they did.
struct ShCert {
    double eps;  // scaled units of the current epoch
    double shs;  // the current epoch's scale
    bool ok;
};
// the pivot values pv[te - 1 .. k] (PE + 1 <= 33 of them), one load per lane (read back with
// readlane: a loop of dependent scalar loads cost ~5 us at PE ~ 26, phase profile of round 3); a
// separate step so that the load goes out first and sh_cert's wait counts only the loads after it
template <bool COH = false>
__device__ __forceinline__ double sh_cert_load(const double* pv, int k, int PE) {
    const int lane = threadIdx.x & 63, ix = k - PE + lane;
    // unconditional, unmasked: sh_cert reads lanes 0 .. PE only, and lane 0 (pivot te - 1) only
    // when te >= 1 (for te = 0 it takes |pivot 0| instead), so the clamped lanes are never read
    (void)lane;
    return ldc<COH>(pv + min(max(ix, 0), k));
}
__device__ __forceinline__ ShCert sh_cert(double w, int k, int PS, int PE, int nbs) {
    const int te = k - PE + 1, t0 = k - PS + 1;
    auto at = [&](int t) { return readlane_dbl(w, t - te + 1); };
    double d = 0.0;
    ShCert c{0.0, 0.0, false};
    for (int e = te;; e += nbs) {
        const bool cur = e >= t0;
        const int ke = cur ? k : e + nbs - 1;  // the pass whose certificate this is
        const int P = ke - e + 1;
        double sumM = 0.0, maxM = 0.0;
        for (int t = e; t <= ke; ++t) {
            sumM += fabs(at(t));
            maxM = fmax(maxM, fabs(at(t)));
        }
        const double B = e == 0 ? fabs(at(0)) : 2.0 * fabs(at(e - 1));  // sh_bound(pv, e)
        const double s = sh_scale(B);
        // >= 1 / s without a division: fp16, s is a power of two (or 0, then unused), so x / s ==
        // x * rs exactly -- the two fp64 divisions per epoch had been ~1/3 of this function's time on
        // the pass's critical path; u8, B / 127 rounded up
        const double rs = kShHalf ? (s > 0.0 ? sh_rscale(B) : 0.0) : 1.0;
        const double Mfd = fabs(at(e)) + d;
        const double mag = Mfd + 2.0 * sumM;
        double ea = 0.0;
        if (s > 0.0) {
            if constexpr (kShU8) {
                // the 8-bit code: half a unit from the rounding to an integer (the clamp can only move
                // a value towards the exact one: |s v| <= 127 for every stale value), 2^-14 for the
                // fp32 scaling and rescaling products; the accumulator's partial sums also carry the
                // byte offset (+-128 +- 255) and one more term (the offset slot)
                ea = d + (0.5 + 0x1p-14) * rs + 0x1p-19 * sumM + (double)P * 0x1p-24 * rs +
                     (double)(3 * P + 5) * 0x1p-23 * (mag + 384.0 * rs);
            } else {
                ea = d + 0x1p-11 * (1.0 + 0x1p-9) * Mfd + 0x1p-25 * rs + 0x1p-19 * sumM + (double)P * 0x1p-24 * rs +
                     (double)(3 * P + 4) * 0x1p-23 * mag;
            }
        }
        c.ok = s > 0.0 && mag < 0x1p100 && maxM * s <= 0x1p15 && ea * s < ldexp(fabs(at(ke)) * s, -kShTight);
        if (cur) {
            c.eps = ea * s;
            c.shs = s;
            return c;
        }
        d = c.ok ? ea : 0.0;  // a refresh that could not certify its bound wrote exact values
    }
}

// Returns 0 when the factorisation has stopped, 1 after the pass, 2 when the certificate fails
// (nothing done: the caller runs the exact body). The certificate is derived after the
// pivot-independent loads are issued, so its pivot-value round trip overlaps theirs.
constexpr int kMfStop = 0, kMfDone = 1, kMfExact = 2;
// The persistent epoch kernel's per-pass inputs of pass_mf_body (COH): the pivot k the workgroup
// selected itself (every workgroup reduces the previous pass's candidates), the positions of its rows
// and columns (LDS copies, patched by every selection), and the pivot values selected inside the
// launch (LDS; pivots <= k0 are in the global pivot values).
struct EpochIn {
    int a, b;             // pivot k: physical row / column
    double piv;           // its value
    const int32_t* lrow;  // LDS: position of tile row r at lrow[r - tile base]
    const int16_t* lcol;  // LDS: position of the workgroup's column j at lcol[t cb + (j mod cb)], t its tile's
                          // sequence number among the workgroup's tiles; -1 past n (n <= 32768)
    const double* lpiv;   // LDS: pivot k0 + 1 + i at lpiv[i]
    int k0;               // pivots <= k0 were committed before the launch
    __device__ __forceinline__ double pivot(const double* pv, int t) const { return t > k0 ? lpiv[t - k0 - 1] : pv[t]; }
};
template <int P, bool EXT = false, bool RF = false, bool COH = false>
__device__ __forceinline__ int pass_mf_body(const PassK& g, const SelArgs& sel, P2MfLds<P, EXT>& L,
                                            CandR& best, unsigned long long (&pt)[8], const int Pr = P,
                                            const EpochIn* ep = nullptr) {
    static_assert(P >= 1 && P <= kMfMaxP, "at most two MFMA K-steps per tile");
    using Gm = MfGeom<P, EXT>;
    // Pr: the shadow-pending count, P its compile-time bound (register arrays, LDS strides): equal in
    // the per-pass kernels, P = kEpochMaxP in the persistent epoch kernel (one body for every depth)
    const int PE = EXT ? g.pe : Pr;  // exact pending updates; the shadow's are slots off .. PE - 1
    const int off = PE - Pr;
    constexpr int KS = Gm::KS, KSP = Gm::KSP, KSt = KS / 32;
    RrluState* st = sel.st;
    const int32_t* colpos = sel.colpos;
    const int32_t* rowpos = sel.rowpos;
    const double* pv = sel.pivvals;
    const int m = g.m, n = g.n, k = g.k, cb = g.cb, rev = g.rev, leftorth = g.leftorth;
    const int64_t lda = g.lda, ldx = g.ldx, ldy = g.ldy, lds = g.lds;
    const int t0 = k - Pr + 1;
    // The certificate's pivot values and the pivot the previous pass committed: the pass's first
    // loads. The compiler moves the pivot to scalar registers at once, i.e. waits for it right
    // here -- one round trip, after which the prologue's pivot-independent loads (maps, first
    // chunks, pending slots) go out together with the pivot-dependent ones. (Requested after the
    // prefetches instead, that wait also covered the first shadow chunks of the whole grid: +0.2
    // ms per step; read after the certificate and behind serial map loads, the pivot had been the
    // third or fourth round trip.) Vector loads: as scalar loads they were waited for by the next
    // kernel-argument reload (lgkmcnt(0)).
    // COH (the persistent epoch kernel): the pivot comes from the workgroup's own reduction of the
    // previous pass's candidates, the maps from its LDS copies, the pivots of this launch from LDS
    double certw;
    int st_done, a, bq;
    double piv;
    if constexpr (COH) {
        certw = ep->pivot(pv, min(max(k - PE + (int)(threadIdx.x & 63), 0), k));
        st_done = 0;
        a = ep->a;
        bq = ep->b;
        piv = ep->piv;
    } else {
        certw = sh_cert_load<COH>(pv, k, PE);
        st_done = ldc<true>(&st->done);
        a = (int)ldc<true>(&st->p);
        bq = (int)ldc<true>(&st->q);
        piv = ldc<true>(&st->pval);
    }
#if TCI_PASS_PROF
    if (threadIdx.x == 0) asm volatile("" ::"s"(a), "s"(bq));  // (the pivot in hand)
#endif
    PPROFX(0);
    // thread / workgroup indices: inside the persistent epoch kernel (COH) made opaque per pass, so
    // that nothing derived from them is hoisted out of its pass loop (kept live across every pass,
    // those values spilled the body's registers)
    int tx = (int)threadIdx.x, bx = (int)blockIdx.x, gx = (int)gridDim.x;
    if constexpr (COH) asm volatile("" : "+v"(tx), "+s"(bx), "+s"(gx));
    const int lane = tx & 63, wave = tx >> 6;
    const int slice = wave % kMfSlices, rep = wave / kMfSlices;
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile;
    const int tiles_c = (n + cb - 1) / cb;
    const int nq = gx / tiles_r;
    const int wid = xcd_spread(bx, gx);
    const int tr = wid % tiles_r;
    // (COH: a workgroup keeps its column set in every pass -- its LDS map covers it; the serpentine
    // order is kept by walking its tiles backwards, which walks the bands backwards as well)
    const int q = (rev && !COH) ? nq - 1 - wid / tiles_r : wid / tiles_r;
    const int ntc = q < tiles_c ? (tiles_c - 1 - q) / nq + 1 : 0;
    const int G = kP2StageCols / cb;
    const int cbs = __builtin_ctz(cb);  // cb is 8 or 16
    const int tb = tr * kRowsPerTile;
    const int sb = tb + slice * kMfRows;        // the slice's first row
    const int gq = lane >> 4, lcol = lane & 15;  // lane's row quad / column within a chunk
    const int rl = sb + 16 * gq;                 // first of the lane's 16 loaded rows
    const bool rload = rl < lds;                 // lds is a multiple of 16
    const shT* const sbase = reinterpret_cast<const shT*>(g.S) + (rload ? rl : 0);
    auto col_of = [&](int g0, int lc) -> int {  // global column of staged local column lc
        const int it = g0 + (lc >> cbs);
        return ((q + (rev ? ntc - 1 - it : it) * nq) << cbs) + (lc & (cb - 1));
    };
    // COH: index of staged local column lc in the workgroup's LDS column map (by tile sequence)
    [[maybe_unused]] auto lcol_of = [&](int g0, int lc) -> int {
        const int it = g0 + (lc >> cbs);
        return ((rev ? ntc - 1 - it : it) << cbs) + (lc & (cb - 1));
    };
    // positions of a row of the tile / a staged column: global maps, or (COH) the LDS copies
    auto rowpos_of = [&](int r) -> int {
        if constexpr (COH)
            return ep->lrow[r - tb];
        else
            return rowpos[r];
    };
    // Every chunk load is issued unconditionally (a lane past the last column reads the last one,
    // a lane past the last row tile row 0: approx() masks both), so that a fixed number of memory
    // instructions follows each chunk's loads and the compiler waits for that chunk alone.
    // a lane's 16 rows of one column: 32 B of fp16 (two h8v) or 16 B of 8-bit codes (one u32x4v)
    auto load_chunk = [&](int g0, int gcols, int h, ShVec (&v)[kShVecs]) {
        const int lc = h * 16 + lcol;
        const int j = lc < gcols ? col_of(g0, lc) : n;
        const ShVec* p = reinterpret_cast<const ShVec*>(sbase + (int64_t)(j < n ? j : n - 1) * lds);
#pragma unroll
        for (int i = 0; i < kShVecs; ++i) v[i] = p[i];
    };
    // staging: threads 0 .. 511 (one staged column each); the tile's rows: threads 512 .. 1023
    const bool stager = tx < kP2StageCols;
    auto stage_col = [&](int g0) -> int {
        const int gn = min(G, ntc - g0);
        const int lc = tx;
        if (!stager || lc >= gn * cb) return -1;
        return col_of(g0, lc);
    };
    // Map loads: every one issued unconditionally at a clamped index and tested afterwards -- with
    // the test folded into the load's condition (r < m && rowpos[r] > k) each became a branch
    // with its own wait, four (a refresh: twenty) dependent round trips before the pivot read.
    // wave activity from the rows of its slice (lanes 0..15 x 4: every row once)
    int rpa[kMfBlk];
#pragma unroll
    for (int b = 0; b < kMfBlk; ++b) rpa[b] = rowpos_of(min(sb + 16 * (lcol >> 2) + 4 * b + (lcol & 3), m - 1));
    // refresh: which of the lane's 16 loaded rows are trailing (the others get shadow 0)
    [[maybe_unused]] int rpt[RF ? 16 : 1];
    if constexpr (RF) {
#pragma unroll
        for (int i = 0; i < 16; ++i) rpt[i] = rowpos_of(min(rl + i, m - 1));
    }
    // refresh stores: the shadow as one buffer (the host keeps it below 4 GB for refreshes), the
    // second 16 B of a lane's 32 through a resource 16 B further on (an out-of-range offset stays so)
    [[maybe_unused]] const int shb = (int)(unsigned)min((int64_t)lds * n * (int64_t)sizeof(shT), (int64_t)0xFFFFFFF0);
    [[maybe_unused]] const auto rsS0 = buf_rsrc(g.S, shb);
    [[maybe_unused]] const auto rsS1 = buf_rsrc(reinterpret_cast<const char*>(g.S) + 16, shb - 16);
    int jst = ntc > 0 ? stage_col(0) : -1;
    int cpl;
    if constexpr (COH)
        cpl = ep->lcol[jst >= 0 ? lcol_of(0, tx) : 0];
    else
        cpl = colpos[min(max(jst, 0), n - 1)];
    const int prow = tx - kP2StageCols;  // this thread's tile row (row threads)
    const int rrow = tb + (prow >= 0 ? prow : 0);
    const int rpl = rowpos_of(min(rrow, m - 1));
    ShVec va[kShVecs], vb[kShVecs];
    const int gc0 = ntc > 0 ? min(G, ntc) * cb : 0;
    const int nch0 = (gc0 + 15) / 16;
    // unconditional (no columns: chunk 0 of an empty group reads column n - 1, never used)
    load_chunk(0, gc0, max(min(rep, nch0 - 1), 0), va);
    load_chunk(0, gc0, max(min(rep + kMfReps, nch0 - 1), 0), vb);
    // (the map values are tested where they are first needed, after the pivot-dependent loads have
    // gone out: tested here, their wait held those loads back by a round trip)
    // EXT: the pivot-independent side of this thread's chain (row thread: X[s][row]; stager:
    // Y[s][column]), all PE - 1 of them requested before the pivot is read
    [[maybe_unused]] PendPre pre;
    if constexpr (EXT) {
        // one call for both roles (the row threads' x slots, the stagers' y slots): as two
        // calls under the role's branch, the second began with a wait for the first's loads
        pend_pre<COH>(pre, stager ? g.Y + (jst >= 0 && jst < n ? jst : 0) : g.X + (rrow < m ? rrow : 0),
                 stager ? ldy : ldx, PE - 1);
    }
    PPROFX(1);
    // The pivot-dependent chain inputs go out before the certificate is derived, so that its scalar
    // arithmetic (~2 us at PE ~ 28, EXT prologue profile of round 5) overlaps their round trip: EXT,
    // lane s of every wave holds the pivot's side, X[s][a] (stager waves) or Y[s][bq] (row waves) --
    // one load per lane, no barrier; the row threads' A[row][bq], the stagers' A[a][column] (EXT).
    // (Clamped: after the last pivot the state's p, q are not meaningful; those values are unused.)
    // The chains that readlane upl run on whole waves (the stager / row split is by wave): a
    // spilled upl reloaded under a partial exec mask would leave the inactive lanes' values undefined.
    const int ac = min(max(a, 0), m - 1), bc = min(max(bq, 0), n - 1);
    const int jj = jst >= 0 && jst < n ? jst : 0;
    [[maybe_unused]] double upl = 0.0;
    if constexpr (EXT) {
        upl = ldc<COH>((stager ? g.X + ac : g.Y + bc) + (int64_t)min(lane, kMaxPendR - 1) * (stager ? ldx : ldy));
    }
    double a0 = 0.0;
    if (!stager)
        a0 = g.A[(rrow < m ? rrow : 0) + (int64_t)bc * lda];
    else if constexpr (EXT)
        a0 = g.A[ac + (int64_t)jj * lda];
    const ShCert cert = sh_cert(certw, k, Pr, PE, g.nbs > 0 ? g.nbs : Pr);
#if TCI_PASS_PROF
    if (threadIdx.x == 0) asm volatile("" ::"v"(cert.eps));
#endif
    PPROFX(2);
#ifdef TCI_EPOCH_DEBUG
    {
        const double c0 = readlane_dbl(certw, 0), c1 = readlane_dbl(certw, 1), c2 = readlane_dbl(certw, 2),
                     c3 = readlane_dbl(certw, 3), c4 = readlane_dbl(certw, 4);
        if (tx == 0 && bx == 0 && k < 12)
            printf("[%s k=%d Pr=%d PE=%d nbs=%d] cert ok=%d eps=%g shs=%g pv lanes %.17g %.17g %.17g %.17g %.17g\n",
                   COH ? "epoch" : "pass", k, Pr, PE, g.nbs, (int)cert.ok, cert.eps, cert.shs, c0, c1, c2, c3, c4);
    }
#endif
    if (!cert.ok) return kMfExact;
    const float eps = (float)(cert.eps * (1.0 + 0x1p-20));
    const double shs = cert.shs;
    [[maybe_unused]] const float rscale =
        RF ? (float)(sh_scale(sh_bound(pv, k + 1)) / shs) : 1.0f;  // a power of two: exact
    if (st_done) return kMfStop;
    PPROF(6);
    if (!stager) {
        // row thread: x_k of its row (the reference's operation order), the split A fragment row
        // -(x_0 .. x_{P-1}) with the data masking of rows outside the trailing block
        const int rr = rrow < m ? rrow : 0;
        double xs[P];
        if constexpr (!EXT) {
#pragma unroll
            for (int s = 0; s < P - 1; ++s)
                if (s < Pr - 1) xs[s] = ldc<COH>(g.X + (int64_t)(off + s) * ldx + rr);
        }
        double xk = a0;
        if constexpr (EXT) {  // all PE - 1 exact pending updates
            // the shadow-pending x's first: pivot-independent, in flight with the chain's loads
            // (requested after the chain they were one more round trip before the barrier)
#pragma unroll
            for (int s = 0; s < P - 1; ++s)
                if (s < Pr - 1) xs[s] = ldc<COH>(g.X + (int64_t)(off + s) * ldx + rr);
            xk = pend_chain<COH>(xk, pre, g.X + rr, ldx, upl, PE - 1);
        } else {
#pragma unroll
            for (int s = 0; s < P - 1; ++s)
                if (s < Pr - 1) xk = __dsub_rn(xk, __dmul_rn(xs[s], ldc<COH>(g.Y + (int64_t)s * ldy + bq)));
        }
        if (leftorth) xk = xk / piv;
        L.xk[prow] = xk;
        const int rpos = rrow < m ? rpl : -1;  // (a row thread)
        if (q == 0 && rpos > k) {
            stc<COH>(g.X + (int64_t)(PE - 1) * ldx + rrow, xk);
            g.Lp[rrow + (int64_t)k * g.ldl] = xk;
        }
#pragma unroll
        for (int s = 0; s < P; ++s)
            if (s == Pr - 1) xs[s] = xk;
        // rows pivoted before this epoch (and rows past m): 0; pivoted at step rp of it: x_s for
        // s < rp - t0, then the pivot's own x (1, or the pivot when not leftorth), then 0
        const int dd = rpos > k ? Pr : (rpos >= t0 ? rpos - t0 : -1);
        double own = 0.0;
        if (!leftorth) {
            if constexpr (COH)
                own = rpos >= t0 && rpos <= k ? ep->pivot(pv, rpos) : 0.0;
            else
                own = rpos >= t0 && rpos <= k ? pv[rpos] : 0.0;
        } else {
            own = 1.0;
        }
        _Float16 sl[KS];
#pragma unroll
        for (int s = 0; s < P; ++s) {
            double x = s < dd ? xs[s] : (s == dd ? own : 0.0);
            if (s >= Pr) x = 0.0;  // (no-op for Pr == P)
            x = -(leftorth ? x : x * shs);
            f16_split(x, sl[3 * s], sl[3 * s + 2]);
            sl[3 * s + 1] = sl[3 * s];
        }
#pragma unroll
        for (int z = 3 * P; z < KS; ++z) sl[z] = (_Float16)0.0f;
        if constexpr (kShU8) sl[3 * P] = (_Float16)1.0f;  // the 8-bit codes' offset: 1 x (-128)
#pragma unroll
        for (int z = 0; z < KS / 8; ++z) {
            h8v w;
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = sl[8 * z + e];
            *reinterpret_cast<h8v*>(&L.u.xa[prow * KSP + 8 * z]) = w;
        }
    }
    // EXT: the first staged group's y_k chain here (whole stager waves; columns that are not
    // trailing compute a value nobody reads), so that pre is dead before the streaming loop
    [[maybe_unused]] double yk0 = 0.0;
    // (Requesting the first group's shadow-pending y's here too, with the chain's loads, would save
    // the staging's round trip for them, but holding them across the chain spills: 2 VGPRs at
    // P = 3, 4, 10-14 at P = 9, 10.)
    PPROFX(3);
    if constexpr (EXT) {
        if (stager) yk0 = pend_chain<COH>(a0, pre, g.Y + jj, ldy, upl, PE - 1);
    }
    PPROF(1);
    bool act = false;
#pragma unroll
    for (int b = 0; b < kMfBlk; ++b) act |= sb + 16 * (lcol >> 2) + 4 * b + (lcol & 3) < m && rpa[b] > k;
    [[maybe_unused]] unsigned tmask = 0;
    if constexpr (RF) {
#pragma unroll
        for (int i = 0; i < 16; ++i) tmask |= (rl + i < m && rpt[i] > k ? 1u : 0u) << i;
    }
    int cpst = (jst >= 0 && jst < n) ? cpl : -1;
    const bool wact = RF || __any(act);  // a refresh rewrites every row's shadow (non-trailing: 0)
    const float margin = 0x1p-20f;
    float tau = 0.0f;
    h8v af[kMfBlk][KSt];  // A fragments (registers for the whole pass)
    // chunk h: the lane's column's maximum |w| over its 16 rows and per 4-row block (-1: not a
    // trailing column)
    int g0r = 0;  // the staged group approx() works on (its columns, for the refresh stores)
    auto approx = [&](int h, int gcols, const ShVec (&v)[kShVecs], float (&mbs)[kMfBlk]) -> float {
        const int lc = h * 16 + lcol;
        const int cp = lc < gcols ? L.cpos[lc] : -1;
        h8v bf[KSt];
#pragma unroll
        for (int u = 0; u < KSt; ++u)
            bf[u] = *reinterpret_cast<const h8v*>(&L.yb[(lc < gcols ? lc : 0) * KSP + 32 * u + 8 * gq]);
        float c = 0.0f;
        [[maybe_unused]] h8v wout[2];
        [[maybe_unused]] u32x4v wq;
#pragma unroll
        for (int b = 0; b < kMfBlk; ++b) {
            f4v acc;
            if constexpr (kShU8) {
                // block b: rows 4 b .. 4 b + 3 = the bytes of dword b (v_cvt_f32_ubyte0..3); the offset
                // -128 comes from the MFMA's constant slot
                const uint32_t d = __builtin_bit_cast(u32x4v, v[0])[b];
                acc = f4v{(float)(d & 0xFFu), (float)((d >> 8) & 0xFFu), (float)((d >> 16) & 0xFFu), (float)(d >> 24)};
                if (!rload) acc = f4v{128.0f, 128.0f, 128.0f, 128.0f};  // rows past the shadow: W = 0
            } else {
                const h8v hv = __builtin_bit_cast(h8v, v[(b >> 1) % kShVecs]);
                const int o = 4 * (b & 1);
                acc = f4v{(float)hv[o], (float)hv[o + 1], (float)hv[o + 2], (float)hv[o + 3]};
                if (!rload) acc = f4v{0.0f, 0.0f, 0.0f, 0.0f};  // rows past the shadow: W = 0
            }
#pragma unroll
            for (int u = 0; u < KSt; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[b][u], bf[u], acc, 0, 0, 0);
            mbs[b] = __builtin_fmaxf(__builtin_fmaxf(fabsf(acc[0]), fabsf(acc[1])),
                                     __builtin_fmaxf(fabsf(acc[2]), fabsf(acc[3])));
            c = __builtin_fmaxf(c, mbs[b]);
            if constexpr (RF) {  // rows rl + 4 b + t: the new epoch's shadow, 0 off the trailing block
                if constexpr (kShU8) {
                    uint32_t q = 0;
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        q |= ((tmask >> (4 * b + t)) & 1u ? sh_u8(acc[t] * rscale) : kShU8Zero) << (8 * t);
                    wq[b] = q;
                } else {
                    const int o = 4 * (b & 1);
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        wout[b >> 1][o + t] = (tmask >> (4 * b + t)) & 1u ? (_Float16)(acc[t] * rscale) : (_Float16)0.0f;
                }
            }
        }
        if constexpr (RF) {  // buffer stores, dropped out of range: a fixed count per chunk
            const int j = lc < gcols ? col_of(g0r, lc) : n;
            const unsigned off =
                rload && j < n && cp > k ? (unsigned)(((int64_t)j * lds + rl) * (int64_t)sizeof(shT)) : 0xFFFFFFF0u;
            if constexpr (kShU8) {
                __builtin_amdgcn_raw_buffer_store_b128(wq, rsS0, (int)off, 0, 0);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, wout[0]), rsS0, (int)off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, wout[1]), rsS1, (int)off, 0, 0);
            }
        }
        if (cp <= k) {
#pragma unroll
            for (int b = 0; b < kMfBlk; ++b) mbs[b] = -1.0f;
            c = -1.0f;
        }
        return c;
    };
    // Exact examinations are deferred: blocks (4 rows of one column) that may hold the maximum
    // or a tie with it go to the wave's list in LDS, and the whole wave examines them together
    // -- one element per lane, all its loads in flight at once -- when the list fills and at the
    // end of each staged group, after pruning them against the latest bound tau.
    unsigned* const exl = L.u.e.ex + wave * kMfExCap;
    float* const exm = L.u.e.exm + wave * kMfExCap;
    int nex = 0;  // wave-uniform list length
    // FAST: all P - 1 pending x's of an element in flight at once (the final flush, when the
    // streaming registers are dead); otherwise one at a time (a full list mid-stream: rare)
    auto flush = [&](int g0, auto fast) {
        const float thr = tau - tau * margin;
        for (int e = lane; e < 4 * nex; e += 64) {
            const unsigned key = exl[e >> 2];
            if (exm[e >> 2] + eps < thr) continue;
            const int lc = (int)(key & 1023u), rq = (int)(key >> 10);
            const int r = sb + 4 * rq + (e & 3);
            if (r >= m) continue;
            const int j = col_of(g0, lc);
            double v = g.A[r + (int64_t)j * lda];
            const int rp = rowpos_of(r);
            // take v now: a load left in flight by the continue below (into a register the
            // streaming loop reuses) would cost a wait for every load at the loop's head
            asm volatile("" : "+v"(v));
            if (rp <= k) continue;
            if constexpr (decltype(fast)::value) {
                if constexpr (Gm::ymem) {
                    // x's and y's from memory, kExB pending updates in flight at a time (the
                    // streaming registers are dead here): at PE = 30 two round trips, not eight
                    for (int s0 = 0; s0 < PE - 1; s0 += kExB) {
                        double xv[kExB], yv[kExB];
#pragma unroll
                        for (int i = 0; i < kExB; ++i)
                            if (s0 + i < PE - 1) {
                                xv[i] = ldc<COH>(g.X + (int64_t)(s0 + i) * ldx + r);
                                yv[i] = ldc<COH>(g.Y + (int64_t)(s0 + i) * ldy + j);
                            }
#pragma unroll
                        for (int i = 0; i < kExB; ++i)
                            if (s0 + i < PE - 1) v = __dsub_rn(v, __dmul_rn(xv[i], yv[i]));
                    }
                } else {
                    double xv[P];
#pragma unroll
                    for (int s = 0; s < P - 1; ++s)
                        if (s < Pr - 1) xv[s] = ldc<COH>(g.X + (int64_t)s * ldx + r);
#pragma unroll
                    for (int s = 0; s < P - 1; ++s)
                        if (s < Pr - 1) v = __dsub_rn(v, __dmul_rn(xv[s], L.ys[lc * P + s]));
                }
            } else {
#pragma unroll 1
                for (int s = 0; s < PE - 1; ++s)
                    v = __dsub_rn(v, __dmul_rn(ldc<COH>(g.X + (int64_t)s * ldx + r),
                                               Gm::ymem ? ldc<COH>(g.Y + (int64_t)s * ldy + j) : L.ys[lc * P + s]));
            }
            v = __dsub_rn(v, __dmul_rn(L.xk[r - tb], L.ys[lc * Gm::YS + Gm::YS - 1]));
            const double a2 = __dmul_rn(v, v);
            if (a2 >= best.v) cand_take(best, CandR{a2, v, L.cpos[lc], rp, j, r});
#if TCI_PASS_PROF
            atomicAdd(&g_exam_lds, 1u);
#endif
        }
        nex = 0;
    };
    // append the lane's blocks whose maximum reaches bound (chunk h); flushes first if needed
    auto append = [&](int g0, int h, const float (&mbs)[kMfBlk], float bound) {
        const unsigned lc = (unsigned)(h * 16 + lcol);
#pragma unroll
        for (int b = 0; b < kMfBlk; ++b) {
            const bool f = mbs[b] >= 0.0f && mbs[b] + eps >= bound;
            const uint64_t bal = __ballot(f);
            if (bal == 0) continue;
            const int cnt = __popcll(bal);
            if (nex + cnt > kMfExCap) flush(g0, std::false_type{});
            if (f) {
                const int at = nex + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                exl[at] = lc | (unsigned)(4 * gq + b) << 10;
                exm[at] = mbs[b];
            }
            nex += cnt;
        }
    };
    auto test = [&](float c) {
        if (c < 0.0f) return;
        const float lb = fmaxf(c - eps, 0.0f);
        const float ts = __uint_as_float(__hip_atomic_load(&L.tau, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        tau = fmaxf(tau, ts);
        if (lb > tau) {
            tau = lb;
            atomicMax(&L.tau, __float_as_uint(lb));
        }
    };
    for (int g0 = 0; g0 < ntc; g0 += G) {
        const int gn = min(G, ntc - g0);
        const int gcols = gn * cb;
        const int nch = (gcols + 15) / 16;
        g0r = g0;
        if (g0 > 0) {
            jst = stage_col(g0);
            if constexpr (COH)
                cpst = jst >= 0 ? ep->lcol[lcol_of(g0, tx)] : -1;
            else
                cpst = (jst >= 0 && jst < n) ? colpos[jst] : -1;
            // unconditional (an inactive wave loads two chunks it never reads): loads skipped on
            // some paths into the loop would make its head wait for every load in flight
            load_chunk(g0, gcols, min(rep, nch - 1), va);
            load_chunk(g0, gcols, min(rep + kMfReps, nch - 1), vb);
            __syncthreads();
        }
        [[maybe_unused]] double ykg = yk0;  // EXT: this group's y_k chain (whole stager waves)
        if constexpr (EXT) {
            if (g0 > 0 && stager) {
                const int jj = jst >= 0 && jst < n ? jst : 0;
                PendPre pg;
                pend_pre<COH>(pg, g.Y + jj, ldy, PE - 1);
                ykg = pend_chain<COH>(g.A[a + (int64_t)jj * lda], pg, g.Y + jj, ldy, upl, PE - 1);
            }
        }
        if (jst >= 0) {
            int lc = tx;
            asm volatile("" : "+v"(lc));
            L.cpos[lc] = cpst;
            if (cpst > k) {
                double ysv[P];
#pragma unroll
                for (int s = 0; s < P - 1; ++s)
                    if (s < Pr - 1) ysv[s] = ldc<COH>(g.Y + (int64_t)(off + s) * ldy + jst);
                // (taking them from pre's registers -- they are slots off .. PE - 2 of the column
                // pre holds -- by a select per slot spills 16-80 VGPRs: pre would stay live here)
                double yk;
                if constexpr (EXT) {
                    yk = ykg;
                } else {
                    yk = g.A[a + (int64_t)jst * lda];
#pragma unroll
                    for (int s = 0; s < P - 1; ++s)
                        if (s < Pr - 1) yk = __dsub_rn(yk, __dmul_rn(ldc<COH>(g.X + (int64_t)s * ldx + a), ysv[s]));
                }
                if (!leftorth) yk = yk / piv;
#pragma unroll
                for (int s = 0; s < P; ++s)
                    if (s == Pr - 1) ysv[s] = yk;
                if (tr == 0) {
                    stc<COH>(g.Y + (int64_t)(PE - 1) * ldy + jst, yk);
                    g.Up[k + (int64_t)jst * g.ldu] = yk;
                }
                // B fragment: slots (yh_s, yl_s, yh_s) for s < P, zero after
                _Float16 sl[KS];
                L.ys[lc * Gm::YS + Gm::YS - 1] = yk;
#pragma unroll
                for (int s = 0; s < P; ++s) {
                    if (s < Pr) {
                        if constexpr (!Gm::ymem) L.ys[lc * P + s] = ysv[s];
                        f16_split(leftorth ? ysv[s] * shs : ysv[s], sl[3 * s], sl[3 * s + 1]);
                    } else {  // (Pr < P: the persistent epoch kernel)
                        sl[3 * s] = sl[3 * s + 1] = (_Float16)0.0f;
                    }
                    sl[3 * s + 2] = sl[3 * s];
                }
#pragma unroll
                for (int z = 3 * P; z < KS; ++z) sl[z] = (_Float16)0.0f;
                if constexpr (kShU8) sl[3 * P] = (_Float16)-128.0f;  // the 8-bit codes' offset
#pragma unroll
                for (int z = 0; z < KS / 8; ++z) {
                    h8v w;
#pragma unroll
                    for (int e = 0; e < 8; ++e) w[e] = sl[8 * z + e];
                    *reinterpret_cast<h8v*>(&L.yb[lc * KSP + 8 * z]) = w;
                }
            }
        }
        if (g0 == 0) PPROF(7);
        if (tx < kMfSlices) L.cnt[tx] = 2 * kMfReps;
        if (g0 == 0 && tx == 0) L.tau = 0u;
        __syncthreads();
        if (g0 == 0) {
#pragma unroll
            for (int b = 0; b < kMfBlk; ++b) {
                const int pr = slice * kMfRows + 16 * (lcol >> 2) + 4 * b + (lcol & 3);
#pragma unroll
                for (int u = 0; u < KSt; ++u)
                    af[b][u] = *reinterpret_cast<const h8v*>(&L.u.xa[pr * KSP + 32 * u + 8 * gq]);
            }
            PPROF(2);
        }
        auto grab = [&]() -> int {  // wave-uniform (an SGPR): the loop's branches stay scalar
            int h = 0;
            if (lane == 0) h = atomicAdd(&L.cnt[slice], 1);
            return __builtin_amdgcn_readfirstlane(h);
        };
        int h0 = rep, h1 = rep + kMfReps;
        float mb0[kMfBlk], mb1[kMfBlk];
        if (g0 == 0) {
            // seed: the first two chunks of every wave set the workgroup's bound first
            float c0 = -1.0f, c1 = -1.0f;
            const int e0 = h0, e1 = h1;
#pragma unroll
            for (int b = 0; b < kMfBlk; ++b) mb0[b] = mb1[b] = -1.0f;
            // approx() of a chunk past the group is inert (-1, no stores). The grabs and loads run
            // in inactive waves too (a slice's waves share its rows, so they are all inactive and
            // take nothing from an active one): loads skipped on the way into the loop below would
            // make its head wait for every load in flight.
            if (wact) c0 = approx(h0, gcols, va, mb0);
            h0 = grab();
            load_chunk(g0, gcols, min(h0, nch - 1), va);
            if (wact && (RF || EXT || h1 < nch)) c1 = approx(h1, gcols, vb, mb1);
            h1 = grab();
            load_chunk(g0, gcols, min(h1, nch - 1), vb);
            if (wact) {
                float lb = fmaxf(fmaxf(c0, c1) - eps, 0.0f);
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) lb = fmaxf(lb, __shfl_xor(lb, off));
                if (lane == 0) atomicMax(&L.tau, __float_as_uint(lb));
            }
            __syncthreads();
            if (!wact) continue;
            tau = __uint_as_float(L.tau);
            const float bound = tau - tau * margin;
            if (e0 < nch) append(g0, e0, mb0, bound);
            if (e1 < nch) append(g0, e1, mb1, bound);
        } else if (!wact) {
            continue;
        }
        // h0's values in va, h1's in vb; every grab returns a larger index than both, so h1 >= nch
        // only in the last trip. Both halves issue their loads unconditionally: a fixed number of
        // loads per trip lets each chunk's wait count the other chunk's loads (a skipped half
        // would force a wait for every outstanding load). The last trip's h1 >= nch skips its
        // approx() (no loads) in the first-epoch passes: at small sizes (where those are the only
        // read-only passes) a wave streams one or two chunks, and the dead half would double its
        // work. A refresh keeps it, inert, for its fixed count of stores, and the EXT passes too
        // (skipping it there changes their register allocation: prologue spills).
        while (h0 < nch) {
            {
                const float c = approx(h0, gcols, va, mb0);
                const int e = h0;
                h0 = grab();
                load_chunk(g0, gcols, min(h0, nch - 1), va);
                test(c);
                append(g0, e, mb0, tau - tau * margin);
            }
            {
                const int e = h1;
                float c = -1.0f;
                if (RF || EXT || e < nch) c = approx(e, gcols, vb, mb1);
                h1 = grab();
                load_chunk(g0, gcols, min(h1, nch - 1), vb);
                if (RF || EXT || e < nch) {  // (inert past the group: c and mb1 are -1)
                    test(c);
                    append(g0, e, mb1, tau - tau * margin);
                }
            }
        }
        // the latest bound of the workgroup prunes the list
        tau = fmaxf(tau, __uint_as_float(__hip_atomic_load(&L.tau, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
        flush(g0, std::true_type{});
    }
    return kMfDone;
}

// ------------------------------------------------------------------ deep exact pass (two-level epoch)
// The exact body for up to kMaxPendR pending updates: P (= g.pe, runtime) x's per row do not fit
// the registers of k_pass2 (which spills from P = 13), so the tile's x's live in LDS, [s][row], and
// the tile is processed in two 256-row halves (64 KiB of x's each); the staged columns' y's are in
// LDS too, [s][column], 128 columns per group. Per element the reference's arithmetic in its order,
// v = v - x_s[i] * y_s[j] for s = 0 .. P-1 (separate multiply and subtract): bitwise k_pass2's
// values. MODE 0: read only (the exact fallback of a read pass whose shadow bound is not tight);
// 1: write-back of the fp64 values and the fp16 shadow of the new epoch (as k_pass2<P,true,true>);
// 2: the shadow only (a refresh whose MFMA bound is not tight: the new epoch's shadow is then exact
// again, which the bound recursion of k_pass_mf knows -- it re-derives every past decision). Same
// grid, tiles, candidates and tail as k_pass2, so it also serves as k_pass_mf's fallback body.
constexpr int kXHalf = 256;   // rows whose x's are in LDS at a time
#ifndef TCI_XSTAGE
#define TCI_XSTAGE 128
#endif
#ifndef TCI_PX_EXP
#define TCI_PX_EXP 0  // A/B timing probes of the deep write-back's LDS traffic (1: x, 2: y, 3: both); 0 in builds
#endif
constexpr int kXStage = TCI_XSTAGE;  // staged columns per group
#ifndef TCI_PX_DRAIN
#define TCI_PX_DRAIN 1  // deep write-back: explicit drain, then the next chunk's loads, then the arithmetic (0: round-3 order)
#endif
#ifndef TCI_XU
#define TCI_XU 4
#endif
constexpr int kXU = TCI_XU;   // columns per chunk (two chunks in flight per lane); 4 or 8
static_assert(kXU == 4 || kXU == 8, "chunks of 4 or 8 columns (cb is a multiple of 8)");
constexpr int kXSlices = kXHalf / 128;
constexpr int kXReps = kP2Threads / 64 / kXSlices;
// Geometry of the deep exact body by workgroup size: NT = 1024 (one workgroup per CU, 512-row
// tiles in two 256-row halves: also the fallback body of k_pass_mf) or NT = 512 for the write-back
// launch (two workgroups per CU, 256-row tiles in two 128-row halves, 64 KiB of LDS each: one
// workgroup's staging and y_k chains overlap the other's streaming)
template <int NT>
struct PxGeom {
    static constexpr int Half = NT == 1024 ? 256 : 128;  // rows whose x's are in LDS at a time
    static constexpr int Tile = 2 * Half;                // rows of a workgroup's tile
    static constexpr int Slices = Half / 128;
    static constexpr int Reps = NT / 64 / Slices;
};
// (16-B aligned: the update loop reads a lane's two x's and two y's with one ds_read_b128 each -- as
// ds_read2_b64 pairs at a 16-B lane stride the x reads were 4-way bank conflicts, and the loop was
// LDS-bound: round 4's 31.5 M conflict cycles per deep write-back)
template <int NT>
struct alignas(16) PxLdsT {
    alignas(16) double xs[kMaxPendR * PxGeom<NT>::Half];  // x_s of the half-tile's rows
    alignas(16) double ys[kMaxPendR * kXStage];          // y_s of the staged columns
    double xa[kMaxPendR];            // X[s][a] (pivot row a)
    double yb[kMaxPendR];            // Y[s][b] (pivot column b)
    int cpos[kXStage];
    int cnt[PxGeom<NT>::Slices];
};
using PxLds = PxLdsT<kP2Threads>;

template <int MODE, bool COH = false, int NT = kP2Threads>
__device__ __forceinline__ bool passx_body(const PassK& g, const SelArgs& sel, PxLdsT<NT>& L, CandR& best,
                                           unsigned long long (&pt)[8]) {
    constexpr int kXHalf = PxGeom<NT>::Half, kXSlices = PxGeom<NT>::Slices, kXReps = PxGeom<NT>::Reps;
    constexpr int kRowsPerTile = PxGeom<NT>::Tile, kP2Threads = NT;
    RrluState* st = sel.st;
    const int32_t* rowpos = sel.rowpos;
    const int32_t* colpos = sel.colpos;
    double* __restrict__ A = g.A;
    const int64_t lda = g.lda, ldx = g.ldx, ldy = g.ldy;
    const int m = g.m, n = g.n, k = g.k, cb = g.cb, rev = g.rev, leftorth = g.leftorth;
    const int P = g.pe;  // 1 .. kMaxPendR
    // the wave index is uniform: kept in SGPRs, so the chunk (from the slice's counter, read back
    // with readfirstlane) and with it every column index and column pointer of the streaming loop
    // is scalar work -- per column the loop's VALU does the arithmetic and a 32-bit row offset only
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slice = wave % kXSlices, rep = wave / kXSlices;
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile;
    const int tiles_c = (n + cb - 1) / cb;
    const int nq = gridDim.x / tiles_r;
    const int wid = xcd_spread(blockIdx.x, gridDim.x);
    const int tr = wid % tiles_r;
    const int q = rev ? nq - 1 - wid / tiles_r : wid / tiles_r;
    const int ntc = q < tiles_c ? (tiles_c - 1 - q) / nq + 1 : 0;
    const int G = kXStage / cb;
    const int cbs = __builtin_ctz(cb);
    auto col_of = [&](int g0, int lc) -> int {
        const int it = g0 + (lc >> cbs);
        return ((q + (rev ? ntc - 1 - it : it) * nq) << cbs) + (lc & (cb - 1));
    };
    if (st->done) return false;
    const int a = (int)st->p, b = (int)st->q;
    const double piv = st->pval;
    // the pivot row's pending x's and the pivot column's pending y's (same for every thread)
    if (threadIdx.x < P - 1) {
        L.xa[threadIdx.x] = g.X[(int64_t)threadIdx.x * ldx + a];
        L.yb[threadIdx.x] = g.Y[(int64_t)threadIdx.x * ldy + b];
    }
    [[maybe_unused]] const double shs = MODE ? sh_scale(sh_bound(sel.pivvals, k + 1)) : 1.0;
    PPROF(1);
    for (int half = 0; half < kRowsPerTile / kXHalf; ++half) {
        const int hb = tr * kRowsPerTile + half * kXHalf;  // first row of the half
        if (hb >= m) break;
        __syncthreads();  // the previous half's readers are done with xs / ys
        {  // the half's pending x's, all of a thread's loads in flight at once
            constexpr int kPer = kMaxPendR * kXHalf / kP2Threads;  // 8
            double v[kPer];
#pragma unroll
            for (int u = 0; u < kPer; ++u) {  // unconditional loads (slot < kMaxPendR, row clamped),
                // masked after: a load inside the condition became a branch + wait each (serial)
                const int e = threadIdx.x + u * kP2Threads, s = e / kXHalf, rr = e - s * kXHalf;
                v[u] = g.X[(int64_t)s * ldx + min(hb + rr, m - 1)];
                if (!(s < P - 1 && hb + rr < m)) v[u] = 0.0;
            }
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int e = threadIdx.x + u * kP2Threads;
                if (e < (P - 1) * kXHalf) L.xs[e] = v[u];
            }
        }
        __syncthreads();
        if (threadIdx.x < kXHalf) {  // x_k of the half's rows (pivot k's column, updates applied)
            const int rr = threadIdx.x, r = hb + rr;
            double xk = 0.0;
            if (r < m) {
                xk = A[r + (int64_t)b * lda];
                for (int s = 0; s < P - 1; ++s) xk = __dsub_rn(xk, __dmul_rn(L.xs[s * kXHalf + rr], L.yb[s]));
                if (leftorth) xk = xk / piv;
                if (q == 0 && rowpos[r] > k) {
                    stc<COH>(g.X + (int64_t)(P - 1) * ldx + r, xk);
                    g.Lp[r + (int64_t)k * g.ldl] = xk;
                }
            }
            L.xs[(P - 1) * kXHalf + rr] = xk;
        }
        const int lr = slice * 128 + 2 * lane;  // the lane's first row within the half
        const int r0 = hb + lr;
        const bool rowok = r0 < m, pair = r0 + 1 < m;
        const int rp0 = rowok ? rowpos[r0] : -1, rp1 = pair ? rowpos[r0 + 1] : -1;
        const bool in0 = rp0 > k, in1 = rp1 > k;
        const bool wact = MODE != 0 || __any(in0 || in1);
        const uint32_t roff = rowok ? r0 : 0;  // the lane's row offset within a column
        for (int g0 = 0; g0 < ntc; g0 += G) {
            const int gcols = min(G, ntc - g0) * cb;
            const int nch = gcols / kXU;
            if (g0 > 0) __syncthreads();  // the previous group's readers are done with ys / cpos
            // staging in two steps: every thread loads a share of the group's pending y's into LDS
            // (all in flight at once), then one thread per column runs y_k's sequential chain from
            // LDS (the reference's order)
            {
                constexpr int kPer = kMaxPendR * kXStage / kP2Threads;  // 4
                const int lc = threadIdx.x & (kXStage - 1), s0 = threadIdx.x / kXStage;
                const int j = lc < gcols ? col_of(g0, lc) : 0;
                double v[kPer];
#pragma unroll
                for (int u = 0; u < kPer; ++u) {  // unconditional (slot < kMaxPendR), masked after
                    const int s = s0 + u * (kP2Threads / kXStage);
                    v[u] = g.Y[(int64_t)s * ldy + j];
                    if (!(s < P - 1 && lc < gcols)) v[u] = 0.0;
                }
#pragma unroll
                for (int u = 0; u < kPer; ++u) {
                    const int s = s0 + u * (kP2Threads / kXStage);
                    if (s < P - 1) L.ys[s * kXStage + lc] = v[u];
                }
            }
            const int lcs = threadIdx.x, js = lcs < gcols ? col_of(g0, lcs) : 0;
            const int cps = (lcs < gcols && js < n) ? colpos[js] : -1;
            const double ypr = (lcs < gcols && cps > k) ? A[a + (int64_t)js * lda] : 0.0;
            __syncthreads();
            if (lcs < gcols) {
                L.cpos[lcs] = cps;
                if (cps > k) {
                    double yk = ypr;
                    for (int s = 0; s < P - 1; ++s) yk = __dsub_rn(yk, __dmul_rn(L.xa[s], L.ys[s * kXStage + lcs]));
                    if (!leftorth) yk = yk / piv;
                    L.ys[(P - 1) * kXStage + lcs] = yk;
                    if (tr == 0 && half == 0) {
                        stc<COH>(g.Y + (int64_t)(P - 1) * ldy + js, yk);
                        g.Up[k + (int64_t)js * g.ldu] = yk;
                    }
                }
            }
            if (threadIdx.x < kXSlices) L.cnt[threadIdx.x] = 2 * kXReps;
            __syncthreads();
            if (g0 == 0 && half == 0) PPROF(2);
            if (!wact) continue;
            // a chunk is kXU consecutive columns of one column tile (kXU divides cb): one scalar
            // column index per chunk, the column pointers scalar (SGPR base + the lane's row offset)
            auto load_chunk = [&](int h, double2 (&v)[kXU]) {
                const int j0 = col_of(g0, h * kXU);
#pragma unroll
                for (int u = 0; u < kXU; ++u) {
                    const double* colp = A + (int64_t)min(j0 + u, n - 1) * lda;
                    const double2* pa = reinterpret_cast<const double2*>(colp + roff);
                    if constexpr (MODE == 1 && TCI_FLUSH_NTL) {
                        typedef double dv2 __attribute__((ext_vector_type(2)));
                        const dv2 w = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(pa));
                        v[u] = double2{w.x, w.y};
                    } else {
                        v[u] = *pa;
                    }
                }
            };
            auto process = [&](int h, double2 (&v)[kXU]) {
                int cp[kXU];
                bool any = false;
#pragma unroll
                for (int u = 0; u < kXU; ++u) {
                    cp[u] = __builtin_amdgcn_readfirstlane(L.cpos[h * kXU + u]);
                    any |= cp[u] > k;
                }
                if (!any) return;
                const int j0 = col_of(g0, h * kXU);
#pragma unroll 2
                for (int s = 0; s < P; ++s) {
#if TCI_PX_EXP & 1  // timing experiment only (wrong values): no LDS read of the x's
                    const dv2 x = dv2{1.0 + s, 0.5 * s};
#else
                    const dv2 x = *reinterpret_cast<const dv2*>(
                        __builtin_assume_aligned(&L.xs[s * kXHalf + lr], 16));
#endif
                    double y[kXU];
#pragma unroll
                    for (int u = 0; u < kXU; u += 2) {
#if TCI_PX_EXP & 2  // timing experiment only: no LDS read of the y's
                        const dv2 yy = dv2{0.25 * s + u, 0.125 * s};
#else
                        const dv2 yy = *reinterpret_cast<const dv2*>(
                            __builtin_assume_aligned(&L.ys[s * kXStage + h * kXU + u], 16));
#endif
                        y[u] = yy.x;
                        y[u + 1] = yy.y;
                    }
#pragma unroll
                    for (int u = 0; u < kXU; ++u) {
                        v[u].x = __dsub_rn(v[u].x, __dmul_rn(x.x, y[u]));
                        v[u].y = __dsub_rn(v[u].y, __dmul_rn(x.y, y[u]));
                    }
                }
                // the chunk's largest |value| of the lane's trailing elements (0 for the others;
                // NaN never wins a candidate test, and fmax drops it): if its square does not reach
                // the lane's best, no element of the chunk does (x -> x*x is monotone under
                // rounding), and the per-element tests are skipped
                double mx0 = 0.0, mx1 = 0.0;  // (maxnum of subtraction results: one v_max_f64 each)
#pragma unroll
                for (int u = 0; u < kXU; ++u) {
                    if (cp[u] <= k) continue;
                    const int j = j0 + u;
                    if constexpr (MODE == 1) {  // trailing rows only (see k_pass2's write-back)
                        if (in0 || in1) {
                            double2* pa = reinterpret_cast<double2*>(A + (int64_t)j * lda + roff);
                            if (!in1) {
                                pa->x = v[u].x;
                            } else if (!in0) {
                                pa->y = v[u].y;
                            } else {
                                typedef double dv2 __attribute__((ext_vector_type(2)));
                                dv2 w = {v[u].x, v[u].y};
                                __builtin_nontemporal_store(w, reinterpret_cast<dv2*>(pa));
                            }
                        }
                    }
                    if constexpr (MODE != 0 && kShU8) {
                        if (rowok) {
                            uint8_t* ps = reinterpret_cast<uint8_t*>(g.S) + (int64_t)j * g.lds + roff;
                            const uint32_t c0 = in0 ? sh_u8((float)(v[u].x * shs)) : kShU8Zero;
                            if (pair)
                                *reinterpret_cast<uint16_t*>(ps) =
                                    (uint16_t)(c0 | (in1 ? sh_u8((float)(v[u].y * shs)) : kShU8Zero) << 8);
                            else
                                ps[0] = (uint8_t)c0;
                        }
                    } else if constexpr (MODE != 0 && kShHalf) {
                        if (rowok) {
                            _Float16* ps = reinterpret_cast<_Float16*>(g.S) + (int64_t)j * g.lds + roff;
                            const _Float16 h0 = in0 ? (_Float16)(float)(v[u].x * shs) : (_Float16)0.0f;
                            if (pair) {
                                typedef _Float16 h2v __attribute__((ext_vector_type(2)));
                                *reinterpret_cast<h2v*>(ps) = h2v{h0, in1 ? (_Float16)(float)(v[u].y * shs) : (_Float16)0.0f};
                            } else {
                                ps[0] = h0;
                            }
                        }
                    }
                    mx0 = fmax(mx0, fabs(v[u].x));
                    mx1 = fmax(mx1, fabs(v[u].y));
                }
                const double mx = fmax(in0 ? mx0 : 0.0, in1 ? mx1 : 0.0);
                if (__dmul_rn(mx, mx) >= best.v) {
#pragma unroll
                    for (int u = 0; u < kXU; ++u) {
                        if (cp[u] <= k) continue;
                        const int j = j0 + u;
                        const double a0 = __dmul_rn(v[u].x, v[u].x), a1 = __dmul_rn(v[u].y, v[u].y);
                        if ((in0 && a0 >= best.v) || (in1 && a1 >= best.v)) {
                            if (in0) cand_take(best, CandR{a0, v[u].x, cp[u], rp0, j, r0});
                            if (in1) cand_take(best, CandR{a1, v[u].y, cp[u], rp1, j, r0 + 1});
                        }
                    }
                }
            };
            auto grab = [&]() -> int {
                int h = 0;
                if (lane == 0) h = atomicAdd(&L.cnt[slice], 1);
                return __builtin_amdgcn_readfirstlane(h);  // every lane active here: lane 0's ticket
            };
            double2 va[kXU], vb[kXU];
            int h0 = rep, h1 = rep + kXReps;
#if TCI_PX_DRAIN
            // with the write-back's stores in flight the compiler cannot count loads precisely
            // (loads and stores share vmcnt), so every use of a chunk waited for vmcnt(0) -- for the
            // chunk just requested too. Drain explicitly first, then request the next chunk, then
            // process this one: the request overlaps one chunk of arithmetic
            if (h0 < nch) load_chunk(h0, va);
            while (h0 < nch) {
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): va landed, earlier stores done
                if (h1 < nch) load_chunk(h1, vb);
                process(h0, va);
                if (h1 >= nch) break;
                h0 = grab();
                __builtin_amdgcn_s_waitcnt(0x0f70);
                if (h0 < nch) load_chunk(h0, va);
                process(h1, vb);
                h1 = grab();
            }
#else
            if (h0 < nch) load_chunk(h0, va);
            if (h1 < nch) load_chunk(h1, vb);
            while (h0 < nch) {
                process(h0, va);
                h0 = grab();
                if (h0 < nch) load_chunk(h0, va);
                if (h1 >= nch) break;
                process(h1, vb);
                h1 = grab();
                if (h1 < nch) load_chunk(h1, vb);
            }
#endif
        }
    }
    return true;
}

template <int MODE, int NT = kP2Threads>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_pass_x(PassK g, SelArgs sel) {
    __shared__ PxLdsT<NT> L;
    [[maybe_unused]] unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    PPROF(0);
    CandR best = cand_none();
    if (!passx_body<MODE, false, NT>(g, sel, L, best, pt)) return;
    PPROF(3);
    pass_tail<NT>(best, sel, g.cand, pt, g.m, g.pe, MODE);
}

// RT: one instance for every shadow-pending count (P its bound, g.ps the count): the EXT passes of
// all depths then run the same code, which stays in the instruction cache from pass to pass
template <int P, bool EXT, bool RF, bool RT = false>
__global__ __launch_bounds__(kP2Threads) void k_pass_mf(PassK g, SelArgs sel) {
    __shared__ union {
        P2Lds<P> x;
        P2MfLds<P, EXT> f;
        typename std::conditional<(EXT || RF), PxLds, char>::type px;
    } L;
    [[maybe_unused]] unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    PPROF(0);
#if TCI_PASS_PROF
    if (threadIdx.x == 0) g_exam_lds = 0;  // (read after the body's barriers)
#endif
    CandR best = cand_none();
    const int r = pass_mf_body<P, EXT, RF>(g, sel, L.f, best, pt, RT ? g.ps : P);
    bool go = r == kMfDone;
#if TCI_PASS_PROF
    if (r == kMfExact && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_cert_fails, 1u);
    if (r != kMfDone && threadIdx.x == 0) g_exam_lds = 0;  // (the exact bodies examine everything)
#endif
    if (r == kMfExact) {  // uniform: every workgroup derives the same certificate
        if constexpr (RF)
            go = passx_body<2>(g, sel, L.px, best, pt);
        else if constexpr (EXT)
            go = passx_body<0>(g, sel, L.px, best, pt);
        else
            go = pass2_body<P, false, false>(g, sel, L.x, best, pt);
    }
    if (!go) return;
    PPROF(3);
    pass_tail<kP2Threads>(best, sel, g.cand, pt, g.m, P, RF ? 2 : 0);
}

// ------------------------------------------------------------------ persistent shadow epoch
// The read-only passes of one shadow epoch (passes k0 .. k0 + npass - 1, shadow-pending counts
// ps0 .. ps0 + npass - 1 <= kEpochMaxP) in ONE launch: the grid stays resident (one 1024-thread
// workgroup per CU, as the per-pass launches) and no pass ends in a kernel boundary. The pass body is
// k_pass_mf's (pass_mf_body, COH); between two passes (_optimizerrlu!'s loop, matrixlu.jl:356-369):
//   * every wave drains its stores (the X / Y slots of x_k, y_k), the workgroup publishes its candidate
//     (sc1) and adds to the launch's ticket (monotonic: pass i is complete at (i + 1) G);
//   * EVERY workgroup polls the ticket until pass i is complete, reads all G candidates (sc1) and
//     reduces them itself -- the same winner everywhere (cand_better is a strict total order) -- runs
//     the stop test (matrixlu.jl:359-368) and applies the swaps (addpivot!'s swaprow! / swapcol!,
//     :254-275) to its LDS copies of the positions of its rows and columns: no committing workgroup,
//     no flag, no state read back (MI355X_MICROARCH.md hand-off table, first row: sc1 stores drained
//     before the ticket add, sc1 loads after the poll);
//   * the global state is written, stores only, by the workgroups that hold it: the row swap by the
//     q = 0 workgroup of each row tile (the threads that own the two rows), the column swap by the
//     tr = 0 workgroup owning each column, the pivot value and rrLU state by workgroup 0. Nothing in
//     the launch reads them back; the next launch does. They are sc1 (write-through) stores: a
//     position's entry (rowphys[K]) is written by different workgroups in different passes, and
//     plain stores would reach memory in the order the XCD L2s write back at the kernel's end.
// Co-residency is not assumed: a workgroup that waits longer than `timeout` ticks (100 MHz) marks the
// ticket ABORT by a compare-and-swap that succeeds only while the count is short, so either every
// workgroup sees the count complete or every one sees ABORT; the aborting one sets st->done = 2 and
// every later pass launch returns at once. Nothing is selected for the aborted pass, so the host
// resumes with per-pass launches at pass st->np - 1 (every pass write is idempotent). A certificate
// that fails (uniform) or an all-NaN trailing block ends the launch the same way with st->done = 3.
constexpr int kEpochMaxCols = 15360;  // columns per workgroup the LDS column map holds (int16 positions)
#if TCI_EPOCH_GRID
constexpr unsigned kEpochAbort = 0x80000000u;

// thread 0: wait until `target` arrivals. 1: complete, 0: abort
__device__ __forceinline__ int epoch_wait(unsigned* ticket, unsigned target, long long timeout, RrluState* st) {
    long long t0 = (long long)wall_clock64();
    for (;;) {
        unsigned tv = ldc<true>(ticket);
        if (tv & kEpochAbort) return 0;
        if (tv >= target) return 1;
        if ((long long)wall_clock64() - t0 > timeout) {
            // a workgroup is missing (not co-resident) -- or slow: abort only while the count is short
            while (!(tv & kEpochAbort) && tv < target) {
                if (__hip_atomic_compare_exchange_strong((gptr<unsigned>)ticket, &tv, tv | kEpochAbort, __ATOMIC_RELAXED,
                                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    stc<true>(&st->done, 2);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    return 0;
                }
            }
            return (tv & kEpochAbort) ? 0 : 1;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

struct EpochArgs {
    int npass;         // read-only passes in this launch (k = g.k .. g.k + npass - 1)
    int serp;          // serpentine order: pass k walks backwards when (k + 1) is odd
    unsigned* sync;    // this launch's ticket, zero at launch
    long long timeout; // ticks a workgroup waits for the others before it gives up (abort)
};

template <bool EXT>
__global__ __launch_bounds__(kP2Threads) void k_pass_mf_epoch(PassK g0, SelArgs sel0, EpochArgs e) {
    __shared__ __attribute__((aligned(16))) char lds[sizeof(P2MfLds<kEpochMaxP, EXT>)];
    __shared__ int32_t lrow[kRowsPerTile];
    __shared__ int16_t lcol[kEpochMaxCols];
    __shared__ double lpiv[kEpochMaxP];
    __shared__ int s_go;
    __shared__ CandR s_w;
    [[maybe_unused]] unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned G = gridDim.x;
    RrluState* const st = sel0.st;
    // a launch enqueued after the factorisation stopped (or after an earlier persistent launch ended
    // early, st->done = 2 / 3: the host resumes before this launch's passes) does nothing
    if (st->done) return;
    // geometry of the workgroup's rows and columns (the body's, with the column set fixed: q)
    const int m = g0.m, n = g0.n, cb = g0.cb, cbs = __builtin_ctz(g0.cb);
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile, tiles_c = (n + cb - 1) / cb;
    const int nq = (int)G / tiles_r;
    const int wid = xcd_spread(blockIdx.x, G);
    const int tr = wid % tiles_r, q = wid / tiles_r, tb = tr * kRowsPerTile;
    const int ntc = q < tiles_c ? (tiles_c - 1 - q) / nq + 1 : 0;
    const int ncols = ntc * cb;  // <= kEpochMaxCols (host)
    // the maps as the previous launch left them (plain loads: written before this launch)
    for (int t = threadIdx.x; t < kRowsPerTile; t += kP2Threads) lrow[t] = tb + t < m ? sel0.rowpos[tb + t] : -1;
    for (int x = threadIdx.x; x < ncols; x += kP2Threads) {
        const int j = ((q + (x >> cbs) * nq) << cbs) + (x & (cb - 1));
        lcol[x] = (int16_t)(j < n ? sel0.colpos[j] : -1);
    }
    EpochIn ein{(int)st->p, (int)st->q, st->pval, lrow, lcol, lpiv, g0.k};
    double maxerror = st->maxerror;
    __syncthreads();
    for (int i = 0; i < e.npass; ++i) {
        PassK g = g0;
        SelArgs sel = sel0;
        g.k = g0.k + i;
        g.ps = g0.ps + i;
        g.pe = g0.pe + i;
        g.rev = e.serp ? ((g.k + 1) & 1) : 0;
        const int K = g.k + 1;  // the pivot this pass selects (the host never puts the last pass here)
        sel.selk = K;
        CandR best = cand_none();
        const int r = pass_mf_body<kEpochMaxP, EXT, false, true>(g, sel, *reinterpret_cast<P2MfLds<kEpochMaxP, EXT>*>(lds),
                                                                 best, pt, g.ps, &ein);
        if (r != kMfDone) {
            // the certificate failed (uniform: every workgroup derives it from the same pivots),
            // before any store of the pass: the host resumes here with the per-pass exact bodies
            if (blockIdx.x == 0 && threadIdx.x == 0 && ldc<true>(&st->done) == 0) stc<true>(&st->done, 3);
            return;
        }
        // ---- every wave's X / Y slot stores drained before the workgroup's ticket
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        block_reduce_cand<kP2Threads>(best);  // (its barrier orders the waves' drains before the add)
        const unsigned target = (unsigned)(i + 1) * G;
        // candidates double-buffered by pass parity: a workgroup that has finished pass i's reduction
        // may publish pass i + 1's candidate while another still reads pass i's (it cannot get two
        // passes ahead: pass i + 1 completes only once every workgroup has read pass i's records)
        Cand* const cbuf = g.cand + (i & 1) * G;
        if (threadIdx.x == 0) {
            store_cand_sc1(cbuf + blockIdx.x, best);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned old =
                __hip_atomic_fetch_add((gptr<unsigned>)e.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_go = (old & kEpochAbort) ? 0 : old + 1 == target ? 1 : epoch_wait(e.sync, target, e.timeout, st);
        }
        __syncthreads();
        if (!s_go) return;
        // ---- every workgroup: the winner of all G candidates
        CandR w = threadIdx.x < G ? load_cand_sc1(cbuf + threadIdx.x) : cand_none();
        __syncthreads();  // block_reduce_cand's LDS slots are reused
        block_reduce_cand<kP2Threads>(w);
        if (threadIdx.x == 0) s_w = w;
        __syncthreads();
        w = s_w;
        const double err = fabs(w.val);
        if (!(w.v >= 0.0)) {  // every trailing value NaN: the per-pass path commits it (commit_pivot)
            if (blockIdx.x == 0 && threadIdx.x == 0) stc<true>(&st->done, 3);
            return;
        }
        if ((err < sel.reltol * maxerror) || (err < sel.abstol)) {  // the stop test (K >= 1)
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                stc<true>(&st->error, err);
                stc<true>(&st->done, 1);
            }
            return;
        }
        const int rp = w.rpos, cp = w.cpos, pr = w.pr, pc = w.pc;
#ifdef TCI_EPOCH_DEBUG
        if (threadIdx.x == 0 && blockIdx.x < 3 && K < 12)
            printf("[epoch wg %d] K=%d pr=%d pc=%d rp=%d cp=%d val=%.17g a2=%.17g\n", (int)blockIdx.x, K, pr, pc, rp, cp, w.val, w.v);
#endif
        // swaprow!(K, rp) / swapcol!(K, cp) on the LDS maps; the owners store the global maps
        for (int t = threadIdx.x; t < kRowsPerTile; t += kP2Threads) {
            const int pos = lrow[t];
            if (pos == rp) {  // row pr: to position K
                lrow[t] = K;
                if (q == 0) {
                    stc<true>(sel.rowphys + K, (int64_t)pr);
                    stc<true>(sel.rowpos + pr, (int32_t)K);
                }
            } else if (pos == K) {  // the row at position K: to rp
                lrow[t] = rp;
                if (q == 0) {
                    stc<true>(sel.rowphys + rp, (int64_t)(tb + t));
                    stc<true>(sel.rowpos + tb + t, (int32_t)rp);
                }
            }
        }
        for (int x = threadIdx.x; x < ncols; x += kP2Threads) {
            const int pos = lcol[x];
            if (pos == cp || pos == K) {
                const int j = ((q + (x >> cbs) * nq) << cbs) + (x & (cb - 1));
                if (pos == cp) {
                    lcol[x] = (int16_t)K;
                    if (tr == 0) {
                        stc<true>(sel.colphys + K, (int64_t)pc);
                        stc<true>(sel.colpos + pc, (int32_t)K);
                    }
                } else {
                    lcol[x] = (int16_t)cp;
                    if (tr == 0) {
                        stc<true>(sel.colphys + cp, (int64_t)j);
                        stc<true>(sel.colpos + j, (int32_t)cp);
                    }
                }
            }
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            stc<true>(&st->error, err);
            stc<true>(&st->maxerror, jl_max(maxerror, err));
            stc<true>(&st->p, (int64_t)pr);
            stc<true>(&st->q, (int64_t)pc);
            stc<true>(&st->pval, w.val);
            stc<true>(&st->np, (int64_t)(K + 1));
            stc<true>(sel.pivvals + K, w.val);
        }
        if (threadIdx.x == 0) lpiv[i] = w.val;
        maxerror = jl_max(maxerror, err);
        ein.a = pr;
        ein.b = pc;
        ein.piv = w.val;
        __syncthreads();  // the maps, lpiv, s_go and the reduction's LDS before the next pass
    }
}

void launch_pass_epoch(hipStream_t s, const PassArgs& g, int grid, int npass, int serp, unsigned* sync,
                       long long timeout) {
    const SelArgs sel{g.rowpos, g.colpos, g.rowphys, g.colphys, g.pivvals, g.st,
                      g.ticket, g.reltol, g.abstol,  g.selk,    nullptr, 0};
    const PassK a{g.A,  g.lda, g.m,  g.n,   g.k,        g.X,    g.ldx, g.Y,   g.ldy,
                  g.Lp, g.ldl, g.Up, g.ldu, g.leftorth, g.cand, g.cb,  g.rev, g.S, g.lds,
                  g.pe, g.ps, g.nbs, g.Asrc, g.ldsrc};
    const EpochArgs e{npass, serp, sync, timeout};
    if (g.pe > g.ps)
        hipLaunchKernelGGL((k_pass_mf_epoch<true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel, e);
    else
        hipLaunchKernelGGL((k_pass_mf_epoch<false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel, e);
}

#else
void launch_pass_epoch(hipStream_t, const PassArgs&, int, int, int, unsigned*, long long) {}
#endif

// whether the persistent epoch launch takes this shape: its LDS column map holds int16 positions of
// at most kEpochMaxCols columns per workgroup
bool epoch_fits(int m, int n, int cb, int grid) {
    if (!kEpochGrid) return false;
    const int tiles_r = (m + kRowsPerTile - 1) / kRowsPerTile, tiles_c = (n + cb - 1) / cb;
    const int nq = grid / tiles_r;
    if (nq < 1 || n > 32768) return false;
    return (int64_t)((tiles_c + nq - 1) / nq) * cb <= kEpochMaxCols;
}

// tiles_r x nq workgroups: every row tile gets nq = min(tiles_c, max_grid / tiles_r) chunks of
// column tiles (at least one; the host rejects tiles_r > kMaxPassGrid).
int shadow_elem_bytes() { return kShU8 ? 1 : kShHalf ? 2 : 4; }
// the two-level epoch (refresh + EXT passes) exists only in the MFMA search (k_pass_mf): a build
// without it (TCI_SH_MFMA=0) must write back after every shadow epoch
bool shadow_two_level() { return kShHalf && TCI_SH_MFMA; }

int argmax_grid(int m, int n, int k, int cb, int max_grid) {
    (void)k;
    const long long tiles_r = m > 0 ? (m + kRowsPerTile - 1) / kRowsPerTile : 1;
    const long long tiles_c = n > 0 ? (n + cb - 1) / cb : 1;
    long long nq = max_grid / tiles_r;
    if (nq > tiles_c) nq = tiles_c;
    if (nq < 1) nq = 1;
    return (int)(tiles_r * nq);
}

template <int P>
static void launch_pass_p(hipStream_t s, bool flush, bool shadow, const PassArgs& g, int grid, int kind) {
    const SelArgs sel{g.rowpos, g.colpos, g.rowphys, g.colphys, g.pivvals, g.st,
                      g.ticket, g.reltol, g.abstol,  g.selk,    g.lout, g.pc_off};
    const PassK a{g.A,  g.lda, g.m,  g.n,   g.k,        g.X,    g.ldx, g.Y,   g.ldy,
                  g.Lp, g.ldl, g.Up, g.ldu, g.leftorth, g.cand, g.cb,  g.rev, g.S, g.lds,
                  g.pe, g.ps, g.nbs, g.Asrc, g.ldsrc};
    if (shadow && kShHalf) {
        // fp16: the shadow's scale needs |pivot 0|, so the initial pass only selects, and pass 0
        // (exact) writes the shadow of A; write-backs write the shadow of the new stale values
        if (P == 0)
            hipLaunchKernelGGL((k_pass2<0, false, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
        else if (flush)
            hipLaunchKernelGGL((k_pass2<P, true, true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
        else if (P == 1 && g.k == 0)
            hipLaunchKernelGGL((k_pass2<1, false, true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
        else if constexpr (P > 0) {
            // P here is the shadow-pending count g.ps; EXT when the exact epoch is longer
            const bool ext = g.pe > g.ps, rf = kind == 2;
            if constexpr (TCI_SH_MFMA && P <= kMfMaxP) {
                if (ext && rf)
                    hipLaunchKernelGGL((k_pass_mf<P, true, true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
                else if (ext && TCI_PASS_ONEP)
                    hipLaunchKernelGGL((k_pass_mf<kEpochMaxP, true, false, true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
                else if (ext)
                    hipLaunchKernelGGL((k_pass_mf<P, true, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
                else if (rf)
                    hipLaunchKernelGGL((k_pass_mf<P, false, true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
                else
                    hipLaunchKernelGGL((k_pass_mf<P, false, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
            } else if constexpr (kShU8) {  // (k_pass_sh reads an fp16 / fp32 shadow: the exact pass)
                hipLaunchKernelGGL((k_pass2<P, false, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
            } else {
                hipLaunchKernelGGL((k_pass_sh<P>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
            }
        }
    } else if (shadow && !kShHalf) {  // (the fp32 shadow build, TCI_SH_HALF=0)
        if constexpr (!kShHalf) {
            if (flush || P == 0)
                hipLaunchKernelGGL((k_pass2<P, (P > 0), true>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
            else if constexpr (P > 0)
                hipLaunchKernelGGL((k_pass_sh<P>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
        }
    } else if (flush) {
        hipLaunchKernelGGL((k_pass2<P, true, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
    } else {
        hipLaunchKernelGGL((k_pass2<P, false, false>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
    }
}

#ifndef TCI_PASSX_MIN
#define TCI_PASSX_MIN 12  // write-backs with at least this many pending updates: k_pass_x (x's in LDS)
#endif

// kind: -1 legacy (P pending, write-back iff flush); 0 read-only, 1 write-back, 2 refresh, with
// g.pe / g.ps the exact / shadow pending counts (two-level epoch)
void launch_pass(hipStream_t s, int P, bool flush, bool shadow, const PassArgs& g, int grid, int kind) {
    if (kind < 0) kind = flush ? 1 : 0;
    PassArgs h = g;
    if (h.pe <= 0) h.pe = h.ps = P;  // legacy callers (column-sharded driver): one epoch level
    if (kind == 1 && shadow && kShHalf && h.pe >= TCI_PASSX_MIN) {
        const SelArgs sel{h.rowpos, h.colpos, h.rowphys, h.colphys, h.pivvals, h.st,
                          h.ticket, h.reltol, h.abstol,  h.selk,    h.lout, h.pc_off};
        const PassK a{h.A,  h.lda, h.m,  h.n,   h.k,        h.X,    h.ldx, h.Y,   h.ldy,
                      h.Lp, h.ldl, h.Up, h.ldu, h.leftorth, h.cand, h.cb,  h.rev, h.S, h.lds,
                      h.pe, h.ps, h.nbs, h.Asrc, h.ldsrc};
        // 512-thread workgroups, two per CU, over 256-row tiles -- the same column sets (nq) with
        // twice the row tiles: one workgroup's staging and y_k chains overlap the other's streaming
        // (8192^2: 298-300 -> 289-290 us per write-back, profiles/r05_o1_ab_passx_nt.txt; 497 parity
        // tests green on it). TCI_PASSX_NT=1024: one 1024-thread workgroup per 512-row tile
        static const int px_nt = [] {
            const char* e = getenv("TCI_PASSX_NT");
            return e ? atoi(e) : 512;
        }();
        const int tiles_r = (h.m + kRowsPerTile - 1) / kRowsPerTile;
        const int nq = grid / tiles_r;
        const int tiles_r2 = (h.m + PxGeom<512>::Tile - 1) / PxGeom<512>::Tile;
        if (px_nt == 512 && (int64_t)tiles_r2 * nq <= kMaxPassGrid)
            hipLaunchKernelGGL((k_pass_x<1, 512>), dim3(tiles_r2 * nq), dim3(512), 0, s, a, sel);
        else
            hipLaunchKernelGGL((k_pass_x<1>), dim3(grid), dim3(kP2Threads), 0, s, a, sel);
        return;
    }
    const int PP = kind == 1 || !(shadow && kShHalf) ? h.pe : h.ps;
    switch (PP) {
#define TCI_PASS_CASE(p) \
    case p: launch_pass_p<p>(s, kind == 1, shadow, h, grid, kind); break;
        TCI_PASS_CASE(0) TCI_PASS_CASE(1) TCI_PASS_CASE(2) TCI_PASS_CASE(3) TCI_PASS_CASE(4)
        TCI_PASS_CASE(5) TCI_PASS_CASE(6) TCI_PASS_CASE(7) TCI_PASS_CASE(8) TCI_PASS_CASE(9)
        TCI_PASS_CASE(10) TCI_PASS_CASE(11) TCI_PASS_CASE(12) TCI_PASS_CASE(13) TCI_PASS_CASE(14)
        TCI_PASS_CASE(15) TCI_PASS_CASE(16)
#undef TCI_PASS_CASE
    default: break;
    }
}

// ---------------------------------------------------------------- select
// Pivot k: given the winner over all candidates (its value is the current, pending-updated one),
// the stop test of _optimizerrlu! (matrixlu.jl:359-368), and on acceptance addpivot!'s swaps as
// map updates: the rows at positions k and p exchange positions (swaprow!, :254-262), likewise
// the columns at k and q (swapcol!, :269-275). One thread.
template <bool COH>
__device__ void commit_pivot(int k, const CandR& best, RrluState* st, double reltol, double abstol,
                             int32_t* rowpos, int32_t* colpos, int64_t* rowphys, int64_t* colphys,
                             double* pivvals, int64_t rk, int64_t ck, bool has_mxe, double mxe) {
    int pr = best.pr, pc = best.pc, rp = best.rpos, cp = best.cpos;
    double val = best.val;
#ifdef TCI_EPOCH_DEBUG
    if (k < 12) printf("[pass] K=%d pr=%d pc=%d rp=%d cp=%d val=%.17g a2=%.17g\n", k, pr, pc, rp, cp, val, best.v);
#endif
    if (!(best.v >= 0.0)) {
        // every trailing value is NaN: Julia keeps (first(rows), first(cols)) = positions (k, k),
        // whose current value is one of those NaNs
        rp = k;
        cp = k;
        pr = (int)ldc<COH>(rowphys + k);
        pc = (int)ldc<COH>(colphys + k);
        val = __longlong_as_double(0x7ff8000000000000LL);
    }
    const double err = fabs(val);
    stc<COH>(&st->error, err);
    const double maxerror = has_mxe ? mxe : ldc<COH>(&st->maxerror);  // mxe: requested with the candidates
    if (((fabs(err) < reltol * maxerror) || (fabs(err) < abstol)) && k > 0) {
        stc<COH>(&st->done, 1);
        return;
    }
    stc<COH>(&st->maxerror, jl_max(maxerror, err));
    stc<COH>(&st->p, (int64_t)pr);
    stc<COH>(&st->q, (int64_t)pc);
    stc<COH>(&st->pval, val);
    stc<COH>(&st->np, (int64_t)(k + 1));
    stc<COH>(pivvals + k, val);
    // swaprow!(k, rp): the physical row at position k moves to position rp
    if (rk < 0) rk = ldc<COH>(rowphys + k);
    stc<COH>(rowphys + k, (int64_t)pr);
    stc<COH>(rowphys + rp, rk);
    stc<COH>(rowpos + pr, (int32_t)k);
    stc<COH>(rowpos + rk, (int32_t)rp);
    // swapcol!(k, cp)
    if (ck < 0) ck = ldc<COH>(colphys + k);
    stc<COH>(colphys + k, (int64_t)pc);
    stc<COH>(colphys + cp, ck);
    stc<COH>(colpos + pc, (int32_t)k);
    stc<COH>(colpos + ck, (int32_t)cp);
}

__global__ void k_init_state(RrluState* st, int32_t* rowpos, int64_t* rowphys, int m,
                             int32_t* colpos, int64_t* colphys, int n) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int stride = gridDim.x * blockDim.x;
    if (gid == 0) {
        st->np = 0;
        st->done = 0;
        st->maxerror = 0.0;
        st->error = __longlong_as_double(0x7ff8000000000000LL);  // rrLU{T}(...): error = NaN
        st->p = st->q = 0;
        st->pval = 0.0;
    }
    for (int i = gid; i < m; i += stride) {
        rowpos[i] = i;
        rowphys[i] = i;
    }
    for (int j = gid; j < n; j += stride) {
        colpos[j] = j;
        colphys[j] = j;
    }
}

void launch_init_state(hipStream_t s, RrluState* st, int32_t* rowpos, int64_t* rowphys, int m,
                       int32_t* colpos, int64_t* colphys, int n) {
    int work = m > n ? m : n;
    int grid = (work + 255) / 256;
    if (grid > 256) grid = 256;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(k_init_state, dim3(grid), dim3(256), 0, s, st, rowpos, rowphys, m, colpos,
                       colphys, n);
}

// ------------------------------------------------------------ small rrLU
// Pi matrices of a TCI2 sweep at low rank are small (C1: ~120 x 120); there the per-pivot launch
// latency of the pass pipeline dominates. One 1024-thread workgroup holds the whole matrix in
// LDS and runs _optimizerrlu! (matrixlu.jl:346-369) as written: argmax over the trailing block
// (column-major scan order as the tie-break), stop test, swaprow!/swapcol! (physical, in LDS),
// true-division normalisation and the rank-1 update with separate multiply and subtract.
#ifndef TCI_SMALL_THREADS
#define TCI_SMALL_THREADS 1024
#endif
constexpr int kSmallThreads = TCI_SMALL_THREADS;

bool rrlu_small_fits(int64_t m, int64_t n) {
    return m > 0 && n > 0 && (m | 1) * n <= kSmallElems && m + n <= kSmallPerm;
}

static size_t small_lds_bytes(int m, int n) {
    const size_t a = ((size_t)(m | 1) * n * sizeof(double) + 15) / 16 * 16;
    const size_t p = ((size_t)(m + n) * sizeof(int) + 15) / 16 * 16;
    return a + p + (kSmallThreads / 64) * sizeof(CandR) + 32 + (size_t)(m + n) * sizeof(double);
}

__global__ __launch_bounds__(kSmallThreads) void k_rrlu_small(
    const double* __restrict__ A, int64_t lda, int m, int n, int mr, double reltol, double abstol,
    int leftorth, RrluState* st, int64_t* rowphys, int64_t* colphys, double* pivvals,
    double* Lp, int64_t ldl, double* Up, int64_t ldu, SmallOut out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // m x n with an odd leading dimension: row accesses (swaps, the pivot row) hit distinct banks
    const int ldS = m | 1;
    double* S = reinterpret_cast<double*>(smem);
    int* rp = reinterpret_cast<int*>(smem + ((size_t)ldS * n * sizeof(double) + 15) / 16 * 16);
    int* cp = rp + m;
    CandR* red = reinterpret_cast<CandR*>(reinterpret_cast<char*>(rp) +
                                          ((size_t)(m + n) * sizeof(int) + 15) / 16 * 16);
    int* ctl = reinterpret_cast<int*>(red + kSmallThreads / 64);  // [3] np, [4] NaN flags
    double* xv = reinterpret_cast<double*>(ctl + 8);  // column k (normalised if leftorth)
    double* yv = xv + m;                             // row k (normalised otherwise)
    // thread (w, l) owns rows l, l + 64, ... of columns w, w + 16, ...: no index division
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    constexpr int NW = kSmallThreads / 64;
    for (int j = w; j < n; j += NW)
        for (int i = l; i < m; i += 64) S[i + j * ldS] = A[i + (int64_t)j * lda];
    double maxerror, error;
    int np = small_lu_core<kSmallThreads>(S, ldS, m, n, mr, reltol, abstol, leftorth, rp, cp,
                                          reinterpret_cast<SmallCand*>(red), xv, yv, pivvals, error, maxerror);
    if (tid == 0) {
        st->np = np;
        st->done = 1;
        st->maxerror = maxerror;
        st->error = error;
        ctl[3] = np;
        ctl[4] = 0;
        if (out.maxout) *out.maxout = *out.maxin;
    }
    __syncthreads();
    np = ctl[3];  // thread 0's count, for every thread
    // outputs in the pass pipeline's conventions (physical-order L columns / U rows)
    for (int i = tid; i < m; i += kSmallThreads) rowphys[i] = rp[i];
    for (int j = tid; j < n; j += kSmallThreads) colphys[j] = cp[j];
    if (Lp)
        for (int e = tid; e < m * np; e += kSmallThreads) {
            const int pos = e % m, t = e / m;
            if (pos > t) Lp[rp[pos] + (int64_t)t * ldl] = S[pos + t * ldS];
        }
    if (Up)
        for (int e = tid; e < np * n; e += kSmallThreads) {
            const int t = e % np, pos = e / np;
            if (pos > t) Up[t + (int64_t)cp[pos] * ldu] = S[t + pos * ldS];
        }
    if (!out.flag) return;
    // NaN checks of tril(A[:, 1:np]) / triu(A[1:np, :]) before the unit diagonal is set
    // (matrixlu.jl:376-381); the pivot values sit on S's diagonal
    {
        int fl = 0;
        for (int e = tid; e < m * np; e += kSmallThreads) {
            const int pos = e % m, t = e / m;
            if (pos >= t && isnan(S[pos + t * ldS])) fl |= 1;
        }
        for (int e = tid; e < np * n; e += kSmallThreads) {
            const int t = e % np, pos = e / np;
            if (pos >= t && isnan(S[t + pos * ldS])) fl |= 2;
        }
        if (fl) atomicOr(&ctl[4], fl);
        __syncthreads();
        if (tid == 0) *out.flag = ctl[4];
    }
    if (np == 0) return;
    // MatrixLUCI factors (matrixluci.jl:161-283) straight from LDS, in the same operation order
    // as the pass pipeline's factor kernels (tci_device.hip). Position-order L / U are
    //   leftorth:  L[a,t] = (t == a ? 1 : S[a,t]),  U[t,j] = S[t,j]          (t <= a, t <= j)
    //   otherwise: L[i,t] = S[i,t],                 U[t,j] = (t == j ? 1 : S[t,j])
    if (leftorth) {
        if (out.right)  // rowmatrix = L11 * U, column-scattered
            for (int e = tid; e < np * n; e += kSmallThreads) {
                const int a = e % np, j = e / np;
                double s = 0.0;
                for (int t = 0; t <= min(a, j); ++t)
                    s = __dadd_rn(s, __dmul_rn(t == a ? 1.0 : S[a + t * ldS], S[t + j * ldS]));
                out.right[a + (int64_t)cp[j] * np] = s;
            }
        if (out.left) {  // colstimespivotinv: rows >= np solve X L11 = L21 in place
            __syncthreads();
            for (int i = np + tid; i < m; i += kSmallThreads)
                for (int j = np - 1; j >= 0; --j) {
                    double s = S[i + j * ldS];
                    for (int t = j + 1; t < np; ++t) s = __dsub_rn(s, __dmul_rn(S[i + t * ldS], S[t + j * ldS]));
                    S[i + j * ldS] = s;
                }
            __syncthreads();
            for (int e = tid; e < m * np; e += kSmallThreads) {
                const int i = e % m, j = e / m;
                out.left[rp[i] + (int64_t)j * m] = i < np ? (i == j ? 1.0 : 0.0) : S[i + j * ldS];
            }
        }
    } else {
        if (out.left)  // colmatrix = L * U11, row-scattered
            for (int e = tid; e < m * np; e += kSmallThreads) {
                const int i = e % m, j = e / m;
                double s = 0.0;
                for (int t = 0; t <= min(i, j); ++t)
                    s = __dadd_rn(s, __dmul_rn(S[i + t * ldS], t == j ? 1.0 : S[t + j * ldS]));
                out.left[rp[i] + (int64_t)j * m] = s;
            }
        if (out.right) {  // pivotinvtimesrows: columns >= np solve U11 x = U[:, c] in place
            __syncthreads();
            for (int c = np + tid; c < n; c += kSmallThreads)
                for (int a = np - 1; a >= 0; --a) {
                    double s = S[a + c * ldS];
                    for (int t = a + 1; t < np; ++t) s = __dsub_rn(s, __dmul_rn(S[a + t * ldS], S[t + c * ldS]));
                    S[a + c * ldS] = s;
                }
            __syncthreads();
            for (int e = tid; e < np * n; e += kSmallThreads) {
                const int a = e % np, j = e / np;
                out.right[a + (int64_t)cp[j] * np] = j < np ? (a == j ? 1.0 : 0.0) : S[a + j * ldS];
            }
        }
    }
}

hipError_t launch_rrlu_small(hipStream_t s, const double* A, int64_t lda, int m, int n, int mr,
                             double reltol, double abstol, int leftorth, RrluState* st,
                             int64_t* rowphys, int64_t* colphys, double* pivvals, double* Lp,
                             int64_t ldl, double* Up, int64_t ldu, SmallOut out) {
    const size_t bytes = small_lds_bytes(m, n);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rrlu_small),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rrlu_small, dim3(1), dim3(kSmallThreads), bytes, s, A, lda, m, n, mr,
                       reltol, abstol, leftorth, st, rowphys, colphys, pivvals, Lp, ldl, Up, ldu,
                       out);
    return hipGetLastError();
}

// ------------------------------------------------------------ mid-size rrLU
// Pi matrices of a few MiB (C3': 1024^2 at rank 64) are too big for one workgroup's LDS and too
// small for the pass pipeline, whose ~16 us per pivot is a chain of dependent memory round trips
// plus a launch. Here the matrix lives in the LDS of a persistent grid (one
// workgroup per CU), split by column blocks; each pivot costs one grid barrier:
//   1. every workgroup publishes its local argmax candidate and that candidate's (current,
//      updated) column (sc1 stores), then arrives at the barrier (agent-scope atomic counter);
//   2. every workgroup reduces the candidates to the same winner (reference tie order), applies
//      the stop test, swaprow!(k, p) on its own columns, swapcol!(k, q) on the replicated column
//      position maps, and takes the pivot column from the winner's published copy;
//   3. normalisation and the rank-1 update of its own trailing columns, fused with the next
//      local argmax.
// Same arithmetic as the reference (separate multiply / subtract, true division): bitwise equal
// to the other paths. Outputs in the pass pipeline's conventions.
constexpr int kMidThreads = 256;
constexpr int kMidMaxGrid = 256;
constexpr size_t kMidLds = 150 * 1024;

struct MidArgs {
    const double* A;
    int64_t lda;
    int m, n, mr, ncl, leftorth;
    double reltol, abstol;
    RrluState* st;
    int64_t* rowphys;
    int64_t* colphys;
    double* pivvals;
    double* Lp;
    int64_t ldl;
    double* Up;
    int64_t ldu;
    Cand* cand;       // one per workgroup
    double* colbuf;   // gridDim.x x m: the published candidate columns
    unsigned* count;  // barrier arrivals (monotonic; zeroed before launch)
    int* fault;       // set on a barrier timeout
};

static size_t mid_lds_bytes(int m, int n, int ncl) {
    return ((size_t)m * ncl * 8 + 15) / 16 * 16 + (size_t)m * 8 + ((size_t)(2 * n + m) * 4 + 15) / 16 * 16 +
           (kMidThreads / 64) * sizeof(CandR) + 64;
}

// grid-wide barrier on a monotonic arrival counter: barrier number e completes at
// (e + 1) * gridDim.x arrivals. Every wave drains its stores first (hand-off table, row 1).
__device__ __forceinline__ bool mid_grid_sync(unsigned* count, unsigned& epoch, int* fault, int* lflag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned target = (epoch + 1) * gridDim.x;
        const unsigned old = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int bad = 0;
        if (old + 1 < target) {
            // bounded by wall time (100 MHz counter): 4 ms is ~300x a pivot's barrier wait, so only
            // workgroups that are not co-resident (another stream or process holding CUs) reach it
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t0 > 400000ull ||
                    __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    bad = 1;  // a peer is missing or has failed: give up instead of hanging
                    __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        *lflag = bad;
    }
    ++epoch;
    __syncthreads();
    return *lflag == 0;
}

__global__ __launch_bounds__(kMidThreads) void k_rrlu_mid(MidArgs g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int m = g.m, n = g.n, ncl = g.ncl;
    const int c0 = blockIdx.x * ncl;
    const int nc = max(0, min(ncl, n - c0));  // local columns: global c0 .. c0 + nc - 1
    double* S = reinterpret_cast<double*>(smem);  // m x ncl, ld m
    double* xv = reinterpret_cast<double*>(smem + ((size_t)m * ncl * 8 + 15) / 16 * 16);
    int* cpos = reinterpret_cast<int*>(xv + m);  // replicated column position map (n)
    int* cphys = cpos + n;                       // its inverse (n)
    int* rperm = cphys + n;                      // row permutation (m), identical everywhere
    CandR* red = reinterpret_cast<CandR*>(reinterpret_cast<char*>(cpos) +
                                          ((size_t)(2 * n + m) * 4 + 15) / 16 * 16);
    int* ctl = reinterpret_cast<int*>(red + kMidThreads / 64);
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    for (int e = tid; e < m * nc; e += kMidThreads)
        S[e] = g.A[(e % m) + (int64_t)(c0 + e / m) * g.lda];
    for (int j = tid; j < n; j += kMidThreads) {
        cpos[j] = j;
        cphys[j] = j;
    }
    for (int i = tid; i < m; i += kMidThreads) rperm[i] = i;
    double maxerror = 0.0, error = __longlong_as_double(0x7ff8000000000000LL);
    int np = 0;
    unsigned epoch = 0;
    __syncthreads();
    // local argmax of the initial matrix
    CandR best = cand_none();
    for (int j = w; j < nc; j += kMidThreads / 64)
        for (int i = l; i < m; i += 64) {
            const double v = S[i + j * m];
            const double a2 = __dmul_rn(v, v);
            if (cand_better(a2, cpos[c0 + j], i, best.v, best.cpos, best.rpos))
                best = CandR{a2, v, cpos[c0 + j], i, c0 + j, i};
        }
    for (int k = 0; k < g.mr; ++k) {
        // 1. publish the local candidate and its column
        wave_reduce_cand(best);
        if (l == 0) red[w] = best;
        __syncthreads();
        if (tid == 0) {
            CandR b = red[0];
            for (int i = 1; i < kMidThreads / 64; ++i) cand_take(b, red[i]);
            store_cand_sc1(g.cand + blockIdx.x, b);
            ctl[0] = b.v >= 0.0 ? b.pc - c0 : -1;
        }
        __syncthreads();
        if (ctl[0] >= 0) {
            const double* col = S + (int64_t)ctl[0] * m;
            double* dst = g.colbuf + (int64_t)blockIdx.x * m;
            for (int i = tid; i < m; i += kMidThreads)
                __hip_atomic_store(reinterpret_cast<uint64_t*>(dst + i), (uint64_t)__double_as_longlong(col[i]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!mid_grid_sync(g.count, epoch, g.fault, ctl + 4)) return;
        // 2. the same winner everywhere
        CandR b = cand_none();
        for (int i = tid; i < (int)gridDim.x; i += kMidThreads) cand_take(b, load_cand_sc1(g.cand + i));
        wave_reduce_cand(b);
        __syncthreads();  // red reuse
        if (l == 0) red[w] = b;
        __syncthreads();
        b = red[0];
        for (int i = 1; i < kMidThreads / 64; ++i) cand_take(b, red[i]);
        int p = b.rpos, q = b.pc;  // row position (= physical LDS row), global column
        double val = b.val;
        const bool allnan = !(b.v >= 0.0);
        if (allnan) {  // every trailing value NaN: Julia keeps (k, k); the pivot column is NaN there
            p = k;
            q = cphys[k];
            val = __longlong_as_double(0x7ff8000000000000LL);
        }
        error = fabs(val);
        if (((fabs(error) < g.reltol * maxerror) || (fabs(error) < g.abstol)) && k > 0) break;
        maxerror = jl_max(maxerror, error);
        np = k + 1;
        if (blockIdx.x == 0 && tid == 0) g.pivvals[k] = val;
        // pivot column (pre-swap rows) from the winner's copy; its rows k and p trade places below
        const int owner = q / ncl;
        // (all-NaN case: only rows >= k are used, and there every value is NaN)
        for (int i = tid; i < m; i += kMidThreads)
            xv[i] = allnan ? __longlong_as_double(0x7ff8000000000000LL)
                           : __longlong_as_double((long long)__hip_atomic_load(
                                 reinterpret_cast<const uint64_t*>(g.colbuf + (int64_t)owner * m + i),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        __syncthreads();
        if (tid == 0 && p != k) {
            const double t = xv[k];
            xv[k] = xv[p];
            xv[p] = t;
            const int r = rperm[k];
            rperm[k] = rperm[p];
            rperm[p] = r;
        }
        // swaprow!(k, p) on the local columns
        if (p != k)
            for (int j = tid; j < nc; j += kMidThreads) {
                const double t = S[k + j * m];
                S[k + j * m] = S[p + j * m];
                S[p + j * m] = t;
            }
        // swapcol!(k, q): positions only
        if (tid == 0) {
            const int cq = cpos[q], ck = cphys[k];
            cphys[k] = q;
            cphys[cq] = ck;
            cpos[q] = k;
            cpos[ck] = cq;
        }
        __syncthreads();
        // 3. normalisation (matrixlu.jl:300-305): the L column in xv (and in the owner's S), the
        // U row in place
        const double piv = xv[k];
        if (g.leftorth)
            for (int i = k + 1 + tid; i < m; i += kMidThreads) xv[i] = xv[i] / piv;
        for (int j = tid; j < nc; j += kMidThreads)
            if (cpos[c0 + j] > k && !g.leftorth) S[k + j * m] = S[k + j * m] / piv;
        __syncthreads();
        if (q >= c0 && q < c0 + nc)  // the owner's pivot column becomes L column k
            for (int i = k + tid; i < m; i += kMidThreads) S[i + (q - c0) * m] = xv[i];
        // rank-1 update of the local trailing columns fused with the next local argmax
        best = cand_none();
        for (int j = w; j < nc; j += kMidThreads / 64) {
            const int cp = cpos[c0 + j];
            if (cp <= k) continue;
            const double y = S[k + j * m];
            for (int i = l; i < m; i += 64) {
                if (i <= k) continue;
                const double v = __dsub_rn(S[i + j * m], __dmul_rn(xv[i], y));
                S[i + j * m] = v;
                const double a2 = __dmul_rn(v, v);
                if (cand_better(a2, cp, i, best.v, best.cpos, best.rpos)) best = CandR{a2, v, cp, i, c0 + j, i};
            }
        }
        __syncthreads();
    }
    // outputs: state, permutations (workgroup 0), L columns / U rows of the local columns
    if (blockIdx.x == 0) {
        if (tid == 0) {
            g.st->np = np;
            g.st->done = 1;
            g.st->maxerror = maxerror;
            g.st->error = error;
        }
        for (int i = tid; i < m; i += kMidThreads) g.rowphys[i] = rperm[i];
        for (int j = tid; j < n; j += kMidThreads) g.colphys[j] = cphys[j];
    }
    for (int j = 0; j < nc; ++j) {
        const int pos = cpos[c0 + j];
        if (pos < np)
            for (int i = pos + 1 + tid; i < m; i += kMidThreads) g.Lp[rperm[i] + (int64_t)pos * g.ldl] = S[i + j * m];
        for (int t = tid; t < min(np, pos); t += kMidThreads) g.Up[t + (int64_t)(c0 + j) * g.ldu] = S[t + j * m];
    }
}

bool rrlu_mid_fits(int64_t m, int64_t n, int ncu) {
    if (m <= 0 || n <= 0 || m * n > (int64_t)1 << 21) return false;
    const int G = (int)std::min<int64_t>(std::min(ncu, kMidMaxGrid), n);
    const int ncl = (int)((n + G - 1) / G);
    return mid_lds_bytes((int)m, (int)n, ncl) <= kMidLds;
}

hipError_t launch_rrlu_mid(hipStream_t s, int ncu, const double* A, int64_t lda, int m, int n, int mr,
                           double reltol, double abstol, int leftorth, RrluState* st, int64_t* rowphys,
                           int64_t* colphys, double* pivvals, double* Lp, int64_t ldl, double* Up,
                           int64_t ldu, Cand* cand, double* colbuf, unsigned* count, int* fault) {
    const int G = std::min(std::min(ncu, kMidMaxGrid), n);
    MidArgs g{A, lda, m, n, mr, (n + G - 1) / G, leftorth, reltol, abstol, st, rowphys, colphys, pivvals,
              Lp, ldl, Up, ldu, cand, colbuf, count, fault};
    const size_t bytes = mid_lds_bytes(m, n, g.ncl);
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rrlu_mid),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_rrlu_mid),
                                                     kMidThreads, bytes);
    if (e != hipSuccess) return e;
    if ((int64_t)per_cu * ncu < G) return hipErrorCooperativeLaunchTooLarge;
    if ((e = hipMemsetAsync(count, 0, sizeof(unsigned), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(fault, 0, sizeof(int), s)) != hipSuccess) return e;
    // An ordinary launch, not hipLaunchCooperativeKernel: G <= one workgroup per CU fits the chip
    // at once, and the barrier's timeout + fault flag bound the wait if another stream's kernels
    // hold CUs (the host then reruns the factorisation on the pass pipeline). HIP's cooperative
    // queue was also what faulted in exit() after rocprofv3's finalisation.
    hipLaunchKernelGGL(k_rrlu_mid, dim3(G), dim3(kMidThreads), bytes, s, g);
    return hipGetLastError();
}

// ------------------------------------------------------------ extraction
// L (m x np, position order) and U (np x n) as _optimizerrlu! leaves them (matrixlu.jl:372-388):
//   L[pos, t] = 0 (pos < t), diag (pos == t), Lp[rowphys[pos], t] (pos > t)
//   U[t, pos] = 0 (pos < t), diag (pos == t), Up[t, colphys[pos]] (pos > t)
// with the pivot value on U's diagonal and 1 on L's when leftorth, the reverse otherwise.
// NaN check on the way (flag bit 0: L, bit 1: U).
__global__ void k_extract(const double* __restrict__ Lp, int64_t ldlp, const double* __restrict__ Up,
                          int64_t ldup, const double* __restrict__ pivvals,
                          const int64_t* __restrict__ rowphys, const int64_t* __restrict__ colphys,
                          int m, int n, int np, int leftorth, double* __restrict__ L, int64_t ldl,
                          double* __restrict__ U, int64_t ldu, int* flag, int64_t c0, int64_t nloc) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int f = 0;
    for (int64_t e = gid; e < (int64_t)m * np; e += stride) {
        const int pos = (int)(e % m), t = (int)(e / m);
        double v;
        if (pos < t) v = 0.0;
        else if (pos == t) v = leftorth ? 1.0 : pivvals[t];
        else v = Lp[rowphys[pos] + (int64_t)t * ldlp];
        if (pos >= t && isnan(pos == t ? pivvals[t] : v)) f |= 1;
        if (L) L[pos + (int64_t)t * ldl] = v;
    }
    for (int64_t e = gid; e < (int64_t)np * n; e += stride) {
        const int t = (int)(e % np), pos = (int)(e / np);
        const int64_t pc = colphys[pos] - c0;  // local physical column (sharded: others skip)
        if (pc < 0 || pc >= nloc) continue;
        double v;
        if (pos < t) v = 0.0;
        else if (pos == t) v = leftorth ? pivvals[t] : 1.0;
        else v = Up[t + pc * ldup];
        if (pos >= t && isnan(pos == t ? pivvals[t] : v)) f |= 2;
        if (U) U[t + (int64_t)pos * ldu] = v;
    }
    if (f) atomicOr(flag, f);
}

void launch_extract(hipStream_t s, const double* Lp, int64_t ldlp, const double* Up, int64_t ldup,
                    const double* pivvals, const int64_t* rowphys, const int64_t* colphys, int m,
                    int n, int np, int leftorth, double* L, int64_t ldl, double* U, int64_t ldu,
                    int* flag) {
    long long work = (long long)m * np + (long long)np * n;
    long long g = (work + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_extract, dim3((int)g), dim3(256), 0, s, Lp, ldlp, Up, ldup, pivvals, rowphys,
                       colphys, m, n, np, leftorth, L, ldl, U, ldu, flag, (int64_t)0, (int64_t)n);
}

void launch_extract_shard(hipStream_t s, const double* Lp, int64_t ldlp, const double* Up, int64_t ldup,
                          const double* pivvals, const int64_t* rowphys, const int64_t* colphys, int m,
                          int n, int np, int leftorth, double* L, int64_t ldl, double* U, int64_t ldu,
                          int* flag, int64_t c0, int nloc) {
    long long work = (long long)m * np + (long long)np * n;
    long long g = (work + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_extract, dim3((int)g), dim3(256), 0, s, Lp, ldlp, Up, ldup, pivvals, rowphys,
                       colphys, m, n, np, leftorth, L, ldl, U, ldu, flag, c0, (int64_t)nloc);
}

// ------------------------------------------------------------ column-sharded rrLU (tci_internal.h)
__global__ void k_shard_init(int32_t* colpos_loc, int nloc, int64_t c0) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j <= nloc) colpos_loc[j] = j < nloc ? (int32_t)(c0 + j) : -1;  // the ghost is never trailing
}

void launch_shard_init(hipStream_t s, int32_t* colpos_loc, int nloc, int64_t c0) {
    hipLaunchKernelGGL(k_shard_init, dim3((nloc + 256) / 256), dim3(256), 0, s, colpos_loc, nloc, c0);
}

__device__ __forceinline__ double bits_dbl(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t dbl_bits(double d) { return (uint64_t)__double_as_longlong(d); }

// every block reduces the N published candidates in rank order (the reference's tie order) to the
// same winner; -1: no rank has a candidate. Rank r's record at recv + r * rstride (uint64 words: 4
// for the two-collective exchange's packed records, the fused record + column stride otherwise)
__device__ __forceinline__ int shard_winner(const uint64_t* __restrict__ recv, int64_t rstride, int nranks,
                                            CandR& w) {
    w = cand_none();
    int wr = -1;
    for (int r = 0; r < nranks; ++r) {
        const Cand h = *reinterpret_cast<const Cand*>(recv + r * rstride);
        if (h.v >= 0.0 && cand_better(h.v, h.cpos, h.rpos, w.v, w.cpos, w.rpos)) {
            w = CandR{h.v, h.val, h.cpos, h.rpos, h.pcol, h.prow};
            wr = r;
        }
    }
    return wr;
}

// the rank owning the winning column writes [pending y's | stale column] as bits, the others zeros
__global__ __launch_bounds__(256) void k_shard_pick(const Cand* __restrict__ recv, int nranks,
                                                    const double* __restrict__ A, int64_t lda, int m,
                                                    const double* __restrict__ Y, int64_t ldy, int64_t c0, int nloc,
                                                    uint64_t* __restrict__ colsend) {
    __shared__ int own_s;
    if (threadIdx.x == 0) {
        CandR w;
        const int wr = shard_winner(reinterpret_cast<const uint64_t*>(recv), kCandWords, nranks, w);
        own_s = (wr >= 0 && w.pc >= c0 && w.pc < c0 + nloc) ? (int)(w.pc - c0) : -1;
    }
    __syncthreads();
    const int own = own_s;
    const double* col = A + (int64_t)(own >= 0 ? own : 0) * lda;
    if (blockIdx.x == 0 && threadIdx.x < kMaxPendR)
        colsend[threadIdx.x] = own >= 0 ? dbl_bits(Y[(int64_t)threadIdx.x * ldy + own]) : 0ull;
    const int i0 = blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        if (i < m) colsend[kMaxPendR + i] = own >= 0 ? dbl_bits(col[i]) : 0ull;
    }
}

void launch_shard_pick(hipStream_t s, const Cand* recv, int nranks, const double* A, int64_t lda, int m,
                       const double* Y, int64_t ldy, int64_t c0, int nloc, uint64_t* colsend) {
    hipLaunchKernelGGL(k_shard_pick, dim3((m + 1023) / 1024 > 0 ? (m + 1023) / 1024 : 1), dim3(256), 0, s, recv,
                       nranks, A, lda, m, Y, ldy, c0, nloc, colsend);
}

// the fused exchange (one all-gather per pivot): every rank publishes [its own record | the pending
// y's and stale values of its own candidate column] (kCandWords + shard_col(m) words); the record
// is written by block 0, the column only when the rank has a candidate (never read otherwise)
__global__ __launch_bounds__(256) void k_shard_pack(const Cand* __restrict__ own_rec,
                                                    const double* __restrict__ A, int64_t lda, int m,
                                                    const double* __restrict__ Y, int64_t ldy, int64_t c0, int nloc,
                                                    uint64_t* __restrict__ send) {
    const Cand h = *own_rec;
    if (blockIdx.x == 0 && threadIdx.x < kCandWords)
        send[threadIdx.x] = reinterpret_cast<const uint64_t*>(own_rec)[threadIdx.x];
    const int own = (h.v >= 0.0 && h.pcol >= c0 && h.pcol < c0 + nloc) ? (int)(h.pcol - c0) : -1;
    if (own < 0) return;
    uint64_t* colsend = send + kCandWords;
    const double* col = A + (int64_t)own * lda;
    if (blockIdx.x == 0 && threadIdx.x < kMaxPendR) colsend[threadIdx.x] = dbl_bits(Y[(int64_t)threadIdx.x * ldy + own]);
    const int i0 = blockIdx.x * 1024 + threadIdx.x;
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        v[u] = i < m ? col[i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        if (i < m) colsend[kMaxPendR + i] = dbl_bits(v[u]);
    }
}

void launch_shard_pack(hipStream_t s, const Cand* own_rec, const double* A, int64_t lda, int m, const double* Y,
                       int64_t ldy, int64_t c0, int nloc, uint64_t* send) {
    hipLaunchKernelGGL(k_shard_pack, dim3((m + 1023) / 1024 > 0 ? (m + 1023) / 1024 : 1), dim3(256), 0, s, own_rec,
                       A, lda, m, Y, ldy, c0, nloc, send);
}

// Every block reduces the N candidates to the same winner and installs its slice of the ghost
// column; block 0 alone commits (stop test, maps, st). A ghost installed after a stop is never read
// (the passes return at once). colrecv null: one rank, the winning column is this rank's own.
__global__ __launch_bounds__(256) void k_shard_commit(const uint64_t* __restrict__ recv, int64_t rstride,
                                                      int nranks, const uint64_t* __restrict__ colrecv,
                                                      int fused, int m, int k,
                                                      RrluState* st, double reltol, double abstol, int32_t* rowpos,
                                                      int32_t* colpos_g, int64_t* rowphys, int64_t* colphys_g,
                                                      double* pivvals, int32_t* colpos_loc, int64_t c0, int nloc,
                                                      double* A, int64_t lda, double* Y, int64_t ldy) {
    __shared__ int win_s, own_s;
    if (threadIdx.x == 0) {
        CandR w;
        const int wr = shard_winner(recv, rstride, nranks, w);
        win_s = wr;
        own_s = (wr >= 0 && w.pc >= c0 && w.pc < c0 + nloc) ? (int)(w.pc - c0) : -1;
        if (blockIdx.x == 0 && !st->done) {
            const int64_t rk = rowphys[k], ck = colphys_g[k];
            commit_pivot(k, w, st, reltol, abstol, rowpos, colpos_g, rowphys, colphys_g, pivvals, rk, ck);
            if (!st->done) {
                const int64_t pcg = st->q;  // global physical column of the pivot
                if (pcg >= c0 && pcg < c0 + nloc) colpos_loc[pcg - c0] = k;
                if (ck >= c0 && ck < c0 + nloc) colpos_loc[ck - c0] = colpos_g[ck];
                colpos_loc[nloc] = k;
                st->q = nloc;  // the passes take the pivot column from the ghost
            }
        }
    }
    __syncthreads();
    // the ghost: the winner's stale column and its pending y's (no winner: every trailing value
    // NaN, as the reference's column would be after the division by a NaN pivot)
    const int wr = win_s, own = own_s;
    if (fused) colrecv = recv + (int64_t)(wr >= 0 ? wr : 0) * rstride + kCandWords;  // the winner's column
    double* gcol = A + (int64_t)nloc * lda;
    const double qnan = __longlong_as_double(0x7ff8000000000000LL);
    const double* lcol = A + (int64_t)(own >= 0 ? own : 0) * lda;
    const int i0 = blockIdx.x * 1024 + threadIdx.x;
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // all reads before any write: own may alias nothing, but be safe
        const int i = i0 + u * 256;
        v[u] = qnan;
        if (i < m && wr >= 0) v[u] = colrecv ? bits_dbl(colrecv[kMaxPendR + i]) : lcol[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * 256;
        if (i < m) gcol[i] = v[u];
    }
    if (blockIdx.x == 0 && threadIdx.x < kMaxPendR) {
        const int t = threadIdx.x;
        const double y = wr < 0 ? 0.0 : colrecv ? bits_dbl(colrecv[t]) : Y[(int64_t)t * ldy + own];
        Y[(int64_t)t * ldy + nloc] = y;
    }
}

void launch_shard_commit(hipStream_t s, const uint64_t* recv, int64_t rstride, int nranks, const uint64_t* colrecv,
                         int fused, int m, int k, RrluState* st, double reltol, double abstol, int32_t* rowpos,
                         int32_t* colpos_g, int64_t* rowphys, int64_t* colphys_g, double* pivvals,
                         int32_t* colpos_loc, int64_t c0, int nloc, double* A, int64_t lda, double* Y,
                         int64_t ldy) {
    hipLaunchKernelGGL(k_shard_commit, dim3((m + 1023) / 1024 > 0 ? (m + 1023) / 1024 : 1), dim3(256), 0, s, recv,
                       rstride, nranks, colrecv, fused, m, k, st, reltol, abstol, rowpos, colpos_g, rowphys, colphys_g, pivvals,
                       colpos_loc, c0, nloc, A, lda, Y, ldy);
}

}  // namespace tci

#ifdef TCI_EXPERIMENT_RT
namespace tci {
// register-pressure experiment: one pass with a runtime pending count, no persistent loop
template <bool EXT, bool COH>
__global__ __launch_bounds__(kP2Threads) void k_pass_mf_rt(PassK g, SelArgs sel) {
    __shared__ P2MfLds<kEpochMaxP, EXT> L;
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    CandR best = cand_none();
    const int r = pass_mf_body<kEpochMaxP, EXT, false, COH>(g, sel, L, best, pt, g.ps);
    if (r != kMfDone) return;
    pass_tail<kP2Threads>(best, sel, g.cand, pt, g.m, 1, 0);
}
template __global__ void k_pass_mf_rt<false, false>(PassK, SelArgs);
template __global__ void k_pass_mf_rt<false, true>(PassK, SelArgs);
template __global__ void k_pass_mf_rt<true, true>(PassK, SelArgs);
}  // namespace tci
#endif
