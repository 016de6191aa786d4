// tci_sweep_small.hip -- sweep2site! (tensorci2.jl:1195-1258) resident on the device while every
// bond's Pi fits one workgroup's LDS (the small rrLU of tci_smalllu.h: (m|1) n <= 16384 and
// m + n <= 2048), for the staged integrand kinds. One launch runs niter iterations: per bond the
// kronecker products of the index sets (tensorci2.jl:512-529), Julia's first-seen `union` with
// the previous sweep's sets (:1214-1216), Pi = f(Icomb x Jcomb) evaluated straight into LDS with
// the batched assembly's own arithmetic (tci_funcdev.h), updatemaxsample! (:636-638), the rrLU
// (matrixlu.jl:346-396), the new pivot sets and updateerrors! (:281-289) -- no host round trip
// between bonds (the small configs were bound by ~50 us of host sync per
// bond). A bond that does not fit ends the launch with a resume point; the host loop
// (tci_sweep.cpp) continues from there with the same state. Mode 1 is fillsitetensors!'s
// maxsample update (globalsearch.jl:202-208 with the solve unobservable: max |Pi1| of every site).
//
// State in HBM: six banks of index sets (0 Iset, 1 Jset, then the history and the extra pair,
// whose roles swap per iteration), site p of bank b at ws + off[b L + p], cap entries each;
// per-bond scratch (the concatenated kronecker + extra entries, the combined sets) beside it.
// Host I/O through mapped host memory (SwIO layout, tci_internal.h): read once at the start,
// written once at the end.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tci_funcdev.h"
#include "tci_internal.h"
#include "tci_smalllu.h"

#include <type_traits>

namespace tci {

constexpr int kSwThreads = 256;  // 4 waves, one per SIMD: the small rrLU's per-pivot barriers are cheap
constexpr int kSwWaves = kSwThreads / 64;

// dynamic LDS: S (also the union's scratch) | perms (rows, then columns) | x / y (row / column
// states while Pi is evaluated) | per-wave candidates
constexpr size_t kSwLdsS = (size_t)kSmallElems * 8;
constexpr size_t kSwLdsPerm = (size_t)kSmallPerm * 4;
constexpr size_t kSwLdsXY = (size_t)kSmallPerm * 8;
constexpr size_t kSwLds = kSwLdsS + kSwLdsPerm + kSwLdsXY + kSwWaves * sizeof(SmallCand);
static_assert((size_t)kSwCatCap * 5 <= kSwLdsS, "union scratch (hash + flag per entry) inside S");

__host__ __device__ constexpr size_t sw_al16(size_t b) { return (b + 15) / 16 * 16; }

// dst[0 .. n) = src[0 .. n) by the whole workgroup with kSwCopyB loads in flight per thread (an
// HBM / L2 round trip per kSwCopyB x 256 ints, not one per int)
constexpr int kSwCopyB = 8;
__device__ __forceinline__ void sw_copy(int32_t* dst, const int32_t* src, int n) {
    for (int base = 0; base < n; base += kSwCopyB * kSwThreads) {
        int32_t v[kSwCopyB];
#pragma unroll
        for (int u = 0; u < kSwCopyB; ++u) {
            const int e = base + (int)threadIdx.x + u * kSwThreads;
            v[u] = e < n ? src[e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kSwCopyB; ++u) {
            const int e = base + (int)threadIdx.x + u * kSwThreads;
            if (e < n) dst[e] = v[u];
        }
    }
}

#ifndef TCI_SW_PROF
#define SWP_ACC nullptr
#endif
#ifdef TCI_SW_PROF  // phase profile (thread 0, wall clock ticks): kron+union, Pi, rrLU, selection
#define SWP(i) (swp_t[i] = wall_clock64())
#else
#define SWP(i) ((void)0)
#endif

__device__ __forceinline__ uint32_t sw_hash(const int32_t* e, int w) {
    uint32_t h = 2166136261u;
    for_legs(e, w, [&](int, int32_t x) { h = (h ^ (uint32_t)x) * 16777619u; });
    return h;
}

// e[0 .. w) == f[0 .. w), eight loads of each in flight at a time (a chain of dependent LDS round
// trips per leg otherwise)
__device__ __forceinline__ bool sw_rows_equal(const int32_t* e, const int32_t* f, int w) {
    bool eq = true;
    for (int z0 = 0; z0 < w; z0 += 8) {
        int32_t x[8], y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            x[u] = z0 + u < w ? e[z0 + u] : 0;
            y[u] = z0 + u < w ? f[z0 + u] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) eq = eq && x[u] == y[u];
    }
    return eq;
}

// dst[0 .. w) = src[0 .. w), eight loads in flight
__device__ __forceinline__ void sw_copy_row(int32_t* dst, const int32_t* src, int w) {
    for_legs(src, w, [&](int t, int32_t x) { dst[t] = x; });
}

// exclusive prefix sum of v over the workgroup in thread order; *total gets the sum
__device__ __forceinline__ int sw_scan(int v, int* scr, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) scr[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int q = 0; q < kSwWaves; ++q) {
        const int s = scr[q];
        base += q < w ? s : 0;
        tot += s;
    }
    __syncthreads();  // scr reusable
    *total = tot;
    return base + x - v;
}

// union of the n entries cat[0 .. n) (width w, n <= kSwCatCap): the first occurrence of every
// distinct entry, in order, into dst; returns the count (Julia's union over Vector{MultiIndex},
// the order of tci_sweep.cpp's union_sets)
__device__ int sw_union(const int32_t* __restrict__ cat, int n, int w, int32_t* __restrict__ dst,
                        char* scratch, int* scr) {
    const int tid = threadIdx.x;
    uint32_t* hs = reinterpret_cast<uint32_t*>(scratch);
    unsigned char* keep = reinterpret_cast<unsigned char*>(scratch) + (size_t)n * 4;
    for (int t = tid; t < n; t += kSwThreads) hs[t] = sw_hash(cat + (int64_t)t * w, w);
    __syncthreads();
    for (int t = tid; t < n; t += kSwThreads) {
        const uint32_t h = hs[t];
        const int32_t* et = cat + (int64_t)t * w;
        bool dup = false;
        for (int s = 0; s < t && !dup; ++s) {
            if (hs[s] != h) continue;
            dup = sw_rows_equal(cat + (int64_t)s * w, et, w);
        }
        keep[t] = dup ? 0 : 1;
    }
    __syncthreads();
    // stable compaction: thread tid owns the contiguous chunk [t0, t1)
    const int per = (n + kSwThreads - 1) / kSwThreads;
    const int t0 = min(n, tid * per), t1 = min(n, t0 + per);
    int nk = 0;
    for (int t = t0; t < t1; ++t) nk += keep[t];
    int total;
    int pos = sw_scan(nk, scr, &total);
    for (int t = t0; t < t1; ++t)
        if (keep[t]) {
            sw_copy_row(dst + (int64_t)pos * w, cat + (int64_t)t * w, w);
            ++pos;
        }
    __syncthreads();
    return total;
}

// Julia's max over |v| (NaN-propagating) across the workgroup, as the unsigned maximum of the bit
// patterns of |v| (the batched assembly's block_maxabs order): the same in every thread
__device__ __forceinline__ double sw_maxabs(double mx, unsigned long long* slot) {
    unsigned long long b = (unsigned long long)__double_as_longlong(fabs(mx));
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off);
        b = o > b ? o : b;
    }
    if (threadIdx.x == 0) *slot = 0ull;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicMax(slot, b);
    __syncthreads();
    const double r = __longlong_as_double((long long)*slot);
    __syncthreads();
    return r;
}


// ---- one-wave union (every bond of the small configs: a few dozen entries): the hashes stay in
// registers and are broadcast with readlane, so the duplicate test is a register compare per
// earlier entry, not a chain of dependent LDS loads; the compaction is a ballot prefix
constexpr int kSwWaveU = 512;  // entries a one-wave union takes

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one whole wave: the union of cat[0 .. n) (LDS, width w, n <= kSwWaveU) into dst (LDS), first
// occurrences in order; returns the count (the same in every lane)
__device__ int sw_union_wave(const int32_t* cat, int n, int w, int32_t* dst) {
    constexpr int U = kSwWaveU / 64;
    const int lane = threadIdx.x & 63;
    if (n <= 64) {  // one entry per lane (every bond of the small configs)
        bool keep = lane < n;
        const uint32_t h = keep ? sw_hash(cat + lane * w, w) : 0u;
        // the first earlier entry with the same hash, found in registers; then every lane compares
        // its pair at once (the duplicates are the extra sets' entries already in the kronecker
        // product). A hash collision that is not an equal entry falls back to the remaining
        // earlier entries, one at a time (rare).
        int cand = -1;
        for (int s = 0; s < n - 1; ++s) {
            const uint32_t hs = (uint32_t)__builtin_amdgcn_readlane((int)h, s);
            if (cand < 0 && keep && lane > s && h == hs) cand = s;
        }
        bool fb = false;
        if (cand >= 0) {
            if (sw_rows_equal(cat + cand * w, cat + lane * w, w))
                keep = false;
            else
                fb = true;
        }
        if (__any(fb)) {  // uniform loop: readlane needs every lane
            for (int s = 0; s < n - 1; ++s) {
                const uint32_t hs = (uint32_t)__builtin_amdgcn_readlane((int)h, s);
                if (fb && keep && s > cand && lane > s && h == hs && sw_rows_equal(cat + s * w, cat + lane * w, w))
                    keep = false;
            }
        }
        const uint64_t bal = __ballot(keep);
        if (keep) {
            const int pos = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
            sw_copy_row(dst + pos * w, cat + lane * w, w);
        }
        return __popcll(bal);
    }
    const int nu = (n + 63) >> 6;
    uint32_t h[U];
    bool keep[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = lane + 64 * u;
        keep[u] = t < n;
        h[u] = keep[u] ? sw_hash(cat + t * w, w) : 0u;
    }
#pragma unroll
    for (int su = 0; su < U; ++su) {
        if (su >= nu) break;
        for (int sl = 0; sl < 64; ++sl) {
            const int s = su * 64 + sl;
            if (s >= n) break;
            const uint32_t hs = (uint32_t)__builtin_amdgcn_readlane((int)h[su], sl);
#pragma unroll
            for (int u = su; u < U; ++u) {
                const int t = lane + 64 * u;
                if (u < nu && keep[u] && t > s && h[u] == hs && sw_rows_equal(cat + s * w, cat + t * w, w))
                    keep[u] = false;
            }
        }
    }
    int base = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t bal = __ballot(keep[u]);
        if (keep[u]) {
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
            const int t = lane + 64 * u;
            sw_copy_row(dst + pos * w, cat + t * w, w);
        }
        base += __popcll(bal);
    }
    return base;
}

// ---- register-tile rrLU for m, n <= 64: tci_smalllu.h's algorithm with the matrix in registers
// (thread (tr, tc) of a 16 x 16 grid owns rows tr + 16 a, columns tc + 16 b) and position maps in
// place of the physical swaps -- the same candidates in the same (value, column position, row
// position) order, the same multiply / subtract / divide on the same values, so the same pivots
// and bits. Two barriers per pivot (winner; pivot row / column), no LDS traffic per element.
constexpr int kSwRegN = 64;

// the wave's best candidate (larger abs2, then the smaller key; abs2 is -1 or >= 0, never NaN),
// uniform in every lane: the maximum abs2 by DPP (IEEE max) within rows of 16 and readlane across
// them, then, unless one lane holds it alone, the smallest key among the lanes that hold it --
// a short dependent chain, not the full (value, key, payload) tournament of wave_argmax3
template <int CTRL>
__device__ __forceinline__ unsigned dpp_min_u32(unsigned v) {
    return min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ void wave_best(double& bv, unsigned& bk, double& bx) {
    double m = bv;
    m = fmax(m, dpp_f64<0xb1>(m));
    m = fmax(m, dpp_f64<0x4e>(m));
    m = fmax(m, dpp_f64<0x141>(m));
    m = fmax(m, dpp_f64<0x140>(m));
    const double vmax = fmax(fmax(readlane_f64(m, 0), readlane_f64(m, 16)), fmax(readlane_f64(m, 32), readlane_f64(m, 48)));
    const uint64_t hold = __ballot(bv == vmax);
    int lane;
    if (__popcll(hold) == 1) {
        lane = __builtin_ctzll(hold);
    } else {
        unsigned k = bv == vmax ? bk : 0xffffffffu;
        k = dpp_min_u32<0xb1>(k);
        k = dpp_min_u32<0x4e>(k);
        k = dpp_min_u32<0x141>(k);
        k = dpp_min_u32<0x140>(k);
        const unsigned kmin = min(min((unsigned)__builtin_amdgcn_readlane((int)k, 0), (unsigned)__builtin_amdgcn_readlane((int)k, 16)),
                                  min((unsigned)__builtin_amdgcn_readlane((int)k, 32), (unsigned)__builtin_amdgcn_readlane((int)k, 48)));
        lane = __builtin_ctzll(__ballot(bv == vmax && bk == kmin));
    }
    bk = (unsigned)__builtin_amdgcn_readlane((int)bk, lane);
    bx = readlane_f64(bx, lane);
    bv = vmax;
}

#ifdef TCI_SW_PROF
#define LUP(i)                                                       \
    do {                                                             \
        const unsigned long long t_ = wall_clock64();                \
        if (lup_acc) lup_acc[i] += t_ - lup_t;                       \
        lup_t = t_;                                                  \
    } while (0)
#else
#define LUP(i) ((void)0)
#endif

__device__ int sw_lu_regs(double* S, int ldS, int m, int n, int mr, double reltol, double abstol,
                          int leftorth, int* rowphys, int* colphys, double* xv, double* yv, SmallCand* red,
                          double* pvl, int* nslot, double* dslot, double& error, double& maxerror, int& nanfl,
                          unsigned long long* lup_acc, bool posout = false) {
    (void)lup_acc;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int tr = tid & 15, tc = tid >> 4;
#ifdef TCI_SW_PROF
    unsigned long long lup_t = wall_clock64();
#endif
    double v[4][4];
    int rpos[4], cpos[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) rpos[a] = tr + 16 * a < m ? tr + 16 * a : -1;
#pragma unroll
    for (int b = 0; b < 4; ++b) cpos[b] = tc + 16 * b < n ? tc + 16 * b : -1;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            v[a][b] = (rpos[a] >= 0 && cpos[b] >= 0) ? S[tr + 16 * a + (tc + 16 * b) * ldS] : 0.0;
    for (int i = tid; i < m; i += kSwThreads) rowphys[i] = i;
    for (int j = tid; j < n; j += kSwThreads) colphys[j] = j;
    if (tid == 0) *nslot = 0;
    double bv, bx;
    unsigned bk;
    auto take = [&](double a2, unsigned key, double val) {
        const bool better = (a2 > bv) || (a2 == bv && key < bk);  // NaN never wins
        bv = better ? a2 : bv;
        bk = better ? key : bk;
        bx = better ? val : bx;
    };
    // candidates of the trailing block (positions >= k0): abs2, key = (column << 16 | row) positions
    auto scan = [&](int k0) {
        bv = -1.0;
        bk = 0xffffffffu;
        bx = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (rpos[a] >= k0 && cpos[b] >= k0)
                    take(__dmul_rn(v[a][b], v[a][b]), ((unsigned)cpos[b] << 16) | (unsigned)rpos[a], v[a][b]);
    };
    scan(0);
    maxerror = 0.0;
    error = __longlong_as_double(0x7ff8000000000000LL);
    int np = 0, fl = 0;
    LUP(0);
    for (int k = 0; k < mr; ++k) {
        wave_best(bv, bk, bx);
        LUP(1);
        if (lane == 0) red[w] = SmallCand{bv, bk, 0u, bx};
        __syncthreads();
        LUP(2);
        double cv = red[0].v, cx = red[0].val;
        unsigned ck = red[0].key;
#pragma unroll
        for (int q = 1; q < kSwWaves; ++q) {
            const SmallCand o = red[q];
            const bool t = (o.v > cv) || (o.v == cv && o.key < ck);
            cv = t ? o.v : cv;
            ck = t ? o.key : ck;
            cx = t ? o.val : cx;
        }
        LUP(3);
        int pp = (int)(ck & 0xffffu), qq = (int)(ck >> 16);
        double val = cx;
        if (!(cv >= 0.0)) {  // every trailing value NaN: Julia keeps (k, k)
            pp = qq = k;
            const int r0 = rowphys[k], c0 = colphys[k];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (tr + 16 * a == r0 && tc + 16 * b == c0) *dslot = v[a][b];
            __syncthreads();
            val = *dslot;
        }
        error = fabs(val);
        if (((fabs(error) < reltol * maxerror) || (fabs(error) < abstol)) && k > 0) break;
        maxerror = jl_max(maxerror, error);
        np = k + 1;
        if (tid == 0) pvl[k] = val;
        if (isnan(val)) fl |= 3;  // the pivot sits on both tril and triu
        const int pr = rowphys[pp], pc = colphys[qq];
        LUP(4);
        // swaprow!(k, pp) / swapcol!(k, qq) as position swaps
#pragma unroll
        for (int a = 0; a < 4; ++a) rpos[a] = rpos[a] == k ? pp : (rpos[a] == pp ? k : rpos[a]);
#pragma unroll
        for (int b = 0; b < 4; ++b) cpos[b] = cpos[b] == k ? qq : (cpos[b] == qq ? k : cpos[b]);
        // normalisation (true division) of the pivot column below / pivot row right of the pivot:
        // the owners are one thread column / row, the tile slot b = pc / 16 (a = pr / 16) uniform
        const double piv = val;
        auto norm_col = [&](auto bc) {
            constexpr int b = decltype(bc)::value;
#pragma unroll
            for (int a = 0; a < 4; ++a)
                if (rpos[a] > k) {
                    const double x = leftorth ? v[a][b] / piv : v[a][b];
                    v[a][b] = x;
                    xv[tr + 16 * a] = x;
                    fl |= isnan(x) ? 1 : 0;
                }
        };
        auto norm_row = [&](auto ac) {
            constexpr int a = decltype(ac)::value;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (cpos[b] > k) {
                    const double y = leftorth ? v[a][b] : v[a][b] / piv;
                    v[a][b] = y;
                    yv[tc + 16 * b] = y;
                    fl |= isnan(y) ? 2 : 0;
                }
        };
        if (tc == (pc & 15)) {
            switch (pc >> 4) {
            case 0: norm_col(std::integral_constant<int, 0>{}); break;
            case 1: norm_col(std::integral_constant<int, 1>{}); break;
            case 2: norm_col(std::integral_constant<int, 2>{}); break;
            default: norm_col(std::integral_constant<int, 3>{}); break;
            }
        }
        if (tr == (pr & 15)) {
            switch (pr >> 4) {
            case 0: norm_row(std::integral_constant<int, 0>{}); break;
            case 1: norm_row(std::integral_constant<int, 1>{}); break;
            case 2: norm_row(std::integral_constant<int, 2>{}); break;
            default: norm_row(std::integral_constant<int, 3>{}); break;
            }
        }
        LUP(5);
        __syncthreads();
        LUP(6);
        if (tid == 0) {
            int t = rowphys[k];
            rowphys[k] = rowphys[pp];
            rowphys[pp] = t;
            t = colphys[k];
            colphys[k] = colphys[qq];
            colphys[qq] = t;
        }
        // rank-1 update of the trailing block (mul then sub), then the next pivot's candidates
        double xr[4], yc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) xr[a] = rpos[a] > k ? xv[tr + 16 * a] : 0.0;
#pragma unroll
        for (int b = 0; b < 4; ++b) yc[b] = cpos[b] > k ? yv[tc + 16 * b] : 0.0;
        bv = -1.0;
        bk = 0xffffffffu;
        bx = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (rpos[a] > k && cpos[b] > k) {
                    const double nv = __dsub_rn(v[a][b], __dmul_rn(xr[a], yc[b]));
                    v[a][b] = nv;
                    take(__dmul_rn(nv, nv), ((unsigned)cpos[b] << 16) | (unsigned)rpos[a], nv);
                }
        LUP(7);
    }
    LUP(8);
    // tril(A[:, 1:np]) / triu(A[1:np, :]) NaN checks (matrixlu.jl:376-381): their entries are the
    // pivots and the normalised column / row values, flagged as they were made
    if (fl) atomicOr(nslot, fl);
    if (posout) {
        // the packed factors in position order into S (what small_lu_core's physical swaps leave
        // there), for the MatrixLUCI factors: every tile was read at the start, barriers since
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (rpos[a] >= 0 && cpos[b] >= 0) S[rpos[a] + cpos[b] * ldS] = v[a][b];
    }
    __syncthreads();  // also publishes thread 0's last position swap (and the position-order S)
    nanfl = *nslot;
    LUP(9);
    return np;
}

// ---- one-wave rrLU for m, n <= 64 (the bonds of C3 / C4): sw_lu_regs's algorithm on ONE wave,
// lane (tr, tc) of an 8 x 8 grid owning rows tr + 8 a and columns tc + 8 b (a, b < TILE: 4 for
// m, n <= 32, 8 for <= 64; the kernel runs one 256-thread workgroup, so a lane may hold 64 doubles).
// The winner is found by DPP + readlane and is then uniform in every lane, so a pivot needs no
// workgroup barrier: the pivot column / row go through LDS under wave-level fences only
// (wave_sync). The same candidates in the same (abs2, column position, row position) order, the same
// true division and separate multiply / subtract on the same values as sw_lu_regs, hence the same
// pivots and bits. The other waves wait at the closing barrier.
constexpr int kSwWaveN = 64;

// x / p for a divisor p shared by many x, bitwise the IEEE quotient: with y = RN(1 / p) computed
// once, q = RN(x y), r = x - p q (exact, one fma) and RN(q + r y) is the correctly rounded x / p
// (Markstein's theorem) while no intermediate is subnormal or overflows -- |x|, |p| in
// [2^-400, 2^400], x != 0 (pok: the test on p, once per pivot); otherwise the true division. No
// v_div_scale / v_div_fmas, hence no VCC chain: a lane's divisions overlap (the normalisation of a
// pivot column was ~0.57 us of a C4 pivot's ~1.6 us). oracle/tci_oracle.c orc_div_shared_check
// compares the sequence with x / p on random and edge-case operands (tests/test_oracle_kats.py).
__device__ __forceinline__ bool div_shared_ok(double p) {
    const double ap = fabs(p);
    return ap >= 0x1p-400 && ap <= 0x1p400;
}
__device__ __forceinline__ double div_shared(double x, double p, double y, bool pok) {
    const double ax = fabs(x);
    if (pok && ax >= 0x1p-400 && ax <= 0x1p400) {  // (false for NaN and 0)
        const double q = __dmul_rn(x, y);
        const double r = __fma_rn(-p, q, x);
        return __fma_rn(r, y, q);
    }
    return x / p;
}

template <int TILE>
__device__ int sw_lu_wave(double* S, int ldS, int m, int n, int mr, double reltol, double abstol, int leftorth,
                          int* rowphys, int* colphys, double* xv, double* yv, SmallCand* red, double* pvl,
                          int* nslot, double* dslot, double& error, double& maxerror, int& nanfl,
                          bool posout = false, unsigned long long* lup_acc = nullptr) {
    static_assert(8 * TILE <= kSwWaveN, "tile");
    const int tid = threadIdx.x;
#ifdef TCI_SW_PROF
    unsigned long long lup_t = wall_clock64();
#endif
    if (tid < 64) {
        const int lane = tid, tr = lane & 7, tc = lane >> 3;
        double v[TILE][TILE];
        int rpos[TILE], cpos[TILE];
#pragma unroll
        for (int a = 0; a < TILE; ++a) rpos[a] = tr + 8 * a < m ? tr + 8 * a : -1;
#pragma unroll
        for (int b = 0; b < TILE; ++b) cpos[b] = tc + 8 * b < n ? tc + 8 * b : -1;
#pragma unroll
        for (int a = 0; a < TILE; ++a)
#pragma unroll
            for (int b = 0; b < TILE; ++b)
                v[a][b] = (rpos[a] >= 0 && cpos[b] >= 0) ? S[tr + 8 * a + (tc + 8 * b) * ldS] : 0.0;
        if (lane < m) rowphys[lane] = lane;
        if (lane < n) colphys[lane] = lane;
        if (lane == 0) *nslot = 0;
        double bv, bx;
        unsigned bk;
        auto take = [&](double a2, unsigned key, double val) {
            const bool better = (a2 > bv) || (a2 == bv && key < bk);  // NaN never wins
            bv = better ? a2 : bv;
            bk = better ? key : bk;
            bx = better ? val : bx;
        };
        bv = -1.0;
        bk = 0xffffffffu;
        bx = 0.0;
#pragma unroll
        for (int a = 0; a < TILE; ++a)
#pragma unroll
            for (int b = 0; b < TILE; ++b)
                if (rpos[a] >= 0 && cpos[b] >= 0)
                    take(__dmul_rn(v[a][b], v[a][b]), ((unsigned)cpos[b] << 16) | (unsigned)rpos[a], v[a][b]);
        double mxe = 0.0, err = __longlong_as_double(0x7ff8000000000000LL);
        int np = 0, fl = 0;
        wave_sync();
        LUP(0);
        for (int k = 0; k < mr; ++k) {
            wave_best(bv, bk, bx);  // uniform from here on
            LUP(1);
            int pp = (int)(bk & 0xffffu), qq = (int)(bk >> 16);
            double val = bx;
            if (!(bv >= 0.0)) {  // every trailing value NaN: Julia keeps (k, k)
                pp = qq = k;
                const int r0 = rowphys[k], c0 = colphys[k];
#pragma unroll
                for (int a = 0; a < TILE; ++a)
#pragma unroll
                    for (int b = 0; b < TILE; ++b)
                        if (tr + 8 * a == r0 && tc + 8 * b == c0) *dslot = v[a][b];
                wave_sync();
                val = *dslot;
            }
            err = fabs(val);
            if (((fabs(err) < reltol * mxe) || (fabs(err) < abstol)) && k > 0) break;
            mxe = jl_max(mxe, err);
            np = k + 1;
            if (lane == 0) pvl[k] = val;
            if (isnan(val)) fl |= 3;  // the pivot sits on both tril and triu
            const int pr = rowphys[pp], pc = colphys[qq];
#pragma unroll
            for (int a = 0; a < TILE; ++a) rpos[a] = rpos[a] == k ? pp : (rpos[a] == pp ? k : rpos[a]);
#pragma unroll
            for (int b = 0; b < TILE; ++b) cpos[b] = cpos[b] == k ? qq : (cpos[b] == qq ? k : cpos[b]);
            LUP(2);
            // normalisation (true division) of the pivot column / row by their owners: lane column
            // pc mod 8 holds physical column pc in slot pc / 8 (uniform), lane row pr mod 8 row pr
            const double piv = val;
            const bool pok = div_shared_ok(piv);
            const double rpiv = 1.0 / piv;  // (uniform; used only when pok)
            const int bsel = pc >> 3, asel = pr >> 3;
            if (tc == (pc & 7)) {
#pragma unroll
                for (int b = 0; b < TILE; ++b)
                    if (b == bsel) {
#pragma unroll
                        for (int a = 0; a < TILE; ++a)
                            if (rpos[a] > k) {
                                const double x = leftorth ? div_shared(v[a][b], piv, rpiv, pok) : v[a][b];
                                v[a][b] = x;
                                xv[tr + 8 * a] = x;
                                fl |= isnan(x) ? 1 : 0;
                            }
                    }
            }
            if (tr == (pr & 7)) {
#pragma unroll
                for (int a = 0; a < TILE; ++a)
                    if (a == asel) {
#pragma unroll
                        for (int b = 0; b < TILE; ++b)
                            if (cpos[b] > k) {
                                const double y = leftorth ? v[a][b] : div_shared(v[a][b], piv, rpiv, pok);
                                v[a][b] = y;
                                yv[tc + 8 * b] = y;
                                fl |= isnan(y) ? 2 : 0;
                            }
                    }
            }
            LUP(3);
            wave_sync();
            if (lane == 0) {
                int t = rowphys[k];
                rowphys[k] = rowphys[pp];
                rowphys[pp] = t;
                t = colphys[k];
                colphys[k] = colphys[qq];
                colphys[qq] = t;
            }
            double xr[TILE], yc[TILE];
#pragma unroll
            for (int a = 0; a < TILE; ++a) xr[a] = rpos[a] > k ? xv[tr + 8 * a] : 0.0;
#pragma unroll
            for (int b = 0; b < TILE; ++b) yc[b] = cpos[b] > k ? yv[tc + 8 * b] : 0.0;
            LUP(4);
            bv = -1.0;
            bk = 0xffffffffu;
            bx = 0.0;
#pragma unroll
            for (int a = 0; a < TILE; ++a)
#pragma unroll
                for (int b = 0; b < TILE; ++b)
                    if (rpos[a] > k && cpos[b] > k) {
                        const double nv = __dsub_rn(v[a][b], __dmul_rn(xr[a], yc[b]));
                        v[a][b] = nv;
                        take(__dmul_rn(nv, nv), ((unsigned)cpos[b] << 16) | (unsigned)rpos[a], nv);
                    }
            LUP(5);
            wave_sync();  // this pivot's xv / yv reads before the next pivot's writes
            LUP(6);
        }
        LUP(7);
        if (fl) atomicOr(nslot, fl);
        if (posout) {
#pragma unroll
            for (int a = 0; a < TILE; ++a)
#pragma unroll
                for (int b = 0; b < TILE; ++b)
                    if (rpos[a] >= 0 && cpos[b] >= 0) S[rpos[a] + cpos[b] * ldS] = v[a][b];
        }
        if (lane == 0) red[0] = SmallCand{err, (unsigned)np, 0u, mxe};
    }
    __syncthreads();  // the permutations, pivots, flags, position-order S and the results
    nanfl = *nslot;
    error = red[0].v;
    maxerror = red[0].val;
    const int np = (int)red[0].key;
    __syncthreads();  // red[] is reused by the caller
    LUP(8);
    return np;
}

// dispatch by size: 4 x 4 tiles per lane up to 32, 8 x 8 up to 64
__device__ __forceinline__ int sw_lu_wave_any(double* S, int ldS, int m, int n, int mr, double reltol, double abstol,
                                              int leftorth, int* rowphys, int* colphys, double* xv, double* yv,
                                              SmallCand* red, double* pvl, int* nslot, double* dslot, double& error,
                                              double& maxerror, int& nanfl, bool posout = false,
                                              unsigned long long* lup_acc = nullptr) {
    if (m <= 32 && n <= 32)
        return sw_lu_wave<4>(S, ldS, m, n, mr, reltol, abstol, leftorth, rowphys, colphys, xv, yv, red, pvl, nslot,
                             dslot, error, maxerror, nanfl, posout, lup_acc);
    return sw_lu_wave<8>(S, ldS, m, n, mr, reltol, abstol, leftorth, rowphys, colphys, xv, yv, red, pvl, nslot,
                         dslot, error, maxerror, nanfl, posout, lup_acc);
}

// ---- the kernel
// Index-set slots: every site has three slots per kind (I / J), physical banks 2 s (I) and 2 s + 1
// (J) of slot s; per site the roles current / history / extra point at slots. An iteration's
// history is its starting sets (tensorci2.jl:1211-1212): history := current (no copy, the slot is
// shared until the site is written), extra := the old history; a bond writes its new set into the
// slot that is neither the history nor the extra (copy-on-write). The host's image arrives as
// current = slot 0, history = slot 1.
__device__ __forceinline__ int sw_other(int h, int e) { return h != e ? 3 - h - e : (h + 1) % 3; }

// ---- setsitetensor!'s solve (tensorci2.jl:620-627): T = transpose(transpose(P) \ transpose(Pi1)),
// LAPACK getrf / getrs of P^T with partial pivoting, each element's operations in the order of the
// oracle's restatement (oracle/tci_oracle.c orc_sitetensor_solve).
// getrf of A = P^T (r x r, ld r, LDS; r <= 64) by one wave, lane i owning row i: per column k the
// first maximal |a| at or below the diagonal (a NaN on the diagonal keeps k; NaNs below never win,
// as the oracle's strict '>' scan), the interchange of whole rows, the column divided by the pivot,
// the rank-1 update (a separate multiply and subtract). piv[k] (LDS): the row swapped with k.
__device__ void sw_getrf_wave(double* A, int r, int* piv) {
    const int i = threadIdx.x & 63;
    for (int k = 0; k < r; ++k) {
        const double v = (i >= k && i < r) ? fabs(A[i + k * r]) : -1.0;
        const double vk = readlane_f64(v, k);
        int p = k;
        if (!isnan(vk)) {
            double bv = (i >= k && i < r && !isnan(v)) ? v : -1.0, bx = 0.0;
            unsigned bk = (unsigned)i;
            wave_best(bv, bk, bx);  // the largest |a|, then the smallest row
            p = (int)bk;
        }
        if (i == 0) piv[k] = p;
        if (p != k && i < r) {  // lane i: column i of rows k and p
            const double t = A[k + i * r];
            A[k + i * r] = A[p + i * r];
            A[p + i * r] = t;
        }
        wave_sync();
        const double d = A[k + k * r];
        if (i > k && i < r) {
            const double l = A[i + k * r] / d;
            A[i + k * r] = l;
            for (int j = k + 1; j < r; ++j) A[i + j * r] = __dsub_rn(A[i + j * r], __dmul_rn(l, A[k + j * r]));
        }
        wave_sync();
    }
}

// getrs with the factors of sw_getrf_wave: every right-hand side c (a row of Pi1, R x r, ld R, in
// place -- it becomes the row of T) by one thread: the interchanges, the unit lower solve, the upper
// solve with true division. RB >= r: the solution vector in registers (constant indices: the
// interchanges as selects); RB = 0: in LDS (r > 32).
template <int RB>
__device__ void sw_getrs_rows(double* X, int R, int r, const double* A, const int* piv) {
    for (int c = threadIdx.x; c < R; c += kSwThreads) {
        double* x = X + c;
        if constexpr (RB > 0) {
            double v[RB];
#pragma unroll
            for (int i = 0; i < RB; ++i) v[i] = i < r ? x[(int64_t)i * R] : 0.0;
            // (guards instead of break / continue: the loops must unroll for v[] to stay in registers)
#pragma unroll
            for (int k = 0; k < RB; ++k) {
                const int pk = k < r ? piv[k] : k;
#pragma unroll
                for (int i = k + 1; i < RB; ++i)
                    if (i == pk) {
                        const double t = v[k];
                        v[k] = v[i];
                        v[i] = t;
                    }
            }
#pragma unroll
            for (int k = 0; k < RB; ++k) {
#pragma unroll
                for (int i = k + 1; i < RB; ++i)
                    if (i < r) v[i] = __dsub_rn(v[i], __dmul_rn(A[i + k * r], v[k]));
            }
#pragma unroll
            for (int k = RB - 1; k >= 0; --k) {
                if (k < r) {
                    v[k] = v[k] / A[k + k * r];
#pragma unroll
                    for (int i = 0; i < RB; ++i)
                        if (i < k) v[i] = __dsub_rn(v[i], __dmul_rn(A[i + k * r], v[k]));
                }
            }
#pragma unroll
            for (int i = 0; i < RB; ++i)
                if (i < r) x[(int64_t)i * R] = v[i];
        } else {
            for (int k = 0; k < r; ++k)
                if (piv[k] != k) {
                    const double t = x[(int64_t)k * R];
                    x[(int64_t)k * R] = x[(int64_t)piv[k] * R];
                    x[(int64_t)piv[k] * R] = t;
                }
            for (int k = 0; k < r; ++k) {
                const double xk = x[(int64_t)k * R];
                for (int i = k + 1; i < r; ++i) x[(int64_t)i * R] = __dsub_rn(x[(int64_t)i * R], __dmul_rn(A[i + k * r], xk));
            }
            for (int k = r - 1; k >= 0; --k) {
                const double xk = x[(int64_t)k * R] / A[k + k * r];
                x[(int64_t)k * R] = xk;
                for (int i = 0; i < k; ++i) x[(int64_t)i * R] = __dsub_rn(x[(int64_t)i * R], __dmul_rn(A[i + k * r], xk));
            }
        }
    }
}

template <int KIND>
__global__ __launch_bounds__(kSwThreads) void k_sweep_small(SweepSmallArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* S = reinterpret_cast<double*>(smem);
    int* perm = reinterpret_cast<int*>(smem + kSwLdsS);
    double* xy = reinterpret_cast<double*>(smem + kSwLdsS + kSwLdsPerm);
    SmallCand* red = reinterpret_cast<SmallCand*>(smem + kSwLdsS + kSwLdsPerm + kSwLdsXY);
    __shared__ int cnt[6 * kSwMaxL];                    // set counts per physical bank and site
    __shared__ unsigned char rol[2][3][kSwMaxL];        // [I / J][current / history / extra][site] -> slot
    __shared__ int ldm[kSwMaxL];                        // localdims
    __shared__ double bonderr[kSwMaxL];
    __shared__ double pe[kSwPE];                        // pivoterrors of the current iteration
    __shared__ double pvl[kSwPE];                       // the bond's pivot values
    __shared__ int scr[kSwWaves + 4];
    __shared__ unsigned long long mxs;
    __shared__ int nanflag;
    __shared__ int mn[2];
    __shared__ int xsel[2][64];  // lazy union: the kept extras (I / J side), in order
    __shared__ double dslot;
    __shared__ int64_t hdr[16];

    const int tid = threadIdx.x;
    const int L = a.L;
    const FuncDev& f = a.f;
    const double* p = f.params;
    const double p0 = (KIND == F_SUM || KIND == F_TABLE) ? 0.0 : p[0];
    const SwIO io = sw_io(L);
    if (a.ctl) {  // chained optimize!: nothing after the stop (the closing sweep only after a clean end)
        const unsigned long long stop = __hip_atomic_load(&a.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.opt_it > 0 ? stop != 0 : stop != 1) {
            if (tid == 0 && a.fmap) a.fmap[0] = 0;
            return;
        }
    }
#ifdef TCI_SW_PROF
    unsigned long long lu_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define SWP_ACC lu_acc
    unsigned long long swp_t[8] = {0, 0, 0, 0, 0, 0, 0, 0}, swp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int swp_n = 0, swp_piv = 0;
    const unsigned long long swp_c0 = clock64(), swp_w0 = wall_clock64();
#endif
    const int64_t half = (int64_t)L * (L - 1) / 2;
    auto width = [&](int bank, int site) { return (bank & 1) ? L - 1 - site : site; };
    // bank b, site p at ws + cap (b half + sum of the widths before p) (the host's layout)
    auto bank_ptr = [&](int bank, int site) -> int32_t* {
        const int64_t pre = (bank & 1) ? (int64_t)site * (L - 1) - (int64_t)site * (site - 1) / 2
                                       : (int64_t)site * (site - 1) / 2;
        return a.ws + a.cap * (bank * half + pre);
    };
    // logical role r (0 current, 1 history, 2 extra) of kind k (0 I, 1 J) at a site
    auto bank_of = [&](int k, int r, int site) { return 2 * (int)rol[k][r][site] + k; };
    auto set_ptr = [&](int k, int r, int site) { return bank_ptr(bank_of(k, r, site), site); };
    auto set_cnt = [&](int k, int r, int site) -> int& { return cnt[bank_of(k, r, site) * kSwMaxL + site]; };
    // Copies between the packed image (segments bank-major, site-minor, ne(i) ints each) and the set
    // slots: the packed offsets by one workgroup scan (two segments per thread), then every wave
    // copies segments wave, wave + 4, ... two at a time with all their loads in flight -- a few
    // round trips per launch instead of one per segment (up to 6 L of them, each ~1 us).
    __shared__ int segoff[6 * kSwMaxL];
    auto copy_segments = [&](int nseg, auto ne_of, auto src_of, auto dst_of) {
        {
            const int i0 = 2 * tid, i1 = i0 + 1;
            const int n0 = i0 < nseg ? ne_of(i0) : 0, n1 = i1 < nseg ? ne_of(i1) : 0;
            int total;
            const int o = sw_scan(n0 + n1, scr, &total);
            if (i0 < nseg) segoff[i0] = o;
            if (i1 < nseg) segoff[i1] = o + n0;
        }
        __syncthreads();
        const int lane = tid & 63, w = tid >> 6;
        for (int sg = w; sg < nseg; sg += 2 * kSwWaves) {
            const int sa = sg, sb = sg + kSwWaves;
            const int na = ne_of(sa), nb = sb < nseg ? ne_of(sb) : 0;
            const int32_t* pa = src_of(sa, segoff[sa]);
            const int32_t* pb = sb < nseg ? src_of(sb, segoff[sb]) : pa;
            int32_t* da = dst_of(sa, segoff[sa]);
            int32_t* db = sb < nseg ? dst_of(sb, segoff[sb]) : da;
            for (int base = 0; base < max(na, nb); base += 4 * 64) {
                int32_t va[4], vb[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = base + lane + 64 * u;
                    va[u] = e < na ? pa[e] : 0;
                    vb[u] = e < nb ? pb[e] : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int e = base + lane + 64 * u;
                    if (e < na) da[e] = va[u];
                    if (e < nb) db[e] = vb[u];
                }
            }
        }
    };

    // ---- input (DMA'd to a.inbuf by the host): header, counts, bond errors, the four banks. The
    // closing sweep of a chain, enqueued before the host knows where the loop stops, takes the image
    // of the stop iteration ctl[1] (iteration i's image is img_sel[i & 1]).
    const char* inb = a.inbuf;
    if (a.ctl && a.opt_it < 0 && a.img_sel[0])
        inb = a.img_sel[__hip_atomic_load(&a.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1];
    if (tid < 16) hdr[tid] = reinterpret_cast<const int64_t*>(inb)[tid];
    for (int i = tid; i < 6 * L; i += kSwThreads)
        cnt[(i / L) * kSwMaxL + i % L] = i < 4 * L ? (int)reinterpret_cast<const int64_t*>(inb + io.counts)[i] : 0;
    for (int i = tid; i < L - 1; i += kSwThreads) bonderr[i] = reinterpret_cast<const double*>(inb + io.bonderr)[i];
    for (int i = tid; i < L; i += kSwThreads) {
        ldm[i] = f.localdims[i];
        for (int k = 0; k < 2; ++k)
            for (int r = 0; r < 3; ++r) rol[k][r][i] = (unsigned char)r;
    }
    __syncthreads();
    {
        const int32_t* src = reinterpret_cast<const int32_t*>(inb + io.sets);
        copy_segments(
            4 * L, [&](int i) { return cnt[(i / L) * kSwMaxL + i % L] * width(i / L, i % L); },
            [&](int, int off) { return src + off; }, [&](int i, int) { return bank_ptr(i / L, i % L); });
    }
    int has_history = (int)hdr[3];
    double maxsample = __longlong_as_double((long long)hdr[6]);
    if (a.fmax_in) {  // chained: the previous iteration's fill (|v| bits: Julia's NaN-propagating max)
        unsigned long long mb = (unsigned long long)hdr[6] & 0x7fffffffffffffffull;
        for (int q = 0; q < L; ++q) {
            const unsigned long long v = a.fmax_in[q];
            mb = v > mb ? v : mb;
        }
        maxsample = __longlong_as_double((long long)mb);
    }
    // optimize!'s abstol = tol * errornormalization (tensorci2.jl:1049-1050) in a chain
    const double abstol = a.ctl ? (a.opt_norm ? a.opt_tol * maxsample : a.opt_tol) : a.abstol;
    if (a.ctl && a.opt_it < 0 && tid == 0) {
        a.ctl[2] = (unsigned long long)__double_as_longlong(maxsample);
        a.ctl[3] = (unsigned long long)__double_as_longlong(abstol);
    }
    int npe = 0;
    int status = 0, s_it = 0, s_q = 0, esite = 0, extra_valid = 0, fstatus = -1, fsite = 0;
    __syncthreads();

    if (a.mode == 0) {
        for (int it = a.iter1; it < a.iter1 + a.niter && status == 0; ++it) {
            const bool extra = !a.strictlynested && has_history;
            for (int i = tid; i < L; i += kSwThreads)
                for (int k = 0; k < 2; ++k) {
                    if (extra) rol[k][2][i] = rol[k][1][i];  // extra := the previous history
                    rol[k][1][i] = rol[k][0][i];             // history := the current sets
                }
            has_history = 1;
            extra_valid = extra;
            npe = 0;  // flushpivoterror!
            __syncthreads();
            const bool fwd = a.strategy == 1 || (a.strategy == 0 && it % 2 == 1);
            for (int q = 1; q < L; ++q) {
                const int b = fwd ? q : L - q;  // 1-based bond
                SWP(0);
                // Icomb = union(kronecker(Iset[b-1], d), extra Iset[b]) (width b);
                // Jcomb = union(kronecker(d, Jset[b]), extra Jset[b-1]) (width L - b)
                const int dI = ldm[b - 1], nI = set_cnt(0, 0, b - 1), wI0 = b - 1;
                const int neI = extra ? set_cnt(0, 2, b) : 0;
                const int dJ = ldm[b], nJ = set_cnt(1, 0, b), wJ0 = L - 1 - b, wJ1 = wJ0 + 1;
                const int neJ = extra ? set_cnt(1, 2, b - 1) : 0;
                const int catI = nI * dI + neI, catJ = nJ * dJ + neJ;
                const int gI = nI * wI0, gJ = nJ * wJ0, gEI = neI * b, gEJ = neJ * wJ1;  // staged ints
                // LDS: [staged sources | concatenation I | concatenation J | hash / flags] at the
                // bottom of S, Icomb / Jcomb at its top (below them, later, Pi)
                const size_t bI = sw_al16((size_t)catI * b * 4), bJ = sw_al16((size_t)catJ * wJ1 * 4);
                const size_t bG = sw_al16((size_t)(gI + gJ + gEI + gEJ) * 4);
                const size_t bH = sw_al16((size_t)max(catI, catJ) * 5);
                const bool room = catI <= kSwCatCap && catJ <= kSwCatCap && nI * dI <= kSmallPerm &&
                                  nJ * dJ <= kSmallPerm && bG + 2 * (bI + bJ) + bH <= kSwLdsS;
                char* const R = reinterpret_cast<char*>(S);
                int32_t* const gs = reinterpret_cast<int32_t*>(R);
                int32_t* const catIp = reinterpret_cast<int32_t*>(R + bG);
                int32_t* const catJp = reinterpret_cast<int32_t*>(R + bG + bI);
                char* const uscr = R + bG + bI + bJ;
                int32_t* Ic = reinterpret_cast<int32_t*>(R + kSwLdsS - bI - bJ);
                int32_t* Jc = reinterpret_cast<int32_t*>(R + kSwLdsS - bJ);
                int m = 0, n = 0;
                // Lazy union (round 6): the kronecker products are not materialised. Their entries are
                // distinct (Iset / Jset are sets), so union(kron, extra) keeps every kron entry in order
                // and appends the extras that are neither in the kron product nor earlier extras: only
                // the <= 64 extras are hashed and compared (an extra [I..., j] is a kron entry iff
                // 1 <= j <= d and its prefix is an Iset entry; [i, J...] likewise), and rows, states
                // and the new sets are read from the staged sources by descriptor. The sources stay
                // staged (top of S) until the selection; Pi lives below them. Same entries in the
                // same order as the materialised union, hence the same Pi and pivots. Taken where a leg
                // has d >= 4: with d = 2 (quantics) the materialised kron is a couple of row copies and
                // the materialised path was faster (C4 9.2 vs 9.85 ms; C1 d = 10 6.0 -> 5.1 ms).
                const bool lzu = a.lazy_union && max(dI, dJ) >= 4 && nI <= 64 && neI <= 64 && nJ <= 64 && neJ <= 64 && bG <= kSwLdsS / 2;
                const int KI = nI * dI, KJ = nJ * dJ;
                int32_t* const gsl = reinterpret_cast<int32_t*>(R + kSwLdsS - bG);
                // the four source sets into LDS (dst) in one batched round of loads
                auto stage = [&](int32_t* dst) {
                    const int32_t* s0 = set_ptr(0, 0, b - 1);
                    const int32_t* s1 = set_ptr(1, 0, b);
                    const int32_t* s2 = set_ptr(0, 2, b);
                    const int32_t* s3 = set_ptr(1, 2, b - 1);
                    const int n01 = gI + gJ, n012 = n01 + gEI, tot = n012 + gEJ;
                    for (int base = 0; base < tot; base += kSwCopyB * kSwThreads) {
                        int32_t v[kSwCopyB];
#pragma unroll
                        for (int u = 0; u < kSwCopyB; ++u) {
                            const int e = base + tid + u * kSwThreads;
                            v[u] = e < gI ? s0[e] : e < n01 ? s1[e - gI] : e < n012 ? s2[e - n01] : e < tot ? s3[e - n012] : 0;
                        }
#pragma unroll
                        for (int u = 0; u < kSwCopyB; ++u) {
                            const int e = base + tid + u * kSwThreads;
                            if (e < tot) dst[e] = v[u];
                        }
                    }
                };
                if (lzu) {
                    stage(gsl);
                    __syncthreads();
                    SWP(5);
                    const int wv = tid >> 6, ln = tid & 63;
                    if (wv < 2) {  // wave 0: the I side, wave 1: the J side
                        const bool sideI = wv == 0;
                        const int nk = sideI ? nI : nJ, ne = sideI ? neI : neJ, dk = sideI ? dI : dJ;
                        const int wk = sideI ? wI0 : wJ0, we = wk + 1;
                        const int32_t* K = sideI ? gsl : gsl + gI;                   // Iset[b-1] / Jset[b]
                        const int32_t* E = sideI ? gsl + gI + gJ : gsl + gI + gJ + gEI;  // the extras
                        const int32_t* et = E + ln * we;
                        bool keep = ln < ne;
                        // the extra's leg on the kron side (last for I, first for J) and its other legs
                        const int leg = keep ? (sideI ? et[wk] : et[0]) : 0;
                        const int32_t* rest = sideI ? et : et + 1;
                        const uint32_t hr = keep ? sw_hash(rest, wk) : 0u;         // vs the kron sources
                        const uint32_t hf = (hr ^ (uint32_t)leg) * 16777619u;      // (rest, leg): vs earlier extras
                        const uint32_t hk = ln < nk ? sw_hash(K + ln * wk, wk) : 0u;
                        // in the kron product? (readlane reads lane s2 whatever the exec mask)
                        const bool kin = keep && leg >= 1 && leg <= dk;
                        for (int s2 = 0; s2 < nk; ++s2) {
                            const uint32_t h2 = (uint32_t)__builtin_amdgcn_readlane((int)hk, s2);
                            if (kin && keep && h2 == hr && sw_rows_equal(K + s2 * wk, rest, wk)) keep = false;
                        }
                        for (int s2 = 0; s2 < ne - 1; ++s2) {  // an equal earlier extra
                            const uint32_t h2 = (uint32_t)__builtin_amdgcn_readlane((int)hf, s2);
                            if (keep && s2 < ln && h2 == hf && sw_rows_equal(E + s2 * we, et, we)) keep = false;
                        }
                        const uint64_t bal = __ballot(keep);
                        if (keep) {
                            const int pos = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                          __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                            (sideI ? xsel[0] : xsel[1])[pos] = ln;
                        }
                        if (ln == 0) mn[wv] = __popcll(bal);
                    }
                    __syncthreads();
                    m = KI + mn[0];
                    n = KJ + mn[1];
                } else if (room) {
                    stage(gs);
                    __syncthreads();
                    SWP(5);
                    const int32_t* Ib = gs;
                    const int32_t* Jb = gs + gI;
                    const int32_t* Ex = gs + gI + gJ;
                    const int32_t* Ey = gs + gI + gJ + gEI;
                    const bool wunion = catI <= kSwWaveU && catJ <= kSwWaveU;
                    auto build_I = [&](int t0, int stride) {
                        for (int e = t0; e < nI * dI; e += stride) {
                            const int i = e % nI, j = e / nI;
                            int32_t* o = catIp + e * b;
                            sw_copy_row(o, Ib + i * wI0, wI0);
                            o[wI0] = j + 1;
                        }
                        for (int e = t0; e < gEI; e += stride) catIp[nI * dI * b + e] = Ex[e];
                    };
                    auto build_J = [&](int t0, int stride) {
                        for (int e = t0; e < nJ * dJ; e += stride) {
                            const int i = e % dJ, jj = e / dJ;
                            int32_t* o = catJp + e * wJ1;
                            o[0] = i + 1;
                            sw_copy_row(o + 1, Jb + jj * wJ0, wJ0);
                        }
                        for (int e = t0; e < gEJ; e += stride) catJp[nJ * dJ * wJ1 + e] = Ey[e];
                    };
                    if (wunion) {  // waves 0 and 1 at once
                        const int wv = tid >> 6, ln = tid & 63;
                        if (wv == 0) {
                            build_I(ln, 64);
                            wave_sync();
                            const int c = sw_union_wave(catIp, catI, b, Ic);
                            if (ln == 0) mn[0] = c;
                        } else if (wv == 1) {
                            build_J(ln, 64);
                            wave_sync();
                            const int c = sw_union_wave(catJp, catJ, wJ1, Jc);
                            if (ln == 0) mn[1] = c;
                        }
                        __syncthreads();
                        m = mn[0];
                        n = mn[1];
                    } else {
                        build_I(tid, kSwThreads);
                        build_J(tid, kSwThreads);
                        __syncthreads();
                        m = sw_union(catIp, catI, b, Ic, uscr, scr);
                        n = sw_union(catJp, catJ, wJ1, Jc, uscr, scr);
                    }
                }
                const bool fits = m > 0 && n > 0 && (int64_t)(m | 1) * n <= kSmallElems && m + n <= kSmallPerm;  // rrlu_small_fits
                const int ldS = m | 1;
                if (!(room || lzu) || !fits || a.maxbonddim <= 0 ||
                    (size_t)ldS * n * 8 > (lzu ? kSwLdsS - bG : kSwLdsS - bI - bJ)) {
                    status = 1;  // resume on the host at (it, q)
                    s_it = it;
                    s_q = q;
                    break;
                }
                const int wI = b, wJ = L - b;
                const int mr = (int)(a.maxbonddim < (int64_t)min(m, n) ? a.maxbonddim : (int64_t)min(m, n));
                SWP(1);
                // Pi = f(Icomb x Jcomb) into S (ld m | 1): the row / column states in the x / y space,
                // then one compact loop over the elements (one inlined copy of f, for the I-cache)
                St* rs = reinterpret_cast<St*>(xy);
                St* cs = rs + m;
                const int32_t* const Ibl = gsl;                      // (lazy union) Iset[b-1], Jset[b], the extras
                const int32_t* const Jbl = gsl + gI;
                const int32_t* const Exl = gsl + gI + gJ;
                const int32_t* const Eyl = gsl + gI + gJ + gEI;
                // rows and columns in ONE pass over the m + n entries (one leg_state per thread, not a
                // row pass then a column pass); lazily one leg_state_x per entry (kron rows and extras
                // in one code path)
                for (int t = tid; t < m + n; t += kSwThreads) {
                    const bool row = t < m;
                    const int i = row ? t : t - m;
                    if (lzu) {
                        const bool kr = i < (row ? KI : KJ);
                        const int32_t* e;
                        int w, lead = 0, cv = 0;
                        if (row) {
                            e = kr ? Ibl + (i % nI) * wI0 : Exl + xsel[0][i - KI] * wI;
                            w = kr ? wI0 : wI;
                            cv = kr ? i / nI + 1 : 0;
                        } else {
                            e = kr ? Jbl + (i / dJ) * wJ0 : Eyl + xsel[1][i - KJ] * wJ;
                            w = kr ? wJ0 : wJ;
                            lead = kr ? i % dJ + 1 : 0;
                        }
                        (row ? rs : cs)[i] = leg_state_x(f, lead, e, w, row ? 0 : wI, cv);
                    } else {
                        (row ? rs : cs)[i] = leg_state(f, row ? Ic + i * wI : Jc + i * wJ, row ? wI : wJ, row ? 0 : wI, 0);
                    }
                }
                __syncthreads();
                SWP(6);
                double mx = 0.0, error, maxerror;
                // (i, j) = (e mod m, e / m) stepped incrementally: no integer division per element
                const int di = kSwThreads % m, dj = kSwThreads / m;
                int i = tid % m, j = tid / m;
#pragma unroll 1
                for (int e = tid; e < m * n; e += kSwThreads) {
                    const double v = combine<KIND>(p, p0, rs[i], cs[j], wJ, L, nullptr, 0);
                    S[i + j * ldS] = v;
                    const double av = fabs(v);
                    mx = (isnan(av) || av > mx) ? av : mx;
                    i += di;
                    j += dj;
                    if (i >= m) {
                        i -= m;
                        j += 1;
                    }
                }
                SWP(7);
                mx = sw_maxabs(mx, &mxs);
                SWP(2);
                int* rp = perm;
                int* cp = perm + m;
                int np, fl;
                if (m <= kSwWaveN && n <= kSwWaveN && a.lu_wave) {  // one-wave rrLU
                    np = sw_lu_wave_any(S, ldS, m, n, mr, 1e-14, abstol, fwd ? 1 : 0, rp, cp, xy, xy + kSwRegN, red, pvl,
                                    &nanflag, &dslot, error, maxerror, fl, false, SWP_ACC);
                } else if (m <= kSwRegN && n <= kSwRegN) {  // register-tile rrLU, its tile read from S
                    np = sw_lu_regs(S, ldS, m, n, mr, 1e-14, abstol, fwd ? 1 : 0, rp, cp, xy, xy + kSwRegN, red, pvl,
                                    &nanflag, &dslot, error, maxerror, fl, SWP_ACC);
                } else {
                    np = small_lu_core<kSwThreads>(S, ldS, m, n, mr, 1e-14, abstol, fwd ? 1 : 0, rp, cp, red, xy,
                                                   xy + m, pvl, error, maxerror);
                    fl = small_lu_nanflags<kSwThreads>(S, ldS, m, n, np, &nanflag);
                }
                SWP(3);
                if (fl) {  // tci_update_pivots_h's NaN errors: the state stays as before this bond
                    status = (fl & 1) ? 2 : 3;
                    s_it = it;
                    s_q = q;
                    esite = b;
                    break;
                }
                const double err = np >= min(m, n) ? 0.0 : error;  // matrixlu.jl:391-393
                maxsample = jl_max(fabs(maxsample), fabs(mx));
                // Iset[b] = Icomb[rowidx], Jset[b-1] = Jcomb[colidx], each into its free slot
                const int tIs = sw_other(rol[0][1][b], rol[0][2][b]);
                const int tJs = sw_other(rol[1][1][b - 1], rol[1][2][b - 1]);
                int32_t* Io = bank_ptr(2 * tIs, b);
                int32_t* Jo = bank_ptr(2 * tJs + 1, b - 1);
                // a wave per row / column of the new set, a lane per leg (L <= 64): the row's source
                // (kron entry or kept extra) decoded once per row, no division per element
                {
                    const int wv = tid >> 6, l = tid & 63;
                    for (int rr = wv; rr < 2 * np; rr += kSwWaves) {
                        const bool sI = rr < np;
                        const int k = sI ? rr : rr - np;
                        const int w = sI ? wI : wJ;
                        if (l >= w) continue;
                        int32_t v;
                        if (lzu) {
                            if (sI) {
                                const int r = rp[k];
                                v = r < KI ? (l < wI0 ? Ibl[(r % nI) * wI0 + l] : r / nI + 1) : Exl[xsel[0][r - KI] * wI + l];
                            } else {
                                const int c = cp[k];
                                v = c < KJ ? (l == 0 ? c % dJ + 1 : Jbl[(c / dJ) * wJ0 + l - 1]) : Eyl[xsel[1][c - KJ] * wJ + l];
                            }
                        } else {
                            v = sI ? Ic[rp[k] * wI + l] : Jc[cp[k] * wJ + l];
                        }
                        (sI ? Io : Jo)[k * w + l] = v;
                    }
                }
                // updateerrors!(tci, b, pivoterrors(lu)): elementwise max over zero-padded vectors
                const int ne = max(npe, np + 1);
                for (int i = tid; i < ne; i += kSwThreads) {
                    const double nv = i < np ? fabs(pvl[i]) : (i == np ? err : 0.0);
                    pe[i] = jl_max(i < npe ? pe[i] : 0.0, nv);
                }
                __syncthreads();
                if (tid == 0) {
                    rol[0][0][b] = (unsigned char)tIs;
                    rol[1][0][b - 1] = (unsigned char)tJs;
                    cnt[(2 * tIs) * kSwMaxL + b] = np;
                    cnt[(2 * tJs + 1) * kSwMaxL + b - 1] = np;
                    bonderr[b - 1] = err;
                }
                npe = ne;
                __syncthreads();
#ifdef TCI_SW_PROF
                SWP(4);
                if (tid == 0) {
                    swp_acc[0] += swp_t[1] - swp_t[0];
                    swp_acc[1] += swp_t[2] - swp_t[1];
                    swp_acc[2] += swp_t[3] - swp_t[2];
                    swp_acc[3] += swp_t[4] - swp_t[3];
                    swp_acc[4] += swp_t[5] - swp_t[0];  // staging
                    swp_acc[5] += swp_t[6] - swp_t[1];  // states
                    swp_acc[6] += swp_t[7] - swp_t[6];  // Pi loop
                    swp_acc[7] += swp_t[2] - swp_t[7];  // maxabs
                    swp_n += 1;
                    swp_piv += np;
                }
#endif
            }
        }
#ifdef TCI_SW_PROF
        if (tid == 0 && swp_n > 0)
            printf("[sweep_small] %d bonds %d pivots: union %.2f (staging %.2f) | Pi %.2f (states %.2f loop %.2f maxabs %.2f) | "
                   "rrLU %.2f | select %.2f us per bond\n",
                   swp_n, swp_piv, swp_acc[0] * 0.01 / swp_n, swp_acc[4] * 0.01 / swp_n, swp_acc[1] * 0.01 / swp_n,
                   swp_acc[5] * 0.01 / swp_n, swp_acc[6] * 0.01 / swp_n, swp_acc[7] * 0.01 / swp_n,
                   swp_acc[2] * 0.01 / swp_n, swp_acc[3] * 0.01 / swp_n);
        if (tid == 0)
            printf("[sweep_small] LU us total (regs-LU | one-wave LU): load+take %.1f | wave argmax %.1f | barrier1 %.1f | "
                   "row argmax %.1f | decide+maps %.1f | normalise %.1f | barrier2 %.1f | update %.1f | loop exit %.1f | "
                   "NaN %.1f  (one-wave: 0 load+take, 1 argmax, 2 stop+maps, 3 normalise, 4 swap+xy, 5 update, "
                   "6 sync, 7 exit, 8 closing barriers)\n",
                   lu_acc[0] * 0.01, lu_acc[1] * 0.01, lu_acc[2] * 0.01, lu_acc[3] * 0.01, lu_acc[4] * 0.01,
                   lu_acc[5] * 0.01, lu_acc[6] * 0.01, lu_acc[7] * 0.01, lu_acc[8] * 0.01, lu_acc[9] * 0.01);
        if (tid == 0)
            printf("[sweep_small] shader clock %.3f GHz over %.1f us\n",
                   (double)(clock64() - swp_c0) / ((double)(wall_clock64() - swp_w0) * 10.0),
                   (double)(wall_clock64() - swp_w0) * 0.01);
#endif
    }
    if (a.mode == 2) {
        // sweep1site! (tensorci2.jl:659-725) with every bond in LDS: per bond b the sets of site
        // p = b - 1 combined with the site's leg on the sweep's side -- forward Icomb =
        // kronecker(Iset[p], d) (:671), Jcomb = Jset[p]; backward Icomb = Iset[p], Jcomb =
        // kronecker(d, Jset[p]) (:675) -- Pi, updatemaxsample!, the rrLU (reltol, abstol,
        // maxbonddim; leftorthogonal = forward), the new Iset[p + 1] / Jset[p] (forward) or Iset[p]
        // / Jset[p - 1], updateerrors! at bond b (forward) / b - 1, and with updatetensors the
        // site tensor T[b] = left(luci) / right(luci) (:703-711: the MatrixLUCI factors in
        // k_rrlu_small's operation order) and finally T[L] / T[1] = Pi1 of the last site (:717-722).
        // Any status but 0 leaves the host state untouched: the host loop then runs the sweep
        // (and raises the reference's error where there is one).
        const bool fwd = a.s1fwd != 0;
        int64_t* ttab = reinterpret_cast<int64_t*>(a.tens);
        double* tdat = a.tens + 2 * L;
        int64_t tused = 0;
        npe = 0;  // flushpivoterror!
        for (int q = 1; q < L && status == 0; ++q) {
            const int b = fwd ? q : L + 1 - q;  // 1-based: 1 .. L-1 forward, L .. 2 backward (:667)
            const int ps = b - 1;
            const int d = ldm[ps];
            const int nI = set_cnt(0, 0, ps), nJ = set_cnt(1, 0, ps);
            const int wIs = ps, wJs = L - 1 - ps;  // widths of Iset[p] / Jset[p]
            const int m = fwd ? nI * d : nI, n = fwd ? nJ : nJ * d;
            const int wI = fwd ? ps + 1 : ps, wJ = fwd ? L - 1 - ps : L - ps;
            const size_t bI = sw_al16((size_t)m * wI * 4), bJ = sw_al16((size_t)n * wJ * 4);
            const size_t bG = sw_al16((size_t)(nI * wIs + nJ * wJs) * 4);
            const int ldS = m | 1;
            const bool fits = m > 0 && n > 0 && (int64_t)ldS * n <= kSmallElems && m + n <= kSmallPerm &&
                              a.maxbonddim > 0 && bG + bI + bJ <= kSwLdsS && (size_t)ldS * n * 8 + bI + bJ <= kSwLdsS;
            if (!fits) {
                status = 1;
                break;
            }
            char* const R = reinterpret_cast<char*>(S);
            int32_t* const gs = reinterpret_cast<int32_t*>(R);
            int32_t* const Ic = reinterpret_cast<int32_t*>(R + kSwLdsS - bI - bJ);
            int32_t* const Jc = reinterpret_cast<int32_t*>(R + kSwLdsS - bJ);
            {  // Iset[p] and Jset[p] into LDS in one batched round of loads
                const int32_t* s0 = set_ptr(0, 0, ps);
                const int32_t* s1 = set_ptr(1, 0, ps);
                const int g0 = nI * wIs, tot = g0 + nJ * wJs;
                for (int base = 0; base < tot; base += kSwCopyB * kSwThreads) {
                    int32_t v[kSwCopyB];
#pragma unroll
                    for (int u = 0; u < kSwCopyB; ++u) {
                        const int e = base + tid + u * kSwThreads;
                        v[u] = e < g0 ? s0[e] : e < tot ? s1[e - g0] : 0;
                    }
#pragma unroll
                    for (int u = 0; u < kSwCopyB; ++u) {
                        const int e = base + tid + u * kSwThreads;
                        if (e < tot) gs[e] = v[u];
                    }
                }
            }
            __syncthreads();
            const int32_t* Ib = gs;
            const int32_t* Jb = gs + nI * wIs;
            if (fwd) {
                for (int e = tid; e < m; e += kSwThreads) {  // kronecker(Iset, d): Iset fastest
                    const int i = e % nI, j = e / nI;
                    sw_copy_row(Ic + e * wI, Ib + i * wIs, wIs);
                    Ic[e * wI + wIs] = j + 1;
                }
                for (int e = tid; e < n * wJ; e += kSwThreads) Jc[e] = Jb[e];
            } else {
                for (int e = tid; e < m * wI; e += kSwThreads) Ic[e] = Ib[e];
                for (int e = tid; e < n; e += kSwThreads) {  // kronecker(d, Jset): the leg fastest
                    const int i = e % d, jj = e / d;
                    Jc[e * wJ] = i + 1;
                    sw_copy_row(Jc + e * wJ + 1, Jb + jj * wJs, wJs);
                }
            }
            __syncthreads();
            St* rs = reinterpret_cast<St*>(xy);
            St* cs = rs + m;
            for (int i = tid; i < m; i += kSwThreads) rs[i] = leg_state(f, Ic + i * wI, wI, 0, 0);
            for (int j = tid; j < n; j += kSwThreads) cs[j] = leg_state(f, Jc + j * wJ, wJ, wI, 0);
            __syncthreads();
            double mx = 0.0, error, maxerror;
#pragma unroll 1
            for (int e = tid; e < m * n; e += kSwThreads) {
                const int i = e % m, j = e / m;
                const double v = combine<KIND>(p, p0, rs[i], cs[j], wJ, L, nullptr, 0);
                S[i + j * ldS] = v;
                const double av = fabs(v);
                mx = (isnan(av) || av > mx) ? av : mx;
            }
            mx = sw_maxabs(mx, &mxs);
            const int mr = (int)(a.maxbonddim < (int64_t)min(m, n) ? a.maxbonddim : (int64_t)min(m, n));
            int* rp = perm;
            int* cp = perm + m;
            int np, fl;
            if (m <= kSwWaveN && n <= kSwWaveN && a.lu_wave) {
                np = sw_lu_wave_any(S, ldS, m, n, mr, a.reltol, abstol, fwd ? 1 : 0, rp, cp, xy, xy + kSwRegN, red, pvl,
                                &nanflag, &dslot, error, maxerror, fl, a.s1tens != 0);
            } else if (m <= kSwRegN && n <= kSwRegN) {
                np = sw_lu_regs(S, ldS, m, n, mr, a.reltol, abstol, fwd ? 1 : 0, rp, cp, xy, xy + kSwRegN, red, pvl,
                                &nanflag, &dslot, error, maxerror, fl, SWP_ACC, a.s1tens != 0);
            } else {
                np = small_lu_core<kSwThreads>(S, ldS, m, n, mr, a.reltol, abstol, fwd ? 1 : 0, rp, cp, red, xy,
                                               xy + m, pvl, error, maxerror);
                fl = small_lu_nanflags<kSwThreads>(S, ldS, m, n, np, &nanflag);
            }
            if (fl) {
                status = (fl & 1) ? 2 : 3;
                esite = b;
                break;
            }
            const double err = np >= min(m, n) ? 0.0 : error;  // matrixlu.jl:391-393
            maxsample = jl_max(fabs(maxsample), fabs(mx));
            // the site tensor first (it reads the packed factors in S), then the new sets
            if (a.s1tens) {
                const int64_t cntT = fwd ? (int64_t)m * np : (int64_t)np * n;
                if (tused + cntT > a.tcap) {
                    status = 1;
                    break;
                }
                double* T = tdat + tused;
                if (fwd) {  // colstimespivotinv: rows >= np solve X L11 = L21 in place (matrixluci.jl:207)
                    for (int i = np + tid; i < m; i += kSwThreads)
                        for (int j = np - 1; j >= 0; --j) {
                            double s = S[i + j * ldS];
                            for (int t = j + 1; t < np; ++t) s = __dsub_rn(s, __dmul_rn(S[i + t * ldS], S[t + j * ldS]));
                            S[i + j * ldS] = s;
                        }
                    __syncthreads();
                    int tf = 0;
                    for (int e = tid; e < m * np; e += kSwThreads) {
                        const int i = e % m, j = e / m;
                        const double x = i < np ? (i == j ? 1.0 : 0.0) : S[i + j * ldS];
                        T[rp[i] + (int64_t)j * m] = x;
                        tf |= isnan(x) ? 1 : 0;
                    }
                    if (tf) atomicOr(&nanflag, 4);
                } else {  // pivotinvtimesrows: columns >= np solve U11 x = U[:, c] in place (:235)
                    for (int c = np + tid; c < n; c += kSwThreads)
                        for (int r = np - 1; r >= 0; --r) {
                            double s = S[r + c * ldS];
                            for (int t = r + 1; t < np; ++t) s = __dsub_rn(s, __dmul_rn(S[r + t * ldS], S[t + c * ldS]));
                            S[r + c * ldS] = s;
                        }
                    __syncthreads();
                    int tf = 0;
                    for (int e = tid; e < np * n; e += kSwThreads) {
                        const int r = e % np, j = e / np;
                        const double x = j < np ? (r == j ? 1.0 : 0.0) : S[r + j * ldS];
                        T[r + (int64_t)cp[j] * np] = x;
                        tf |= isnan(x) ? 1 : 0;
                    }
                    if (tf) atomicOr(&nanflag, 4);
                }
                __syncthreads();
                if (nanflag & 4) {  // "Error: NaN in tensor T[b]" (tensorci2.jl:706): the host raises it
                    status = 5;
                    esite = b;
                    break;
                }
                if (tid == 0) {
                    ttab[2 * ps] = tused;
                    ttab[2 * ps + 1] = cntT;
                }
                tused += cntT;
            }
            const int siteI = fwd ? ps + 1 : ps, siteJ = fwd ? ps : ps - 1;
            int32_t* Io = set_ptr(0, 0, siteI);
            int32_t* Jo = set_ptr(1, 0, siteJ);
            for (int e = tid; e < np * wI; e += kSwThreads) Io[e] = Ic[rp[e / wI] * wI + e % wI];
            for (int e = tid; e < np * wJ; e += kSwThreads) Jo[e] = Jc[cp[e / wJ] * wJ + e % wJ];
            // updateerrors!(tci, b (forward) / b - 1 (backward), pivoterrors(lu))
            const int ne = max(npe, np + 1);
            for (int i = tid; i < ne; i += kSwThreads) {
                const double nv = i < np ? fabs(pvl[i]) : (i == np ? err : 0.0);
                pe[i] = jl_max(i < npe ? pe[i] : 0.0, nv);
            }
            __syncthreads();
            if (tid == 0) {
                set_cnt(0, 0, siteI) = np;
                set_cnt(1, 0, siteJ) = np;
                bonderr[(fwd ? b : b - 1) - 1] = err;
            }
            npe = ne;
            __syncthreads();
        }
        if (status == 0 && a.s1tens) {
            // the last site's tensor: Pi1 = f(kronecker(Iset[p], d) x Jset[p]) (sitetensor, no solve)
            const int ps = fwd ? L - 1 : 0;
            const int nI = set_cnt(0, 0, ps), nJ = set_cnt(1, 0, ps), d = ldm[ps];
            const int Rr = nI * d;
            const int64_t cntT = (int64_t)Rr * nJ;
            if ((int64_t)Rr + nJ > kSmallElems || tused + cntT > a.tcap) {
                status = 1;
            } else {
                St* rs = reinterpret_cast<St*>(S);
                St* cs = rs + Rr;
                const int wI = ps, wJ = L - 1 - ps;
                const int32_t* Ib = set_ptr(0, 0, ps);
                const int32_t* Jb = set_ptr(1, 0, ps);
                for (int r = tid; r < Rr; r += kSwThreads) rs[r] = leg_state(f, Ib + (r % nI) * wI, wI, 0, r / nI + 1);
                for (int j = tid; j < nJ; j += kSwThreads) cs[j] = leg_state(f, Jb + j * wJ, wJ, ps + 1, 0);
                __syncthreads();
                double* T = tdat + tused;
#pragma unroll 1
                for (int64_t e = tid; e < cntT; e += kSwThreads)
                    T[e] = combine<KIND>(p, p0, rs[e % Rr], cs[e / Rr], wJ, L, nullptr, 0);
                if (tid == 0) {
                    ttab[2 * ps] = tused;
                    ttab[2 * ps + 1] = cntT;
                }
                tused += cntT;
            }
        }
        if (tid == 0) reinterpret_cast<int64_t*>(a.out)[10] = tused;
    }
    if ((a.mode == 1 || a.fill) && status == 0) {
        // fillsitetensors!(tci, f) (globalsearch.jl:202-208): the checks here -- the pivot matrices
        // square ("Pivot matrix at bond b is not square!", fstatus 4), every site within one
        // workgroup's LDS (else fstatus 5: the host loop runs the fill) -- and the map of the
        // current sets for k_fill_sites, which evaluates every site's Pi1 (updatemaxsample!) and, with
        // a.fsolve, setsitetensor!'s solve T = Pi1 P^-1 (tensorci2.jl:599-629), one workgroup per site
        fstatus = 0;
        int64_t tused = 0;
        for (int s = 0; s < L; ++s) {
            const int nI = set_cnt(0, 0, s), nJ = set_cnt(1, 0, s), d = ldm[s];
            if (s < L - 1 && set_cnt(0, 0, s + 1) != nJ) {
                fstatus = 4;  // "Pivot matrix at bond b is not square!"
                fsite = s + 1;
                break;
            }
            const int64_t R = (int64_t)nI * d, nT = R * nJ;
            const bool fits = a.fsolve ? (nT + (s == L - 1 ? 0 : (int64_t)nJ * nJ) <= kSmallElems &&
                                          R + nJ <= kSmallPerm && nJ <= 64 && tused + nT <= a.tcap)
                                       : R + nJ <= kSmallPerm;
            if (!fits) {
                fstatus = 5;  // the host evaluates it
                fsite = s + 1;
                break;
            }
            if (tid == 0) {
                int32_t* fm = a.fmap + 4 + 4 * s;
                fm[0] = bank_of(0, 0, s);
                fm[1] = bank_of(1, 0, s);
                fm[2] = nI;
                fm[3] = nJ;
                if (a.fsolve) {
                    reinterpret_cast<int64_t*>(a.tens)[2 * s] = tused;
                    reinterpret_cast<int64_t*>(a.tens)[2 * s + 1] = nT;
                }
            }
            tused += a.fsolve ? nT : 0;
        }
        if (tid == 0) {
            a.fmap[0] = fstatus == 0 ? 1 : 0;
            if (a.fsolve) reinterpret_cast<int64_t*>(a.out)[10] = fstatus == 0 ? tused : -1;
        }
    } else if (tid == 0 && a.fmap) {
        a.fmap[0] = 0;  // (no fill: k_fill_sites does nothing)
    }
    if (a.ctl && a.opt_it > 0 && tid == 0) {
        // chained optimize!: errors[it] = pivoterror(tci) (maxbonderror, tensorci2.jl:223-232), ranks[it]
        // = rank(tci) (max linkdims), then convergencecriterion (tensorci2.jl:947-966) over the last
        // ncheckhistory iterations with this iteration's abstol (no global pivots are added)
        const int it = a.opt_it;
        if (status != 0 || fstatus != 0) {
            a.ctl[1] = (unsigned long long)it;
            a.ctl[0] = 2;
        } else {
            double e = bonderr[0];
            for (int b = 1; b < L - 1; ++b) e = jl_max(e, bonderr[b]);
            int rk = 0;
            for (int b = 1; b < L; ++b) rk = max(rk, set_cnt(0, 0, b));
            a.ctl[8 + it] = (unsigned long long)__double_as_longlong(e);
            a.ctl[8 + kSwOptMax + it] = (unsigned long long)rk;
            bool conv = false;
            if (it >= a.opt_ncheck) {
                bool allerr = true, allmax = true;
                int mn = rk;
                for (int j = it - a.opt_ncheck + 1; j <= it; ++j) {
                    const double ej = __longlong_as_double((long long)a.ctl[8 + j]);
                    const int rj = (int)a.ctl[8 + kSwOptMax + j];
                    allerr = allerr && ej < abstol;
                    mn = min(mn, rj);
                    allmax = allmax && (int64_t)rj >= a.maxbonddim;
                }
                conv = (allerr && mn == rk) || allmax;
            }
            if (conv || it >= a.opt_maxiter) {
                a.ctl[1] = (unsigned long long)it;
                a.ctl[0] = 1;
            }
        }
    }
    __syncthreads();

    // ---- output: header, counts (logical banks), bond errors, pivot errors, the sets
    int64_t* out_hdr = reinterpret_cast<int64_t*>(a.out);
    int64_t* out_cnt = reinterpret_cast<int64_t*>(a.out + io.counts);
    if (tid == 0) {
        out_hdr[0] = status;
        out_hdr[1] = s_it;
        out_hdr[2] = s_q;
        out_hdr[3] = has_history;
        out_hdr[4] = extra_valid;
        out_hdr[5] = npe;
        out_hdr[6] = (int64_t)__double_as_longlong(maxsample);
        out_hdr[7] = esite;
        out_hdr[8] = fstatus;
        out_hdr[9] = fsite;
    }
    // logical bank lb: 0 / 1 current I / J, 2 / 3 history, 4 / 5 extra
    for (int i = tid; i < 6 * L; i += kSwThreads) {
        const int lb = i / L, s = i % L;
        out_cnt[i] = (lb >= 4 && !extra_valid) ? 0 : set_cnt(lb & 1, lb >> 1, s);
    }
    for (int i = tid; i < L - 1; i += kSwThreads) reinterpret_cast<double*>(a.out + io.bonderr)[i] = bonderr[i];
    for (int i = tid; i < npe; i += kSwThreads) reinterpret_cast<double*>(a.out + io.pe)[i] = pe[i];
    {
        int32_t* dst = reinterpret_cast<int32_t*>(a.out + io.sets);
        copy_segments(
            (extra_valid ? 6 : 4) * L,
            [&](int i) { const int lb = i / L; return set_cnt(lb & 1, lb >> 1, i % L) * width(lb, i % L); },
            [&](int i, int) { const int lb = i / L; return (const int32_t*)set_ptr(lb & 1, lb >> 1, i % L); },
            [&](int, int off) { return dst + off; });
    }
}

// fillsitetensors! for k_sweep_small's map, one workgroup per site (the sites are independent):
// Pi1 = f(kronecker(Iset[s], d) x Jset[s]) with the assembly's arithmetic, max |Pi1| (fmax[s], |v|
// bits), and with a.fsolve P = f(Iset[s + 1] x Jset[s]) stored transposed, getrf by one wave and
// getrs per row of Pi1 (sw_getrf_wave / sw_getrs_rows: the oracle's operation order), T in place
template <int KIND>
__global__ __launch_bounds__(kSwThreads) void k_fill_sites(SweepSmallArgs a, unsigned long long* fmax) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* S = reinterpret_cast<double*>(smem);
    int* piv = reinterpret_cast<int*>(smem + kSwLdsS);
    St* rs = reinterpret_cast<St*>(smem + kSwLdsS + kSwLdsPerm);
    __shared__ unsigned long long mxs;
    if (a.fmap[0] != 1) return;  // the sweep stopped, or the fill did not fit (the host runs it)
    const int tid = threadIdx.x, s = blockIdx.x, L = a.L;
    const FuncDev& f = a.f;
    const double* p = f.params;
    const double p0 = (KIND == F_SUM || KIND == F_TABLE) ? 0.0 : p[0];
    const int32_t* fm = a.fmap + 4 + 4 * s;
    const int bI = fm[0], bJ = fm[1], nI = fm[2], nJ = fm[3];
    const int d = f.localdims[s];
    const int64_t half = (int64_t)L * (L - 1) / 2;
    auto bank_ptr = [&](int bank, int site) -> const int32_t* {  // (k_sweep_small's layout)
        const int64_t pre = (bank & 1) ? (int64_t)site * (L - 1) - (int64_t)site * (site - 1) / 2
                                       : (int64_t)site * (site - 1) / 2;
        return a.ws + a.cap * (bank * half + pre);
    };
    const int R = nI * d, r = nJ, wI = s, wJ = L - 1 - s;
    const int64_t nT = (int64_t)R * r;
    St* cs = rs + R;
    const int32_t* Ib = bank_ptr(bI, s);
    const int32_t* Jb = bank_ptr(bJ, s);
    for (int q = tid; q < R; q += kSwThreads) rs[q] = leg_state(f, Ib + (q % nI) * wI, wI, 0, q / nI + 1);
    for (int j = tid; j < r; j += kSwThreads) cs[j] = leg_state(f, Jb + j * wJ, wJ, s + 1, 0);
    __syncthreads();
    double mx = 0.0;
    double* Pi1 = S;  // R x r, ld R (T in place after the solve)
#pragma unroll 1
    for (int64_t e = tid; e < nT; e += kSwThreads) {
        const double v = combine<KIND>(p, p0, rs[e % R], cs[e / R], wJ, L, nullptr, 0);
        if (a.fsolve) Pi1[e] = v;
        const double av = fabs(v);
        mx = (isnan(av) || av > mx) ? av : mx;
    }
    mx = sw_maxabs(mx, &mxs);
    if (tid == 0) fmax[s] = (unsigned long long)__double_as_longlong(fabs(mx));
    if (!a.fsolve) return;
    if (s < L - 1) {
        // P = f(Iset[s + 1] x Jset[s]) (the same column legs), stored transposed
        double* Pt = S + nT;
        const int32_t* In = bank_ptr(a.fmap[4 + 4 * (s + 1)], s + 1);
        for (int q = tid; q < r; q += kSwThreads) rs[q] = leg_state(f, In + q * (s + 1), s + 1, 0, 0);
        __syncthreads();
#pragma unroll 1
        for (int e = tid; e < r * r; e += kSwThreads) {
            const int q = e % r, j = e / r;  // P[q][j] -> Pt[j + q r]
            Pt[j + q * r] = combine<KIND>(p, p0, rs[q], cs[j], wJ, L, nullptr, 0);
        }
        __syncthreads();
        if (tid < 64) sw_getrf_wave(Pt, r, piv);
        __syncthreads();
        if (r <= 16)
            sw_getrs_rows<16>(Pi1, R, r, Pt, piv);
        else if (r <= 32)
            sw_getrs_rows<32>(Pi1, R, r, Pt, piv);
        else
            sw_getrs_rows<0>(Pi1, R, r, Pt, piv);
        __syncthreads();
    }
    double* T = a.tens + 2 * L + reinterpret_cast<const int64_t*>(a.tens)[2 * s];
    for (int64_t e = tid; e < nT; e += kSwThreads) T[e] = Pi1[e];
}

hipError_t launch_fill_sites(hipStream_t s, const SweepSmallArgs& a, unsigned long long* fmax) {
    const void* fn = nullptr;
    switch (a.f.kind) {
    case F_SUM: fn = reinterpret_cast<const void*>(&k_fill_sites<F_SUM>); break;
    case F_LORENTZ: fn = reinterpret_cast<const void*>(&k_fill_sites<F_LORENTZ>); break;
    case F_TABLE: fn = reinterpret_cast<const void*>(&k_fill_sites<F_TABLE>); break;
    case F_GAUSS: fn = reinterpret_cast<const void*>(&k_fill_sites<F_GAUSS>); break;
    case F_QOSC: fn = reinterpret_cast<const void*>(&k_fill_sites<F_QOSC>); break;
    case F_QEXP: fn = reinterpret_cast<const void*>(&k_fill_sites<F_QEXP>); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSwLds);
    if (e != hipSuccess) return e;
    switch (a.f.kind) {
#define TCI_FS(K)                                                                                    \
    case K: hipLaunchKernelGGL(k_fill_sites<K>, dim3(a.L), dim3(kSwThreads), kSwLds, s, a, fmax); break;
        TCI_FS(F_SUM) TCI_FS(F_LORENTZ) TCI_FS(F_TABLE) TCI_FS(F_GAUSS) TCI_FS(F_QOSC) TCI_FS(F_QEXP)
#undef TCI_FS
    default: break;
    }
    return hipGetLastError();
}

size_t sweep_small_lds_bytes() { return kSwLds; }

hipError_t launch_sweep_small(hipStream_t s, const SweepSmallArgs& a) {
    const void* fn = nullptr;
    switch (a.f.kind) {
    case F_SUM: fn = reinterpret_cast<const void*>(&k_sweep_small<F_SUM>); break;
    case F_LORENTZ: fn = reinterpret_cast<const void*>(&k_sweep_small<F_LORENTZ>); break;
    case F_TABLE: fn = reinterpret_cast<const void*>(&k_sweep_small<F_TABLE>); break;
    case F_GAUSS: fn = reinterpret_cast<const void*>(&k_sweep_small<F_GAUSS>); break;
    case F_QOSC: fn = reinterpret_cast<const void*>(&k_sweep_small<F_QOSC>); break;
    case F_QEXP: fn = reinterpret_cast<const void*>(&k_sweep_small<F_QEXP>); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSwLds);
    if (e != hipSuccess) return e;
    switch (a.f.kind) {
#define TCI_SW(K)                                                                                    \
    case K: hipLaunchKernelGGL(k_sweep_small<K>, dim3(1), dim3(kSwThreads), kSwLds, s, a); break;
        TCI_SW(F_SUM) TCI_SW(F_LORENTZ) TCI_SW(F_TABLE) TCI_SW(F_GAUSS) TCI_SW(F_QOSC) TCI_SW(F_QEXP)
#undef TCI_SW
    default: break;
    }
    return hipGetLastError();
}

bool sweep_small_kind(int kind) { return staged_kind(kind); }

}  // namespace tci
