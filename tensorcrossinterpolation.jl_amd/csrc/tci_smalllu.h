// tci_smalllu.h -- _optimizerrlu! (matrixlu.jl:346-369) on a matrix held in one workgroup's LDS,
// shared by k_rrlu_small (tci_rrlu.hip, one Pi per launch) and the device-resident small sweep
// (tci_sweep_small.hip, a whole sweep2site! per launch): argmax over the trailing block
// (column-major scan order as the tie-break), stop test, swaprow!/swapcol! (physical, in LDS),
// true-division normalisation and the rank-1 update with separate multiply and subtract. The
// candidate order is a strict total order, so the results do not depend on the thread count.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace tci {

// Base.max for Float64 (NaN-propagating; -0.0 < 0.0)
__device__ __forceinline__ double jl_max(double x, double y) {
    bool ysel = (y > x) || (signbit(y) < signbit(x));
    if (ysel) return isnan(x) ? x : y;
    return isnan(y) ? y : x;
}

// Argmax reductions on DPP lane moves (VALU, no LDS round trip as ds_bpermute has): a candidate
// is (abs2 value, key), larger value first, then the smaller key; NaN never wins.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

template <int CTRL>
__device__ __forceinline__ void dpp_take(double& bv, unsigned& bk, double& bx) {
    const double ov = dpp_f64<CTRL>(bv), ox = dpp_f64<CTRL>(bx);
    const unsigned ok = (unsigned)__builtin_amdgcn_update_dpp(0, (int)bk, CTRL, 0xf, 0xf, false);
    const bool better = (ov > bv) || (ov == bv && ok < bk);
    bv = better ? ov : bv;
    bk = better ? ok : bk;
    bx = better ? ox : bx;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// winner of each row of 16 lanes, in every lane of that row (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror)
__device__ __forceinline__ void row16_argmax_dpp(double& bv, unsigned& bk, double& bx) {
    dpp_take<0xb1>(bv, bk, bx);
    dpp_take<0x4e>(bv, bk, bx);
    dpp_take<0x141>(bv, bk, bx);
    dpp_take<0x140>(bv, bk, bx);
}

// winner of lanes 0..15, uniform in every lane
__device__ __forceinline__ void row_argmax_dpp(double& bv, unsigned& bk, double& bx) {
    row16_argmax_dpp(bv, bk, bx);
    bv = readlane_f64(bv, 0);
    bk = (unsigned)__builtin_amdgcn_readlane((int)bk, 0);
    bx = readlane_f64(bx, 0);
}

// winner of the whole wave, uniform in every lane
__device__ __forceinline__ void wave_argmax_dpp(double& bv, unsigned& bk) {
    double bx = 0.0;
    row16_argmax_dpp(bv, bk, bx);
    double v = readlane_f64(bv, 0);
    unsigned key = (unsigned)__builtin_amdgcn_readlane((int)bk, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double ov = readlane_f64(bv, r);
        const unsigned ok = (unsigned)__builtin_amdgcn_readlane((int)bk, r);
        const bool better = (ov > v) || (ov == v && ok < key);
        v = better ? ov : v;
        key = better ? ok : key;
    }
    bv = v;
    bk = key;
}

struct SmallCand {
    double v;
    unsigned key;
    unsigned pad;
    double val;
};
constexpr int64_t kSmallElems = 16384;  // 128 KiB of fp64 in LDS
constexpr int64_t kSmallPerm = 2048;    // m + n

// winner of the whole wave carrying one more double (the candidate's value), uniform in every lane
__device__ __forceinline__ void wave_argmax3(double& bv, unsigned& bk, double& bx) {
    row16_argmax_dpp(bv, bk, bx);
    double v = readlane_f64(bv, 0), x = readlane_f64(bx, 0);
    unsigned key = (unsigned)__builtin_amdgcn_readlane((int)bk, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double ov = readlane_f64(bv, r), ox = readlane_f64(bx, r);
        const unsigned ok = (unsigned)__builtin_amdgcn_readlane((int)bk, r);
        const bool better = (ov > v) || (ov == v && ok < key);
        v = better ? ov : v;
        key = better ? ok : key;
        x = better ? ox : x;
    }
    bv = v;
    bk = key;
    bx = x;
}

// S: m x n (ld ldS) in LDS, overwritten by the packed factors; rp / cp: m / n ints, xv / yv: m / n
// doubles, red: NT / 64 candidates, all in LDS. pivvals[k] (any memory) gets pivot k's value.
// Returns npivot (the same in every thread); error / maxerror are lu.error and the running
// maximum of _optimizerrlu!.
template <int NT>
__device__ __forceinline__ int small_lu_core(double* S, int ldS, int m, int n, int mr, double reltol,
                                             double abstol, int leftorth, int* rp, int* cp, SmallCand* red2,
                                             double* xv, double* yv, double* pivvals, double& error,
                                             double& maxerror) {
    // thread (w, l) owns rows l, l + 64, ... of columns w, w + NW, ...: no index division
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    constexpr int NW = NT / 64;
    for (int i = tid; i < m; i += NT) rp[i] = i;
    for (int j = tid; j < n; j += NT) cp[j] = j;
    // every thread tracks the loop state (identical everywhere)
    maxerror = 0.0;
    error = __longlong_as_double(0x7ff8000000000000LL);
    int np = 0;
    __syncthreads();
    // argmax of abs2 over the trailing block (submatrixargmax, matrixlu.jl:46-87): the candidate
    // order (value, column, row) is the reference's column-major scan with strict '>'
    // a candidate is (abs2, key = column << 16 | row): larger abs2 wins, then the smaller key
    double bv = -1.0;
    unsigned bk = 0xffffffffu;
    auto take = [&](double a2, unsigned key) {
        const bool better = (a2 > bv) || (a2 == bv && key < bk);  // NaN never wins
        bv = better ? a2 : bv;
        bk = better ? key : bk;
    };
    for (int j = w; j < n; j += NW)
        for (int i = l; i < m; i += 64) {
            const double v = S[i + j * ldS];
            take(__dmul_rn(v, v), ((unsigned)j << 16) | (unsigned)i);
        }
    for (int k = 0; k < mr; ++k) {
        wave_argmax_dpp(bv, bk);  // every lane now holds the wave's winner
        if (l == 0)  // the wave's winner and its value (no swap can be under way here)
            red2[w] = SmallCand{bv, bk, 0u, bv >= 0.0 ? S[(bk & 0xffffu) + (bk >> 16) * ldS] : 0.0};
        __syncthreads();
        // the workgroup's winner: lanes 0..NW-1 of every wave take one wave's entry each
        SmallCand b = l < NW ? red2[l] : SmallCand{-1.0, 0xffffffffu, 0u, 0.0};
        row_argmax_dpp(b.v, b.key, b.val);
        int p = (int)(b.key & 0xffffu), q = (int)(b.key >> 16);
        double val = b.val;
        if (!(b.v >= 0.0)) {  // every trailing value NaN: Julia keeps (k, k)
            p = q = k;
            val = S[k + k * ldS];
        }
        error = fabs(val);
        if (((fabs(error) < reltol * maxerror) || (fabs(error) < abstol)) && k > 0) break;
        maxerror = jl_max(maxerror, error);
        np = k + 1;
        if (tid == 0) pivvals[k] = val;
        // swaprow!(k, p) then swapcol!(k, q) (matrixlu.jl:254-275)
        if (p != k) {
            for (int j = tid; j < n; j += NT) {
                const double t = S[k + j * ldS];
                S[k + j * ldS] = S[p + j * ldS];
                S[p + j * ldS] = t;
            }
            if (tid == 0) {
                const int t = rp[k];
                rp[k] = rp[p];
                rp[p] = t;
            }
            __syncthreads();
        }
        if (q != k) {
            for (int i = tid; i < m; i += NT) {
                const double t = S[i + k * ldS];
                S[i + k * ldS] = S[i + q * ldS];
                S[i + q * ldS] = t;
            }
            if (tid == 0) {
                const int t = cp[k];
                cp[k] = cp[q];
                cp[q] = t;
            }
            __syncthreads();
        }
        // normalisation by the pivot (true division; matrixlu.jl:300-305) into S and xv / yv
        const double piv = S[k + k * ldS];
        for (int i = k + 1 + tid; i < m; i += NT) {
            const double x = leftorth ? S[i + k * ldS] / piv : S[i + k * ldS];
            xv[i] = x;
            S[i + k * ldS] = x;
        }
        for (int j = k + 1 + tid; j < n; j += NT) {
            const double y = leftorth ? S[k + j * ldS] : S[k + j * ldS] / piv;
            yv[j] = y;
            S[k + j * ldS] = y;
        }
        __syncthreads();
        // rank-1 update (mul then sub, matrixlu.jl:314-320) fused with the next pivot's argmax
        bv = -1.0;
        bk = 0xffffffffu;
        if (m <= 64 * 4) {  // this lane's (at most 4) rows: their x's stay in registers
            double xr[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const int i = l + 64 * a;
                xr[a] = (i < m && i > k) ? xv[i] : 0.0;
            }
            // (the update is fp64-VALU-bound here: ~3 us/pivot at 14k elements on one CU)
            for (int j = w; j < n; j += NW) {
                if (j <= k) continue;
                const double y = yv[j];
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    const int i = l + 64 * a;
                    if (i >= m || i <= k) continue;
                    const double v = __dsub_rn(S[i + j * ldS], __dmul_rn(xr[a], y));
                    S[i + j * ldS] = v;
                    take(__dmul_rn(v, v), ((unsigned)j << 16) | (unsigned)i);
                }
            }
        } else {
            for (int j = w; j < n; j += NW) {
                if (j <= k) continue;
                const double y = yv[j];
                for (int i = l; i < m; i += 64) {
                    if (i <= k) continue;
                    const double v = __dsub_rn(S[i + j * ldS], __dmul_rn(xv[i], y));
                    S[i + j * ldS] = v;
                    take(__dmul_rn(v, v), ((unsigned)j << 16) | (unsigned)i);
                }
            }
        }
    }
    return np;
}

// tril(A[:, 1:np]) / triu(A[1:np, :]) NaN checks before the unit diagonal is set (matrixlu.jl:
// 376-381): bit 1 / bit 2, the same in every thread. slot: one int of LDS.
template <int NT>
__device__ __forceinline__ int small_lu_nanflags(const double* S, int ldS, int m, int n, int np, int* slot) {
    const int tid = threadIdx.x;
    if (tid == 0) *slot = 0;
    __syncthreads();
    int fl = 0;
    for (int e = tid; e < m * np; e += NT) {
        const int pos = e % m, t = e / m;
        if (pos >= t && isnan(S[pos + t * ldS])) fl |= 1;
    }
    for (int e = tid; e < np * n; e += NT) {
        const int t = e % np, pos = e / np;
        if (pos >= t && isnan(S[t + pos * ldS])) fl |= 2;
    }
    if (fl) atomicOr(slot, fl);
    __syncthreads();
    return *slot;
}

}  // namespace tci
