// tci_funcdev.h -- device evaluation of the staged integrand kinds (batcheval.jl:131-175 for the
// catalog of include/tci_hip.h), shared by the batched Pi assembly (tci_device.hip) and the
// device-resident small sweep (tci_sweep_small.hip) so that both produce the same bits: a Pi
// element is combine<KIND>(row state, column state), each state a leg_state() over its legs.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tci_internal.h"

namespace tci {

enum { F_SUM = 0, F_LORENTZ = 1, F_TABLE = 2, F_GAUSS = 3, F_GAUSSMIX = 4, F_QOSC = 5, F_QEXP = 6,
       F_TT = 7, F_CP = 8, F_MPO = 9 };

// Kinds that are a sum of K separable terms, f = sum_k rowfactor_k(I, c) * colfactor_k(J): Pi is
// a rank-K product EL * ER^T, assembled by an fp64 MFMA GEMM (k_gemm_cp).
__host__ __device__ __forceinline__ bool cp_kind(int kind) {
    return kind == F_GAUSSMIX || kind == F_CP || kind == F_MPO;
}

__host__ __device__ __forceinline__ bool staged_kind(int kind) {
    return kind == F_SUM || kind == F_LORENTZ || kind == F_TABLE || kind == F_GAUSS ||
           kind == F_QOSC || kind == F_QEXP;
}

// state of a leg value v (1-based) at global position t; combined by integer/double addition or
// bit concatenation.
union St {
    int64_t i;
    double d;
};

// fn(t, e[t]) for t = 0 .. w-1 in order, the loads issued eight at a time (a runtime-length loop
// of dependent LDS / L2 round trips otherwise)
template <class Fn>
__device__ __forceinline__ void for_legs(const int32_t* e, int w, Fn fn) {
    int t = 0;
    for (; t + 8 <= w; t += 8) {
        int32_t x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = e[t + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) fn(t + u, x[u]);
    }
    for (; t < w; ++t) fn(t, e[t]);
}

// The state of legs e[0 .. w-1] at global positions toff .. toff + w - 1, then, if cval > 0, one
// more leg of value cval at position toff + w (the centre index of a site tensor's Pi1 row).
__device__ __forceinline__ St leg_state(const FuncDev& f, const int32_t* e, int w, int toff, int cval) {
    St s;
    s.i = 0;
    switch (f.kind) {
    case F_SUM:
        for_legs(e, w, [&](int, int32_t x) { s.i += x; });
        if (cval > 0) s.i += cval;
        break;
    case F_LORENTZ:
        for_legs(e, w, [&](int, int32_t x) { s.i += (int64_t)x * x; });
        if (cval > 0) s.i += (int64_t)cval * cval;
        break;
    case F_TABLE:
        for_legs(e, w, [&](int t, int32_t x) { s.i += (int64_t)(x - 1) * f.strides[toff + t]; });
        if (cval > 0) s.i += (int64_t)(cval - 1) * f.strides[toff + w];
        break;
    case F_GAUSS: {
        double a = 0.0;
        const double c = f.params[1];
        for_legs(e, w, [&](int, int32_t x) {
            const double u = (double)x - c;
            a = __dadd_rn(a, __dmul_rn(u, u));
        });
        if (cval > 0) {
            const double u = (double)cval - c;
            a = __dadd_rn(a, __dmul_rn(u, u));
        }
        s.d = a;
    } break;
    case F_QOSC:
    case F_QEXP: {
        uint64_t idx = 0;
        for_legs(e, w, [&](int, int32_t x) { idx = (idx << 1) | (uint64_t)(x - 1); });
        if (cval > 0) idx = (idx << 1) | (uint64_t)(cval - 1);
        s.i = (int64_t)idx;
    } break;
    }
    return s;
}

// The state of the legs [lead (if > 0), e[0 .. w-1], cval (if > 0)] at global positions toff, ...
// in that order -- a kronecker(Iset, d) row [I..., j] (cval = j) or kronecker(d, Jset) column
// [i, J...] (lead = i), tensorci2.jl:512-529, without materialising it; the same operations in the
// same order as leg_state over the materialised entry. One code path for every entry, so that the
// lanes of a wave holding kron entries and extras do not diverge into two copies of it.
__device__ __forceinline__ St leg_state_x(const FuncDev& f, int lead, const int32_t* e, int w, int toff, int cval) {
    St s;
    s.i = 0;
    const int o = lead > 0 ? 1 : 0;  // e[t] sits at position toff + o + t
    switch (f.kind) {
    case F_SUM:
        if (lead > 0) s.i += lead;
        for_legs(e, w, [&](int, int32_t x) { s.i += x; });
        if (cval > 0) s.i += cval;
        break;
    case F_LORENTZ:
        if (lead > 0) s.i += (int64_t)lead * lead;
        for_legs(e, w, [&](int, int32_t x) { s.i += (int64_t)x * x; });
        if (cval > 0) s.i += (int64_t)cval * cval;
        break;
    case F_TABLE:
        if (lead > 0) s.i += (int64_t)(lead - 1) * f.strides[toff];
        for_legs(e, w, [&](int t, int32_t x) { s.i += (int64_t)(x - 1) * f.strides[toff + o + t]; });
        if (cval > 0) s.i += (int64_t)(cval - 1) * f.strides[toff + o + w];
        break;
    case F_GAUSS: {
        double a = 0.0;
        const double c = f.params[1];
        if (lead > 0) {
            const double u = (double)lead - c;
            a = __dadd_rn(a, __dmul_rn(u, u));
        }
        for_legs(e, w, [&](int, int32_t x) {
            const double u = (double)x - c;
            a = __dadd_rn(a, __dmul_rn(u, u));
        });
        if (cval > 0) {
            const double u = (double)cval - c;
            a = __dadd_rn(a, __dmul_rn(u, u));
        }
        s.d = a;
    } break;
    case F_QOSC:
    case F_QEXP: {
        uint64_t idx = 0;
        if (lead > 0) idx = (uint64_t)(lead - 1);
        for_legs(e, w, [&](int, int32_t x) { idx = (idx << 1) | (uint64_t)(x - 1); });
        if (cval > 0) idx = (idx << 1) | (uint64_t)(cval - 1);
        s.i = (int64_t)idx;
    } break;
    }
    return s;
}

// value of one Pi element from its row and column states. Lorentzian: the quotient
// p0 / (s + 1) of the integer sum of squares s, from a table of the same quotients when one is
// given (s < ntab): bitwise the same division.
template <int KIND>
__device__ __forceinline__ double combine(const double* __restrict__ p, double p0, St r, St c, int nr,
                                          int L, const double* __restrict__ tab, int64_t ntab) {
    if (KIND == F_SUM) return (double)(r.i + c.i);
    if (KIND == F_LORENTZ) {
        const int64_t s = r.i + c.i;
        return s < ntab ? tab[s] : p0 / (double)(s + 1);
    }
    if (KIND == F_TABLE) return p[r.i + c.i];
    if (KIND == F_GAUSS) return exp(-(p0 * __dadd_rn(r.d, c.d)));
    if (KIND == F_QOSC) {
        const uint64_t idx = ((uint64_t)r.i << nr) | (uint64_t)c.i;
        const double x = ldexp((double)idx, -L);
        return exp(-(p0 * x)) * sin(p[1] * pow(x, p[2]));
    }
    if (KIND == F_QEXP) {
        const uint64_t idx = ((uint64_t)r.i << nr) | (uint64_t)c.i;
        const double x = ldexp((double)idx, -L);
        return __dadd_rn(p0 * exp(-(p[1] * x)), p[2] * exp(-(p[3] * x)));
    }
    return 0.0;
}

}  // namespace tci
