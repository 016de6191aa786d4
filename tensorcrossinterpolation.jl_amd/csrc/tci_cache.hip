// tci_cache.hip -- CachedFunction's memo (src/cachedfunction.jl:53-302) as a device hash table.
//
// The reference memoises f in a Dict keyed by key(x) = sum((x .- 1) .* coeffs) with coeffs =
// cumprod([1; localdims[1:end-1]]) (cachedfunction.jl:197-199), and its batch method looks every
// point up and calls f on the misses (:255-302). Here the table lives in HBM (open addressing,
// linear probing, splitmix64 hash; keys < 2^63, EMPTY = all ones) and a Pi block is served in
// one pass: the key of element (i, c, j) is kI[i] + c coeff[nl] + kJ[j] because it is linear in
// the legs; hits are written straight into Pi, the first thread to claim an empty slot for a key
// records a miss, later threads with the same key in the same batch record a duplicate. The misses
// are gathered into a point table and evaluated in ONE batch evaluation of the device integrand,
// then written to the table and to Pi; duplicates are served from the table afterwards.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tci_internal.h"

namespace tci {

constexpr unsigned long long kCacheEmpty = ~0ull;

__device__ __forceinline__ unsigned long long cache_hash(unsigned long long k) {
    k += 0x9E3779B97F4A7C15ull;
    k = (k ^ (k >> 30)) * 0xBF58476D1CE4E5B9ull;
    k = (k ^ (k >> 27)) * 0x94D049BB133111EBull;
    return k ^ (k >> 31);
}

// partial keys of index-set rows: out[i] = sum_t (T[i, t] - 1) * coeff[t0 + t]
__global__ void k_cache_partial_keys(const int32_t* __restrict__ T, int cnt, int w, const int64_t* __restrict__ coeff,
                                     int t0, int64_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    int64_t k = 0;
    for (int t = 0; t < w; ++t) k += (int64_t)(T[(int64_t)i * w + t] - 1) * coeff[t0 + t];
    out[i] = k;
}

struct CacheProbe {
    unsigned long long* keys;
    double* vals;
    unsigned* state;  // 0 empty, 1 claimed in this batch (value pending), 2 ready
    int64_t cap;      // power of two
    const int64_t* kI;
    const int64_t* kJ;
    int64_t ccoef;  // coeff of the centre leg (M = 1)
    int64_t m, mR, n;
    double* out;
    int64_t ldo;
    int64_t* miss;      // element index, slot (pairs)
    int64_t* dup;       // element index
    unsigned long long* counts;  // [0] misses, [1] duplicates, [2] a duplicate found no ready value
};

__global__ void k_cache_probe(CacheProbe g) {
    const int64_t tot = g.mR * g.n;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t R = e % g.mR, j = e / g.mR;
        const int64_t i = R % g.m, c = R / g.m;
        const unsigned long long key = (unsigned long long)(g.kI[i] + c * g.ccoef + g.kJ[j]);
        int64_t s = (int64_t)(cache_hash(key) & (unsigned long long)(g.cap - 1));
        for (int64_t probe = 0; probe < g.cap; ++probe, s = (s + 1) & (g.cap - 1)) {
            unsigned long long kk = __hip_atomic_load(&g.keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (kk == kCacheEmpty) {
                kk = atomicCAS(&g.keys[s], kCacheEmpty, key);
                if (kk == kCacheEmpty) {  // claimed: a miss to evaluate
                    g.state[s] = 1;
                    const unsigned long long q = atomicAdd(&g.counts[0], 1ull);
                    g.miss[2 * q] = e;
                    g.miss[2 * q + 1] = s;
                    break;
                }
            }
            if (kk == key) {
                if (__hip_atomic_load(&g.state[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 2) {
                    g.out[R + g.ldo * j] = g.vals[s];  // hit (ready since an earlier batch)
                } else {
                    const unsigned long long q = atomicAdd(&g.counts[1], 1ull);
                    g.dup[q] = e;
                }
                break;
            }
        }
    }
}

// miss element -> its full index vector (row-major, width L): I row, centre, J column
__global__ void k_cache_gather_points(const int64_t* __restrict__ miss, int64_t nmiss, const int32_t* __restrict__ I,
                                      int nl, const int32_t* __restrict__ J, int nr, int M, int64_t m, int64_t mR,
                                      int32_t* __restrict__ X) {
    const int L = nl + M + nr;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nmiss; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = miss[2 * q];
        const int64_t R = e % mR, j = e / mR;
        const int64_t i = R % m, c = R / m;
        int32_t* x = X + q * L;
        for (int t = 0; t < nl; ++t) x[t] = I[i * nl + t];
        if (M) x[nl] = (int32_t)c + 1;
        for (int t = 0; t < nr; ++t) x[nl + M + t] = J[j * nr + t];
    }
}

__global__ void k_cache_fill(const int64_t* __restrict__ miss, int64_t nmiss, const double* __restrict__ v,
                             double* __restrict__ vals, unsigned* __restrict__ state, int64_t mR,
                             double* __restrict__ out, int64_t ldo) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nmiss; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = miss[2 * q], s = miss[2 * q + 1];
        vals[s] = v[q];
        state[s] = 2;
        if (out) out[(e % mR) + ldo * (e / mR)] = v[q];
    }
}

__global__ void k_cache_dups(CacheProbe g, int64_t ndup) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < ndup; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = g.dup[q];
        const int64_t R = e % g.mR, j = e / g.mR;
        const int64_t i = R % g.m, c = R / g.m;
        const unsigned long long key = (unsigned long long)(g.kI[i] + c * g.ccoef + g.kJ[j]);
        int64_t s = (int64_t)(cache_hash(key) & (unsigned long long)(g.cap - 1));
        for (int64_t probe = 0; probe < g.cap; ++probe, s = (s + 1) & (g.cap - 1)) {
            if (g.keys[s] == key) {
                if (g.state[s] == 2) {
                    g.out[R + g.ldo * j] = g.vals[s];
                } else {  // never served as a value: the batch reports an error
                    g.out[R + g.ldo * j] = __longlong_as_double(0x7ff8000000000badll);
                    atomicOr(&g.counts[2], 1ull);
                }
                break;
            }
        }
    }
}

// roll back the slots a failed batch claimed (state 1: value never written): EMPTY again. Safe
// under linear probing -- the slots were empty before this batch, so no older key's probe chain
// runs through them, and every key of this batch that probed past one is itself a claim undone here
__global__ void k_cache_unclaim(const int64_t* __restrict__ miss, int64_t nmiss, unsigned long long* keys,
                                unsigned* state) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nmiss; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = miss[2 * q + 1];
        if (state[s] == 1) {
            state[s] = 0;
            keys[s] = kCacheEmpty;
        }
    }
}

// haskey / lookup of npts points (row-major, width L, 1-based): found[q] = 1 and vals[q] when the
// key is in the table with a ready value (cachedfunction.jl:197-240)
__global__ void k_cache_lookup(const int32_t* __restrict__ X, int64_t npts, int L, const int64_t* __restrict__ coeff,
                               const unsigned long long* __restrict__ keys, const double* __restrict__ vals,
                               const unsigned* __restrict__ state, int64_t cap, int32_t* found, double* out) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < npts; q += (int64_t)gridDim.x * blockDim.x) {
        int64_t k = 0;
        for (int t = 0; t < L; ++t) k += (int64_t)(X[q * L + t] - 1) * coeff[t];
        const unsigned long long key = (unsigned long long)k;
        int64_t s = (int64_t)(cache_hash(key) & (unsigned long long)(cap - 1));
        int32_t f = 0;
        double v = 0.0;
        for (int64_t probe = 0; probe < cap; ++probe, s = (s + 1) & (cap - 1)) {
            const unsigned long long kk = keys[s];
            if (kk == kCacheEmpty) break;
            if (kk == key) {
                if (state[s] == 2) {
                    f = 1;
                    v = vals[s];
                }
                break;
            }
        }
        found[q] = f;
        out[q] = v;
    }
}

// max |Pi| with Julia's NaN-propagating max (|v| bit patterns, unsigned max)
__global__ __launch_bounds__(256) void k_cache_maxabs(const double* __restrict__ out, int64_t mR, int64_t n,
                                                      int64_t ldo, unsigned long long* maxbits) {
    unsigned long long b = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < mR * n; e += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long x = (unsigned long long)__double_as_longlong(fabs(out[(e % mR) + ldo * (e / mR)]));
        b = x > b ? x : b;
    }
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long o = __shfl_xor(b, off);
        b = o > b ? o : b;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxbits, b);
}

// rebuild into a larger table (every entry is ready between batches)
__global__ void k_cache_rehash(const unsigned long long* __restrict__ ok, const double* __restrict__ ov,
                               int64_t ocap, unsigned long long* nk, double* nv, unsigned* ns, int64_t ncap) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < ocap; s += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = ok[s];
        if (key == kCacheEmpty) continue;
        int64_t t = (int64_t)(cache_hash(key) & (unsigned long long)(ncap - 1));
        for (;; t = (t + 1) & (ncap - 1))
            if (atomicCAS(&nk[t], kCacheEmpty, key) == kCacheEmpty) break;
        nv[t] = ov[s];
        ns[t] = 2;
    }
}

static unsigned grid_of(int64_t work) {
    int64_t g = (work + 255) / 256;
    return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

void launch_cache_partial_keys(hipStream_t s, const int32_t* T, int cnt, int w, const int64_t* coeff, int t0,
                               int64_t* out) {
    if (cnt <= 0) return;
    hipLaunchKernelGGL(k_cache_partial_keys, dim3((cnt + 255) / 256), dim3(256), 0, s, T, cnt, w, coeff, t0, out);
}

void launch_cache_probe(hipStream_t s, const CacheProbeArgs& a) {
    CacheProbe g{a.keys, a.vals, a.state, a.cap, a.kI, a.kJ, a.ccoef, a.m, a.mR, a.n, a.out, a.ldo, a.miss, a.dup,
                 a.counts};
    hipLaunchKernelGGL(k_cache_probe, dim3(grid_of(a.mR * a.n)), dim3(256), 0, s, g);
}

void launch_cache_gather_points(hipStream_t s, const int64_t* miss, int64_t nmiss, const int32_t* I, int nl,
                                const int32_t* J, int nr, int M, int64_t m, int64_t mR, int32_t* X) {
    if (nmiss <= 0) return;
    hipLaunchKernelGGL(k_cache_gather_points, dim3(grid_of(nmiss)), dim3(256), 0, s, miss, nmiss, I, nl, J, nr, M, m,
                       mR, X);
}

void launch_cache_fill(hipStream_t s, const int64_t* miss, int64_t nmiss, const double* v, double* vals,
                       unsigned* state, int64_t mR, double* out, int64_t ldo) {
    if (nmiss <= 0) return;
    hipLaunchKernelGGL(k_cache_fill, dim3(grid_of(nmiss)), dim3(256), 0, s, miss, nmiss, v, vals, state, mR, out,
                       ldo);
}

void launch_cache_dups(hipStream_t s, const CacheProbeArgs& a, int64_t ndup) {
    if (ndup <= 0) return;
    CacheProbe g{a.keys, a.vals, a.state, a.cap, a.kI, a.kJ, a.ccoef, a.m, a.mR, a.n, a.out, a.ldo, a.miss, a.dup,
                 a.counts};
    hipLaunchKernelGGL(k_cache_dups, dim3(grid_of(ndup)), dim3(256), 0, s, g, ndup);
}

void launch_cache_unclaim(hipStream_t s, const int64_t* miss, int64_t nmiss, unsigned long long* keys,
                          unsigned* state) {
    if (nmiss <= 0) return;
    hipLaunchKernelGGL(k_cache_unclaim, dim3(grid_of(nmiss)), dim3(256), 0, s, miss, nmiss, keys, state);
}

void launch_cache_lookup(hipStream_t s, const int32_t* X, int64_t npts, int L, const int64_t* coeff,
                         const unsigned long long* keys, const double* vals, const unsigned* state, int64_t cap,
                         int32_t* found, double* out) {
    if (npts <= 0) return;
    hipLaunchKernelGGL(k_cache_lookup, dim3(grid_of(npts)), dim3(256), 0, s, X, npts, L, coeff, keys, vals, state,
                       cap, found, out);
}

void launch_cache_maxabs(hipStream_t s, const double* out, int64_t mR, int64_t n, int64_t ldo,
                         unsigned long long* maxbits) {
    if (mR * n <= 0) return;
    hipLaunchKernelGGL(k_cache_maxabs, dim3(grid_of(mR * n)), dim3(256), 0, s, out, mR, n, ldo, maxbits);
}

void launch_cache_rehash(hipStream_t s, const unsigned long long* ok, const double* ov, int64_t ocap,
                         unsigned long long* nk, double* nv, unsigned* ns, int64_t ncap) {
    hipLaunchKernelGGL(k_cache_rehash, dim3(grid_of(ocap)), dim3(256), 0, s, ok, ov, ocap, nk, nv, ns, ncap);
}

}  // namespace tci
