// tci_sweep.cpp -- the per-bond loop of sweep2site! (tensorci2.jl:1195-1258) in C++ behind one ABI
// call (tci_tci2_sweep2site): kronecker products of the index sets (tensorci2.jl:512-529), Julia's
// first-seen `union` with the previous sweep's sets when not strictly nested (:1214-1216), the
// 2-site update on the device (tci_update_pivots_h: Pi in HBM -> maxabs -> rrLU -> pivots), the
// new pivot sets, updatemaxsample! (:636-638, Julia's NaN-propagating max) and updateerrors!
// (:281-289). Host integer work only; every flop runs in the device kernels. The TCI2 state lives
// in a tci_tci2 object the host mirror fills and reads back around the call (tci_amd/tensorci2.py).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/tci_hip.h"

namespace {

// an index set: count entries of width w, row-major (entry e at v[e * w])
struct ISet {
    int32_t w = 0;
    std::vector<int32_t> v;
    int64_t count() const { return w ? (int64_t)v.size() / w : ncount0; }
    int64_t ncount0 = 0;  // width-0 sets: the number of (empty) entries
};

double jl_max(double x, double y) {  // Base.max for Float64
    if (std::isnan(x)) return x;
    if (std::isnan(y)) return y;
    if (y > x || (y == x && std::signbit(x) && !std::signbit(y))) return y;
    return x;
}

// kronecker(Iset, d): [is..., j] with Iset fastest (tensorci2.jl:512-517)
ISet kron_right(const ISet& I, int d) {
    ISet o;
    o.w = I.w + 1;
    const int64_t n = I.count();
    o.v.reserve((size_t)(n * d * o.w));
    for (int j = 1; j <= d; ++j)
        for (int64_t e = 0; e < n; ++e) {
            for (int t = 0; t < I.w; ++t) o.v.push_back(I.v[e * I.w + t]);
            o.v.push_back(j);
        }
    return o;
}

// kronecker(d, Jset): [i, js...] with i fastest (:524-529)
ISet kron_left(int d, const ISet& J) {
    ISet o;
    o.w = J.w + 1;
    const int64_t n = J.count();
    o.v.reserve((size_t)(n * d * o.w));
    for (int64_t e = 0; e < n; ++e)
        for (int i = 1; i <= d; ++i) {
            o.v.push_back(i);
            for (int t = 0; t < J.w; ++t) o.v.push_back(J.v[e * J.w + t]);
        }
    return o;
}

// union(a, b) of Vector{MultiIndex}: first-seen order, deduplicated
ISet union_sets(const ISet& a, const ISet* b) {
    ISet o;
    o.w = a.w;
    if (a.w == 0) {
        o.ncount0 = (a.count() + (b ? b->count() : 0)) > 0 ? 1 : 0;
        return o;
    }
    std::unordered_map<std::string, char> seen;
    seen.reserve((size_t)(a.count() + (b ? b->count() : 0)) * 2);
    auto add = [&](const ISet& s) {
        for (int64_t e = 0; e < s.count(); ++e) {
            std::string k(reinterpret_cast<const char*>(&s.v[e * s.w]), sizeof(int32_t) * s.w);
            if (seen.emplace(std::move(k), 1).second)
                o.v.insert(o.v.end(), s.v.begin() + e * s.w, s.v.begin() + (e + 1) * s.w);
        }
    };
    add(a);
    if (b && b->w == a.w) add(*b);
    return o;
}

ISet select(const ISet& s, const std::vector<int64_t>& idx1) {  // 1-based positions
    ISet o;
    o.w = s.w;
    if (s.w == 0) {
        o.ncount0 = (int64_t)idx1.size();
        return o;
    }
    o.v.reserve(idx1.size() * s.w);
    for (int64_t p : idx1) o.v.insert(o.v.end(), s.v.begin() + (p - 1) * s.w, s.v.begin() + p * s.w);
    return o;
}

}  // namespace

struct tci_tci2 {
    tci_ctx* ctx = nullptr;
    int L = 0;
    std::vector<int32_t> localdims;
    std::vector<ISet> I, J;        // Iset[p] (width p), Jset[p] (width L - 1 - p)
    std::vector<ISet> hI, hJ;      // the last sweep's sets (Iset_history[end])
    bool has_history = false;
    std::vector<double> pivoterrors, bonderrors;
    double maxsample = 0.0;
    std::string err;
};

extern "C" {

int tci_tci2_create(tci_ctx* ctx, int32_t L, const int32_t* localdims, tci_tci2** out) {
    if (!ctx || !out || L < 2 || !localdims) return TCI_ERR_ARG;
    tci_tci2* s = new tci_tci2();
    s->ctx = ctx;
    s->L = L;
    s->localdims.assign(localdims, localdims + L);
    s->I.resize(L);
    s->J.resize(L);
    s->hI.resize(L);
    s->hJ.resize(L);
    for (int p = 0; p < L; ++p) {
        s->I[p].w = s->hI[p].w = p;
        s->J[p].w = s->hJ[p].w = L - 1 - p;
    }
    s->bonderrors.assign(L - 1, 0.0);
    *out = s;
    return TCI_OK;
}

int tci_tci2_destroy(tci_tci2* s) {
    delete s;
    return TCI_OK;
}

// which: 0 = Iset[p], 1 = Jset[p], 2 = Iset_history[p], 3 = Jset_history[p]
int tci_tci2_set_set(tci_tci2* s, int which, int32_t p, const int32_t* entries, int64_t count) {
    if (!s || which < 0 || which > 3 || p < 0 || p >= s->L || count < 0 || (count > 0 && !entries && p > 0))
        return TCI_ERR_ARG;
    ISet& t = (which == 0 ? s->I : which == 1 ? s->J : which == 2 ? s->hI : s->hJ)[p];
    if (t.w == 0) {
        t.v.clear();
        t.ncount0 = count;
    } else {
        t.v.assign(entries, entries + count * t.w);
    }
    if (which >= 2) s->has_history = true;
    return TCI_OK;
}

int tci_tci2_get_set(tci_tci2* s, int which, int32_t p, int32_t* entries, int64_t capacity, int64_t* count) {
    if (!s || !count || which < 0 || which > 3 || p < 0 || p >= s->L) return TCI_ERR_ARG;
    const ISet& t = (which == 0 ? s->I : which == 1 ? s->J : which == 2 ? s->hI : s->hJ)[p];
    *count = t.count();
    if (entries && t.w > 0) {
        const int64_t n = std::min<int64_t>(capacity, t.count());
        memcpy(entries, t.v.data(), (size_t)(n * t.w) * sizeof(int32_t));
    }
    return TCI_OK;
}

int tci_tci2_clear_history(tci_tci2* s) {
    if (!s) return TCI_ERR_ARG;
    s->has_history = false;
    return TCI_OK;
}

int tci_tci2_errors(tci_tci2* s, double* maxsample, double* bonderrors, double* pivoterrors, int64_t capacity,
                    int64_t* npivoterrors) {
    if (!s) return TCI_ERR_ARG;
    if (maxsample) *maxsample = s->maxsample;
    if (bonderrors) memcpy(bonderrors, s->bonderrors.data(), (s->L - 1) * sizeof(double));
    if (npivoterrors) *npivoterrors = (int64_t)s->pivoterrors.size();
    if (pivoterrors)
        memcpy(pivoterrors, s->pivoterrors.data(),
               std::min<size_t>((size_t)capacity, s->pivoterrors.size()) * sizeof(double));
    return TCI_OK;
}

int tci_tci2_set_errors(tci_tci2* s, double maxsample, const double* bonderrors, const double* pivoterrors,
                        int64_t npivoterrors) {
    if (!s) return TCI_ERR_ARG;
    s->maxsample = maxsample;
    if (bonderrors) s->bonderrors.assign(bonderrors, bonderrors + s->L - 1);
    s->pivoterrors.assign(pivoterrors ? pivoterrors : nullptr, pivoterrors ? pivoterrors + npivoterrors : nullptr);
    return TCI_OK;
}

// sweepstrategy: 0 = backandforth, 1 = forward, 2 = backward (sweepstrategies.jl:41-50)
int tci_tci2_sweep2site(tci_tci2* s, const tci_func* f, int32_t niter, int32_t iter1, double abstol,
                        int64_t maxbonddim, int32_t sweepstrategy, int32_t strictlynested) {
    if (!s || !f || niter < 0) return TCI_ERR_ARG;
    const int L = s->L;
    for (int it = iter1; it < iter1 + niter; ++it) {
        const bool extra = !strictlynested && s->has_history;
        std::vector<ISet> eI, eJ;
        if (extra) {
            eI = s->hI;
            eJ = s->hJ;
        }
        s->hI = s->I;
        s->hJ = s->J;
        s->has_history = true;
        s->pivoterrors.clear();  // flushpivoterror!
        const bool fwd = sweepstrategy == 1 || (sweepstrategy == 0 && it % 2 == 1);
        for (int q = 1; q < L; ++q) {
            const int b = fwd ? q : L - q;  // 1-based bond
            const ISet Ik = kron_right(s->I[b - 1], s->localdims[b - 1]);
            const ISet Jk = kron_left(s->localdims[b], s->J[b]);
            const ISet Icomb = union_sets(Ik, extra ? &eI[b] : nullptr);
            const ISet Jcomb = union_sets(Jk, extra ? &eJ[b - 1] : nullptr);
            const int64_t m = Icomb.count(), n = Jcomb.count();
            const int64_t mr = std::max<int64_t>(std::min<int64_t>(std::min<int64_t>(maxbonddim, m), n), 0);
            std::vector<int64_t> rowidx(std::max<int64_t>(mr, 1)), colidx(std::max<int64_t>(mr, 1));
            std::vector<double> pe(mr + 1);
            int64_t np = 0;
            double mx = 0.0;
            const int st = tci_update_pivots_h(s->ctx, f, Icomb.v.data(), m, Icomb.w, Jcomb.v.data(), n, Jcomb.w,
                                               maxbonddim, 1e-14, abstol, fwd ? 1 : 0, 0, rowidx.data(),
                                               colidx.data(), pe.data(), &np, &mx, nullptr, nullptr);
            if (st) return st;
            s->maxsample = jl_max(fabs(s->maxsample), fabs(mx));  // maxabs (util.jl:34-43)
            rowidx.resize(np);
            colidx.resize(np);
            s->I[b] = select(Icomb, rowidx);
            s->J[b - 1] = select(Jcomb, colidx);
            // updateerrors!(tci, b, pivoterrors(lu)) (tensorci2.jl:281-289)
            s->bonderrors[b - 1] = pe[np];
            const size_t ne = std::max(s->pivoterrors.size(), (size_t)(np + 1));
            std::vector<double> upd(ne, 0.0);
            for (size_t i = 0; i < ne; ++i)
                upd[i] = jl_max(i < s->pivoterrors.size() ? s->pivoterrors[i] : 0.0,
                                i < (size_t)(np + 1) ? pe[i] : 0.0);
            s->pivoterrors.swap(upd);
        }
    }
    return TCI_OK;
}

}  // extern "C"
