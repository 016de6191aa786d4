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
#include "tci_internal.h"

// tci_abi.cpp: the device-resident small sweep (tci_sweep_small.hip)
bool tci_sweep_small_ok(tci_ctx* c, const tci_func* f, int L);
int tci_sweep_small_run(tci_ctx* c, const tci_func* f, int L, int64_t cap, const char* in, size_t inbytes,
                        int mode, int fill, int niter, int iter1, int strategy, int strictlynested, double abstol,
                        int64_t maxbonddim, std::vector<char>& out, const tci::SwSweep1* s1 = nullptr);
int tci_sweep_small_error(tci_ctx* c, int status, int64_t bond);
int tci_sweep_small_optimize(tci_ctx* c, const tci_func* f, int L, int64_t cap, const char* in, size_t inbytes,
                             double tol, int norm, int maxiter, int ncheck, int strictlynested, int64_t maxbonddim,
                             int fsolve, int64_t fill_tcap, const tci::SwSweep1* s1, std::vector<char>& out,
                             int* niter, int* ended, int* s1done, double* errors, int64_t* ranks, double* errnorm);

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

}  // extern "C"

namespace {

// The SwIO image of the state (tci_internal.h): banks 0..3 = Iset, Jset, the history's.
int64_t sw_capacity(const tci_tci2* s) {
    int64_t cap = 128;  // the small path's bonds keep at most min(m, n) <= 128 pivots
    for (int p = 0; p < s->L; ++p)
        cap = std::max({cap, s->I[p].count(), s->J[p].count(), s->hI[p].count(), s->hJ[p].count()});
    return cap;
}

std::vector<char> sw_pack(const tci_tci2* s) {
    const int L = s->L;
    const tci::SwIO io = tci::sw_io(L);
    const ISet* banks[4] = {s->I.data(), s->J.data(), s->hI.data(), s->hJ.data()};
    size_t bytes = io.sets;
    for (int b = 0; b < 4; ++b)
        for (int p = 0; p < L; ++p) bytes += banks[b][p].v.size() * 4;
    std::vector<char> img(bytes, 0);
    int64_t* hdr = reinterpret_cast<int64_t*>(img.data());
    hdr[3] = s->has_history ? 1 : 0;
    double ms = s->maxsample;
    memcpy(&hdr[6], &ms, 8);
    int64_t* cn = reinterpret_cast<int64_t*>(img.data() + io.counts);
    double* be = reinterpret_cast<double*>(img.data() + io.bonderr);
    for (int i = 0; i < L - 1; ++i) be[i] = s->bonderrors[i];
    char* dst = img.data() + io.sets;
    for (int b = 0; b < 4; ++b)
        for (int p = 0; p < L; ++p) {
            cn[(size_t)b * L + p] = banks[b][p].count();
            const size_t nbytes = banks[b][p].v.size() * 4;
            if (nbytes) memcpy(dst, banks[b][p].v.data(), nbytes);
            dst += nbytes;
        }
    return img;
}

struct SwOut {
    int64_t status = 0, it = 0, q = 0, bond = 0, fstatus = -1;
    bool extra = false;
    std::vector<ISet> eI, eJ;
};

// the kernel's results into the state (mode 0: sets, errors, maxsample; mode 1: maxsample)
SwOut sw_unpack(tci_tci2* s, const std::vector<char>& img, int mode) {
    const int L = s->L;
    const tci::SwIO io = tci::sw_io(L);
    const int64_t* hdr = reinterpret_cast<const int64_t*>(img.data());
    SwOut o;
    o.status = hdr[0];
    o.it = hdr[1];
    o.q = hdr[2];
    o.bond = hdr[7];
    o.fstatus = hdr[8];
    o.extra = o.status == 1 && hdr[4] != 0;
    memcpy(&s->maxsample, &hdr[6], 8);
    if (mode != 0) return o;
    s->has_history = hdr[3] != 0;
    const int64_t* cn = reinterpret_cast<const int64_t*>(img.data() + io.counts);
    const double* be = reinterpret_cast<const double*>(img.data() + io.bonderr);
    s->bonderrors.assign(be, be + (L - 1));
    const double* pe = reinterpret_cast<const double*>(img.data() + io.pe);
    s->pivoterrors.assign(pe, pe + hdr[5]);
    o.eI.resize(L);
    o.eJ.resize(L);
    std::vector<ISet>* banks[6] = {&s->I, &s->J, &s->hI, &s->hJ, &o.eI, &o.eJ};
    const char* src = img.data() + io.sets;
    for (int b = 0; b < (o.extra ? 6 : 4); ++b)
        for (int p = 0; p < L; ++p) {
            ISet& t = (*banks[b])[p];
            t.w = (b & 1) ? L - 1 - p : p;
            const int64_t c = cn[(size_t)b * L + p];
            if (t.w == 0) {
                t.v.clear();
                t.ncount0 = c;
            } else {
                t.v.resize((size_t)(c * t.w));
                memcpy(t.v.data(), src, (size_t)(c * t.w) * 4);
                src += (size_t)(c * t.w) * 4;
            }
        }
    return o;
}

}  // namespace

extern "C" {

int tci_tci2_set_sets(tci_tci2* s, int which, const int64_t* counts, const int32_t* packed) {
    if (!s || !counts || which < 0 || which > 3) return TCI_ERR_ARG;
    std::vector<ISet>& bank = which == 0 ? s->I : which == 1 ? s->J : which == 2 ? s->hI : s->hJ;
    const int32_t* src = packed;
    for (int p = 0; p < s->L; ++p) {
        ISet& t = bank[p];
        if (counts[p] < 0 || (counts[p] > 0 && t.w > 0 && !src)) return TCI_ERR_ARG;
        if (t.w == 0) {
            t.v.clear();
            t.ncount0 = counts[p];
        } else {
            t.v.assign(src, src + counts[p] * t.w);
            src += counts[p] * t.w;
        }
    }
    if (which >= 2) s->has_history = true;
    return TCI_OK;
}

int tci_tci2_get_sets(tci_tci2* s, int which, int64_t* counts, int32_t* packed, int64_t capacity) {
    if (!s || !counts || which < 0 || which > 3) return TCI_ERR_ARG;
    const std::vector<ISet>& bank = which == 0 ? s->I : which == 1 ? s->J : which == 2 ? s->hI : s->hJ;
    int64_t need = 0;
    for (int p = 0; p < s->L; ++p) {
        counts[p] = bank[p].count();
        need += (int64_t)bank[p].v.size();
    }
    if (!packed) return TCI_OK;
    if (capacity < need) return TCI_ERR_ARG;
    int32_t* dst = packed;
    for (int p = 0; p < s->L; ++p) {
        if (!bank[p].v.empty()) memcpy(dst, bank[p].v.data(), bank[p].v.size() * 4);
        dst += bank[p].v.size();
    }
    return TCI_OK;
}

}  // extern "C"

namespace {

// sweepstrategy: 0 = backandforth, 1 = forward, 2 = backward (sweepstrategies.jl:41-50). fill:
// also fillsitetensors!'s maxsample update on the device after the iterations (*filled = 1 when
// it was done there).
// (solve: the fill also solves every site tensor, tensors / capacity / offsets as tci_tci2_sweep1site)
int sweep2site_impl(tci_tci2* s, const tci_func* f, int32_t niter, int32_t iter1, double abstol,
                    int64_t maxbonddim, int32_t sweepstrategy, int32_t strictlynested, int fill, int* filled,
                    const tci::SwSweep1* solve = nullptr) {
    if (!s || !f || niter < 0) return TCI_ERR_ARG;
    if (filled) *filled = 0;
    const int L = s->L;
    int it0 = iter1, q0 = 1;
    bool resume = false;
    SwOut so;
    if (niter > 0 && tci_sweep_small_ok(s->ctx, f, L)) {
        // whole iterations in one launch while every bond fits the one-workgroup rrLU
        const std::vector<char> in = sw_pack(s);
        std::vector<char> out;
        int st = tci_sweep_small_run(s->ctx, f, L, sw_capacity(s), in.data(), in.size(), 0, fill ? 1 : 0, niter,
                                     iter1, sweepstrategy, strictlynested, abstol, maxbonddim, out,
                                     fill ? solve : nullptr);
        if (st) return st;
        so = sw_unpack(s, out, 0);
        if (so.status == 0) {
            // a fill that stopped (non-square pivot matrix, a site too large) is redone by the
            // caller's loop: the sites it covered only repeat their maxima
            if (filled) *filled = fill && so.fstatus == 0;
            return TCI_OK;
        }
        if (so.status != 1) return tci_sweep_small_error(s->ctx, (int)so.status, so.bond);
        it0 = (int)so.it;  // a bond outgrew it: this loop continues from there
        q0 = (int)so.q;
        resume = true;
    }
    for (int it = it0; it < iter1 + niter; ++it) {
        std::vector<ISet> eI, eJ;
        bool extra;
        int qs = 1;
        if (resume && it == it0) {  // the kernel already began this iteration
            extra = so.extra;
            eI.swap(so.eI);
            eJ.swap(so.eJ);
            qs = q0;
        } else {
            extra = !strictlynested && s->has_history;
            if (extra) {
                eI = s->hI;
                eJ = s->hJ;
            }
            s->hI = s->I;
            s->hJ = s->J;
            s->has_history = true;
            s->pivoterrors.clear();  // flushpivoterror!
        }
        const bool fwd = sweepstrategy == 1 || (sweepstrategy == 0 && it % 2 == 1);
        for (int q = qs; q < L; ++q) {
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

}  // namespace

extern "C" {

int tci_tci2_sweep2site(tci_tci2* s, const tci_func* f, int32_t niter, int32_t iter1, double abstol,
                        int64_t maxbonddim, int32_t sweepstrategy, int32_t strictlynested) {
    return sweep2site_impl(s, f, niter, iter1, abstol, maxbonddim, sweepstrategy, strictlynested, 0, nullptr);
}

int tci_tci2_sweep2site_fill(tci_tci2* s, const tci_func* f, int32_t niter, int32_t iter1, double abstol,
                             int64_t maxbonddim, int32_t sweepstrategy, int32_t strictlynested, int* filled) {
    if (!filled) return TCI_ERR_ARG;
    return sweep2site_impl(s, f, niter, iter1, abstol, maxbonddim, sweepstrategy, strictlynested, 1, filled);
}

int tci_tci2_sweep2site_fillsolve(tci_tci2* s, const tci_func* f, int32_t niter, int32_t iter1, double abstol,
                                  int64_t maxbonddim, int32_t sweepstrategy, int32_t strictlynested,
                                  double* tensors, int64_t capacity, int64_t* offsets, int* filled) {
    if (!s || !filled || !tensors || !offsets || capacity < 0) return TCI_ERR_ARG;
    for (int i = 0; i < 2 * s->L; ++i) offsets[i] = 0;
    const tci::SwSweep1 sv{0, 1, 1e-14, capacity, offsets, tensors};
    return sweep2site_impl(s, f, niter, iter1, abstol, maxbonddim, sweepstrategy, strictlynested, 1, filled, &sv);
}


// sweep1site! (tensorci2.jl:659-725) in one launch of the device-resident sweep (mode 2) when every
// bond fits the one-workgroup rrLU; *handled = 0 (state untouched) otherwise or on any error, and the
// host loop runs it. Site tensors (updatetensors) into tensors[offsets[2 p] ..] of offsets[2 p + 1]
// doubles (column-major, the shape of site p: len(Iset[p]) * d x len(Jset[p]) or its transpose
// layout of the right factor, as tci_update_pivots_h returns them).
int tci_tci2_sweep1site(tci_tci2* s, const tci_func* f, int32_t forward, double reltol, double abstol,
                        int64_t maxbonddim, int32_t updatetensors, double* tensors, int64_t capacity,
                        int64_t* offsets, int* handled) {
    if (!s || !f || !handled || (updatetensors && (!tensors || !offsets || capacity < 0))) return TCI_ERR_ARG;
    *handled = 0;
    if (!tci_sweep_small_ok(s->ctx, f, s->L)) return TCI_OK;
    const std::vector<char> in = sw_pack(s);
    std::vector<char> out;
    tci::SwSweep1 s1{forward ? 1 : 0, updatetensors ? 1 : 0, reltol, updatetensors ? capacity : 0,
                     updatetensors ? offsets : nullptr, updatetensors ? tensors : nullptr};
    if (updatetensors)
        for (int i = 0; i < 2 * s->L; ++i) offsets[i] = 0;
    int st = tci_sweep_small_run(s->ctx, f, s->L, sw_capacity(s), in.data(), in.size(), 2, 0, 0, 1, 0, 0, abstol,
                                 maxbonddim, out, &s1);
    if (st) return st;
    const int64_t status = reinterpret_cast<const int64_t*>(out.data())[0];
    if (status != 0) return TCI_OK;  // the host loop redoes it (and raises the reference's errors)
    sw_unpack(s, out, 0);
    *handled = 1;
    return TCI_OK;
}

// optimize! (tensorci2.jl:1018-1172) without a global pivot search, as one chain of device launches
// (tci_sweep_small_optimize): the sweep2site! iterations with fillsitetensors! after each (solved
// when solvefill, else the maxsample update only), the convergence test on the device, then
// sweep1site!(forward, abstol = tolerance * maxsample) with its site tensors. *handled: 0 nothing
// done (state untouched); 1 with *ended = 1 and *s1done = 1 everything done; otherwise the state
// after the first *niter iterations -- the caller continues the loop (*ended = 0) or runs the closing
// sweep1site! (*ended = 1) on its own path. errors / ranks: iteration i at [i - 1]; *errnorm: the
// maxsample the closing sweep normalised with.
int tci_tci2_optimize_small(tci_tci2* s, const tci_func* f, double tolerance, int64_t maxbonddim, int32_t maxiter,
                            int32_t ncheckhistory, int32_t normalizeerror, int32_t strictlynested, int32_t solvefill,
                            double* tensors, int64_t capacity, int64_t* offsets, double* errors, int64_t* ranks,
                            int32_t* niter, int32_t* ended, int32_t* s1done, double* errnorm, int* handled) {
    if (!s || !f || !handled || !niter || !ended || !s1done || !errnorm || !errors || !ranks || !tensors ||
        !offsets || capacity < 0)
        return TCI_ERR_ARG;
    *handled = 0;
    *niter = *ended = *s1done = 0;
    if (maxiter < 1 || maxiter >= tci::kSwOptMax || ncheckhistory < 1 || !tci_sweep_small_ok(s->ctx, f, s->L))
        return TCI_OK;
    const std::vector<char> in = sw_pack(s);
    std::vector<char> out;
    for (int i = 0; i < 2 * s->L; ++i) offsets[i] = 0;
    const tci::SwSweep1 s1{1, 1, 1e-14, capacity, offsets, tensors};
    std::vector<double> e(tci::kSwOptMax + 1, 0.0);
    std::vector<int64_t> r(tci::kSwOptMax + 1, 0);
    int n = 0, en = 0, sd = 0;
    double norm = 0.0;
    int st = tci_sweep_small_optimize(s->ctx, f, s->L, sw_capacity(s), in.data(), in.size(), tolerance,
                                      normalizeerror, maxiter, ncheckhistory, strictlynested, maxbonddim, solvefill,
                                      capacity, &s1, out, &n, &en, &sd, e.data(), r.data(), &norm);
    if (st) return st;
    if (n == 0 && !en) return TCI_OK;  // nothing ran on the device
    sw_unpack(s, out, 0);
    for (int i = 0; i < n; ++i) {
        errors[i] = e[i + 1];
        ranks[i] = r[i + 1];
    }
    *niter = n;
    *ended = en;
    *s1done = sd;
    *errnorm = norm;
    *handled = 1;
    return TCI_OK;
}

int fill_impl(tci_tci2* s, const tci_func* f, int* handled, const tci::SwSweep1* solve) {
    if (!s || !f || !handled) return TCI_ERR_ARG;
    *handled = 0;
    if (!tci_sweep_small_ok(s->ctx, f, s->L)) return TCI_OK;
    const std::vector<char> in = sw_pack(s);
    std::vector<char> out;
    const double before = s->maxsample;
    int st = tci_sweep_small_run(s->ctx, f, s->L, sw_capacity(s), in.data(), in.size(), 1, 0, 0, 1, 0, 0, 0.0,
                                 0, out, solve);
    if (st) return st;
    const SwOut so = sw_unpack(s, out, 1);
    if (so.fstatus != 0) {  // the caller's loop reports it / evaluates the large site
        s->maxsample = before;
        return TCI_OK;
    }
    *handled = 1;
    return TCI_OK;
}

int tci_tci2_fill_maxsample(tci_tci2* s, const tci_func* f, int* handled) { return fill_impl(s, f, handled, nullptr); }

int tci_tci2_fill_solve(tci_tci2* s, const tci_func* f, double* tensors, int64_t capacity, int64_t* offsets,
                        int* handled) {
    if (!s || !tensors || !offsets || capacity < 0) return TCI_ERR_ARG;
    for (int i = 0; i < 2 * s->L; ++i) offsets[i] = 0;
    const tci::SwSweep1 sv{0, 1, 1e-14, capacity, offsets, tensors};
    return fill_impl(s, f, handled, &sv);
}

}  // extern "C"
