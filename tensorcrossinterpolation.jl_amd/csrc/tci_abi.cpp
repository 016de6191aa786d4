// tci_abi.cpp -- the C ABI of libtci_hip.so (include/tci_hip.h): contexts, device workspaces and
// the host-side orchestration of the per-pivot kernel sequence. All compute is in
// tci_device.hip; nothing here falls back to the CPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cstddef>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/tci_hip.h"
#include "tci_internal.h"

using tci::Cand;
using tci::FuncDev;
using tci::RrluState;

struct tci_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // workspaces (grown on demand, reused across calls)
    double* dA = nullptr;
    size_t capA = 0;  // doubles
    Cand* cand = nullptr;
    size_t capCand = 0;
    RrluState* st = nullptr;
    RrluState* hst = nullptr;  // pinned
    int64_t* rowperm = nullptr;
    int64_t* colperm = nullptr;
    size_t capPerm = 0;
    size_t capColperm = 0;
    double* xbuf = nullptr;  // pending rank-1 update vectors (tci_rrlu.hip)
    size_t capX = 0;
    double* ybuf = nullptr;
    size_t capY = 0;
    int flush_every = 10;  // deferred-update depth nb: the shadow epoch (1 = write back every pivot)
    int epochs = 0;        // shadow epochs per fp64 write-back (two-level epoch; 0 = by shape; env TCI_RRLU_EPOCHS)
    int serpentine = 1;    // alternate the pass's tile order (env TCI_RRLU_SERP=0 disables)
    int shadow = 1;        // certified fp32 search in read-only passes (env TCI_RRLU_SHADOW=0)
    int pass_gridx = 1;    // rrLU pass workgroups per CU (env TCI_PASS_GRIDX; 1 = all resident at once)
    int pass_griddiv = 1;  // A/B: the pass grid over this many fewer CUs (env TCI_PASS_GRIDDIV)
    float* sbuf = nullptr; // its fp32 shadow of the matrix
    size_t capS = 0;
    int small_path = 1;    // single-workgroup LDS rrLU for small matrices (env TCI_RRLU_SMALL=0)
    int mid_path = 1;      // persistent LDS-resident rrLU for mid-size matrices (env TCI_RRLU_MID=0)
    int mid_faulted = 0;   // its grid barrier timed out once on this context: pass pipeline from then on
    int persist = 0;       // read-only passes of a shadow epoch as one persistent launch (env TCI_RRLU_PERSIST=1;
                           // off by default: measured slower)
    int persist_faulted = 0;  // such a launch found its grid not co-resident: per-pass launches from then on
    int persist_kinds = 3;    // diagnostic (env TCI_EPOCH_KINDS): bit 0 first shadow epochs, bit 1 later ones (EXT)
    int persist_maxpass = 1 << 30;  // diagnostic (env TCI_EPOCH_MAXPASS): passes per persistent launch at most
    unsigned* esync = nullptr;  // their sync slots (tci_rrlu.hip k_pass_mf_epoch), one per launch
    size_t capEsync = 0;
    int dense = tci::kDenseAll;  // fp64 MFMA forms of the factors / solve (env TCI_DENSE_MFMA mask)
    int c128_nb = -1;            // ComplexF64 rrLU deferred-update depth (env TCI_C128_NB; 0: round 1;
                                 // -1: 11 with the shadow search, 6 without -- measured best)
    int c128_sh = 1;             // ComplexF64 rrLU certified shadow search (env TCI_C128_SH)
    int ncu = 0;           // compute units of the device
    double* colbuf = nullptr;  // mid path: published candidate columns
    size_t capColbuf = 0;
    unsigned* bar = nullptr;   // mid path: grid-barrier counter
    int* fault = nullptr;      // mid path: barrier timeout flag
    int* flag = nullptr;
    unsigned* ticket = nullptr;  // rrLU pass tail hand-off counters: [0] top, [16 (1 + c)] XCD class c (zero between passes)
    char* hin = nullptr;         // pinned staging for uploads / downloads of the small path
    size_t capHin = 0;
    char* hout = nullptr;
    size_t capHout = 0;
    char* hd2h = nullptr;  // d2h_large's two pinned chunk slots
    size_t capHd2h = 0;
    hipEvent_t d2h_ev[2] = {nullptr, nullptr};
    char* zbuf = nullptr;  // mapped pinned host memory the small path's kernels write into
    char* zdev = nullptr;  // its device address
    int small_sweep = 1;   // device-resident small sweeps (tci_sweep_small.hip; env TCI_SWEEP_SMALL=0)
    int sw_lu_wave = 1;    // their bonds with m, n <= 32 on the one-wave rrLU (env TCI_SW_LUWAVE=0: off)
    int sw_lazy_union = 1;  // their unions without materialised kronecker products (env TCI_SW_LAZYU=0: off)
    int32_t* sw_ws = nullptr;   // their six banks of index sets
    size_t capSwWs = 0;
    char* sw_inbuf = nullptr;   // device copy of the input image
    size_t capSwInbuf = 0;
    char* sw_in = nullptr;      // mapped host I/O images (SwIO)
    char* sw_in_d = nullptr;
    size_t capSwIn = 0;
    char* sw_out = nullptr;
    char* sw_out_d = nullptr;
    size_t capSwOut = 0;
    double* sw_tens = nullptr;  // sweep1site's site tensors (device)
    size_t capSwTens = 0;
    int32_t* sw_fmap = nullptr;  // the fill's map of the current sets (device; k_fill_sites)
    size_t capSwFmap = 0;
    char* sw_fmax = nullptr;     // the fill's per-site max |Pi1| bits (mapped host memory)
    char* sw_fmax_d = nullptr;
    size_t capSwFmax = 0;
    char* sw_img[2] = {nullptr, nullptr};  // chained optimize!: the iterations' images (device, ping-pong)
    size_t capSwImg[2] = {0, 0};
    unsigned long long* sw_ctl = nullptr;  // chained optimize!: control words (SweepSmallArgs.ctl)
    size_t capSwCtl = 0;
    char* hctl = nullptr;                  // their pinned host copy
    size_t capHctl = 0;
    char* sw_s1t = nullptr;                // chained optimize!: the closing sweep's site tensors (mapped host)
    char* sw_s1t_d = nullptr;
    size_t capSwS1t = 0;
    size_t capZ = 0;
    int* hflag = nullptr;  // pinned
    RrluState* hpoll = nullptr;  // pinned, two slots: rrLU stop-flag polling (StopPoll)
    hipEvent_t pollev[2] = {nullptr, nullptr};
    unsigned long long* maxbits = nullptr;
    unsigned long long* hmaxbits = nullptr;  // pinned
    void* scratch = nullptr;
    size_t capScratch = 0;
    char* scratch2 = nullptr;  // tensor-train evaluation block
    size_t capScratch2 = 0;
    int32_t* dI = nullptr;
    size_t capI = 0;
    // tci_batcheval_da's own index tables and pinned stage (no other entry touches them, so its
    // uploads may still be in flight when the call returns); ev_ina: its last upload
    int32_t* dIa = nullptr;
    size_t capIa = 0;
    int32_t* dJa = nullptr;
    size_t capJa = 0;
    char* hina = nullptr;
    size_t capHina = 0;
    hipEvent_t ev_ina = nullptr;
    bool ev_ina_live = false;
    int32_t* dJ = nullptr;
    size_t capJ = 0;
    int32_t* dI2 = nullptr;
    size_t capI2 = 0;
    double* dF1 = nullptr;  // factor / auxiliary buffers
    size_t capF1 = 0;
    double* dF2 = nullptr;
    size_t capF2 = 0;
    double* dDiag = nullptr;
    size_t capDiag = 0;
    int* dPiv = nullptr;
    size_t capPiv = 0;
    double* dPbak = nullptr;  // P kept for a cooperative getrf that gave up (solve_launch)
    size_t capPbak = 0;
    int* hCoop = nullptr;     // pinned: the fault word read back
    int coop_faults = 0;      // cooperative getrfs that gave up (diagnostic)
    // rrLU results (tci_rrlu.hip): position maps, pivot values, physical-order L / U, and the
    // position-order L / U extracted from them
    int32_t* rowpos = nullptr;
    size_t capRowpos = 0;
    int32_t* colpos = nullptr;
    size_t capColpos = 0;
    double* pivv = nullptr;
    size_t capPivv = 0;
    double* Lp = nullptr;
    size_t capLp = 0;
    double* Up = nullptr;
    size_t capUp = 0;
    int64_t ldUp = 1;
    double* dL = nullptr;
    size_t capL = 0;
    double* dU = nullptr;
    size_t capU = 0;
    // column-sharded rrLU: local column positions (+ ghost), exchange records, local winner
    int32_t* colposL = nullptr;
    size_t capColposL = 0;
    double* shsend = nullptr;
    size_t capShSend = 0;
    double* shrecv = nullptr;
    size_t capShRecv = 0;
    int sh_exchange = 0;       // per-pivot exchange: 0 by size, 1 two collectives, 2 fused (one all-gather)
    int sh_exchange_used = 0;  // what the last sharded rrLU ran (0: none, one rank without a communicator)
    Cand* lout = nullptr;
    size_t capLout = 0;
    int64_t sh_np = 0, sh_nloc = 0, sh_c0 = 0, sh_m = 0, sh_n = 0;
    int sh_valid = 0;  // the rrLU buffers hold the last tci_rrlu_sharded_d's result (no other rrLU since)
    int sh_leftorth = 1;
    char* cws = nullptr;  // ComplexF64 rrLU: state, candidates, pivot column / row buffers
    size_t capCws = 0;
    double* dRe = nullptr;  // ComplexF64 2-site update: real values of f before the scaling
    size_t capRe = 0;
    char* hfn = nullptr;    // pinned: the batch a host integrand (TCI_F_HOST) fills
    size_t capHfn = 0;
    // kernel timing (family 0: rrLU pass with write-back, 1: batch evaluation,
    //                2: rrLU read-only pass)
    bool timing = false;
    int timing_stride = 1;  // rrLU passes: only every timing_stride-th pivot's pass is timed
    std::vector<hipEvent_t> evpool;
    size_t evused = 0;
    // (family, sub-family or -1, index of start event); sub-families 3 + P: read-only rrLU pass
    // with P pending updates
    struct EvPair {
        int fam, sub;
        size_t idx;
        int units;  // passes the timed launch covers (1, or a persistent epoch launch's count)
    };
    std::vector<EvPair> evpairs;
    // + 20 solve, 21 LUCI factors, 22 K3, 23 refresh, 24 + P read-only passes of a later shadow epoch
    // (EXT: the exact epoch is longer; 3 + P: the first shadow epoch after a write-back), 41 / 42
    // persistent epoch launches (first shadow epoch / EXT; units = passes), 43 pass 0 (the exact pass
    // after pivot 0 that writes the shadow of A)
    static constexpr int kFamEpoch = 3 + tci::kMaxPend + 1 + 4 + tci::kMaxPend + 1;
    static constexpr int kFamPass0 = kFamEpoch + 2;
    static constexpr int kFams = kFamPass0 + 1;
    double fam_ms[kFams] = {};
    int64_t fam_n[kFams] = {};
    int64_t fam_u[kFams] = {};
};

struct tci_comm {
    tci_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;
    int nranks = 1, rank = 0;
};

struct tci_cache {
    tci_ctx* ctx = nullptr;
    int L = 0;
    std::vector<int64_t> coeffs;
    int64_t* dcoeff = nullptr;
    unsigned long long* keys = nullptr;
    double* vals = nullptr;
    unsigned* state = nullptr;
    int64_t cap = 0, size = 0;
    int64_t *kI = nullptr, *kJ = nullptr, *miss = nullptr, *dup = nullptr;
    size_t capKI = 0, capKJ = 0, capMiss = 0, capDup = 0;
    int32_t* X = nullptr;
    size_t capX = 0;
    double* mv = nullptr;
    size_t capMv = 0;
    unsigned long long* counts = nullptr;
    unsigned long long* hcounts = nullptr;
};

struct tci_func {
    tci_ctx* ctx = nullptr;
    int kind = 0;
    int L = 0;
    std::vector<int32_t> localdims;
    double* dparams = nullptr;
    int32_t* dld = nullptr;
    int64_t* dstrides = nullptr;
    int64_t nparams = 0;
    int32_t cpK = 0;
    int64_t ntab = 0;
    int32_t mpoEnv = 0, mpoTmp = 0;
    tci_host_fn hostfn = nullptr;  // TCI_F_HOST: the user's f on the host (tci_func_create_host)
    void* hostuser = nullptr;
    std::vector<const tci_func*> cparts;  // TCI_F_C128: real parts, then imaginary parts
    int32_t cnre = 0;
    FuncDev view() const {
        FuncDev f;
        f.cpK = cpK;
        f.ntab = ntab;
        f.mpoEnv = mpoEnv;
        f.mpoTmp = mpoTmp;
        f.kind = kind;
        f.L = L;
        f.localdims = dld;
        f.params = dparams;
        f.nparams = nparams;
        f.strides = dstrides;
        return f;
    }
};

namespace {

int set_err(tci_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                    \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, TCI_ERR_DEVICE,                                              \
                           std::string(#expr) + ": " + hipGetErrorString(e_));               \
    } while (0)

template <class T>
int ensure(tci_ctx* c, T** p, size_t* cap, size_t n) {
    if (n <= *cap && *p) return TCI_OK;
    size_t want = std::max<size_t>(n, 64);
    if (*p) {
        hipStreamSynchronize(c->stream);
        hipFree(*p);
        *p = nullptr;
        *cap = 0;
    }
    if (hipMalloc((void**)p, want * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return set_err(c, TCI_ERR_NOMEM, "device allocation of " + std::to_string(want * sizeof(T)) +
                                             " bytes failed");
    }
    *cap = want;
    return TCI_OK;
}

// fp16 shadow: its padding rows [m, lds) of every column are read by the MFMA search (as part of
// a lane's 16-row load) and must be zero; no pass writes them
int zero_shadow_pad(tci_ctx* c, int64_t lds, int64_t m, int64_t n) {
    const int eb = tci::shadow_elem_bytes();
    if (eb > 2 || lds <= m || n <= 0) return TCI_OK;
    // the shadow of 0: fp16 0x0000, 8-bit code 0x80 (offset binary)
    HIPCHK(c, hipMemset2DAsync(reinterpret_cast<char*>(c->sbuf) + eb * m, (size_t)(eb * lds), eb == 1 ? 0x80 : 0,
                               (size_t)(eb * (lds - m)), (size_t)n, c->stream));
    return TCI_OK;
}

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// mapped pinned host buffer (zero-copy results of the small path; the stream is idle whenever it
// is reallocated)
int ensure_mapped(tci_ctx* c, size_t bytes) {
    if (bytes <= c->capZ && c->zbuf) return TCI_OK;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    if (c->zbuf) {
        hipStreamSynchronize(c->stream);
        hipHostFree(c->zbuf);
        c->zbuf = c->zdev = nullptr;
        c->capZ = 0;
    }
    if (hipHostMalloc((void**)&c->zbuf, want, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->zdev, c->zbuf, 0) != hipSuccess) {
        c->zbuf = c->zdev = nullptr;
        return set_err(c, TCI_ERR_NOMEM, "mapped host allocation of " + std::to_string(want) +
                                             " bytes failed");
    }
    c->capZ = want;
    return TCI_OK;
}

// pinned host staging buffer (grown on demand; the stream is idle whenever it is reallocated)
int ensure_mapped_pair(tci_ctx* c, char** h, char** d, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *h) return TCI_OK;
    const size_t want = std::max<size_t>(bytes, 1 << 16);
    if (*h) {
        hipStreamSynchronize(c->stream);
        hipHostFree(*h);
        *h = *d = nullptr;
        *cap = 0;
    }
    if (hipHostMalloc((void**)h, want, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)d, *h, 0) != hipSuccess) {
        *h = *d = nullptr;
        return set_err(c, TCI_ERR_NOMEM, "mapped host allocation of " + std::to_string(want) +
                                             " bytes failed");
    }
    *cap = want;
    return TCI_OK;
}

int ensure_pinned(tci_ctx* c, char** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *p) return TCI_OK;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    if (*p) {
        hipStreamSynchronize(c->stream);
        hipHostFree(*p);
        *p = nullptr;
        *cap = 0;
    }
    if (hipHostMalloc((void**)p, want, 0) != hipSuccess) {
        *p = nullptr;
        return set_err(c, TCI_ERR_NOMEM, "pinned host allocation of " + std::to_string(want) +
                                             " bytes failed");
    }
    *cap = want;
    return TCI_OK;
}

// host memcpy over up to 8 threads (page faults of fresh destination pages and the copy itself
// spread over cores): large device -> pageable host results only
static void par_memcpy(char* dst, const char* src, size_t n) {
    const size_t per = 4u << 20;
    const int nt = (int)std::min<size_t>(8, n / per);
    if (nt <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t blk = ((n / nt) + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const size_t o = (size_t)t * blk;
        if (o < n) th.emplace_back([=] { memcpy(dst + o, src + o, std::min(blk, n - o)); });
    }
    memcpy(dst, src, std::min(blk, n));
    for (auto& x : th) x.join();
}

// n bytes of device memory into pageable host memory (then synchronised). Small copies go straight
// to hipMemcpyAsync; large ones (the site tensors and MatrixLUCI factors of config 5: up to 268 MB)
// in 32-MB chunks through two pinned slots -- chunk k + 1's DMA in flight while the host threads copy
// chunk k out -- instead of the runtime's pageable path (~20 GB/s with one host thread).
static int d2h_large(tci_ctx* c, void* dst, const void* src, size_t n) {
    constexpr size_t kCh = 32u << 20;
    if (n < 2 * kCh) {
        HIPCHK(c, hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        return TCI_OK;
    }
    int st;
    if ((st = ensure_pinned(c, &c->hd2h, &c->capHd2h, 2 * kCh))) return st;
    for (auto& e : c->d2h_ev)
        if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const size_t nch = (n + kCh - 1) / kCh;
    auto issue = [&](size_t k) -> int {
        const size_t len = std::min(kCh, n - k * kCh);
        HIPCHK(c, hipMemcpyAsync(c->hd2h + (k & 1) * kCh, static_cast<const char*>(src) + k * kCh, len,
                                 hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->d2h_ev[k & 1], c->stream));
        return TCI_OK;
    };
    if ((st = issue(0))) return st;
    for (size_t k = 0; k < nch; ++k) {
        if (k + 1 < nch && (st = issue(k + 1))) return st;  // slot (k + 1) & 1 was drained at step k - 1
        HIPCHK(c, hipEventSynchronize(c->d2h_ev[k & 1]));
        par_memcpy(static_cast<char*>(dst) + k * kCh, c->hd2h + (k & 1) * kCh, std::min(kCh, n - k * kCh));
    }
    return TCI_OK;
}

void ev_begin(tci_ctx* c, int fam, bool sampled = true, int sub = -1, int units = 1) {
    if (!c->timing || !sampled) return;
    if (c->evused + 2 > c->evpool.size()) {
        size_t add = std::max<size_t>(64, c->evpool.size());
        for (size_t i = 0; i < add; ++i) {
            hipEvent_t e;
            hipEventCreate(&e);
            c->evpool.push_back(e);
        }
    }
    c->evpairs.push_back({fam, sub, c->evused, units});
    hipEventRecord(c->evpool[c->evused], c->stream);
    c->evused += 2;
}
void ev_end(tci_ctx* c, bool sampled = true) {
    if (!c->timing || !sampled) return;
    hipEventRecord(c->evpool[c->evpairs.back().idx + 1], c->stream);
}
void ev_reset(tci_ctx* c) {
    c->evused = 0;
    c->evpairs.clear();
    for (int f = 0; f < tci_ctx::kFams; ++f) {
        c->fam_ms[f] = 0;
        c->fam_n[f] = 0;
        c->fam_u[f] = 0;
    }
}
void ev_collect(tci_ctx* c) {
    if (!c->timing) return;
    hipStreamSynchronize(c->stream);
    for (auto& pr : c->evpairs) {
        float ms = 0;
        hipEventElapsedTime(&ms, c->evpool[pr.idx], c->evpool[pr.idx + 1]);
        c->fam_ms[pr.fam] += ms;
        c->fam_n[pr.fam] += 1;
        c->fam_u[pr.fam] += pr.units;
        if (pr.sub >= 0) {
            c->fam_ms[pr.sub] += ms;
            c->fam_n[pr.sub] += 1;
            c->fam_u[pr.sub] += pr.units;
        }
    }
    c->evpairs.clear();
    c->evused = 0;
}

constexpr int kMaxGrid = tci::kMaxPassGrid;

// columns per rrLU tile (multiple of the kernel's 8-column batch): wide tiles when the matrix
// is large, narrower ones so that small matrices still spread over every CU
int pick_cb(int64_t m, int64_t n) {
    const int64_t tiles_r = (m + tci::kRowsPerTile - 1) / tci::kRowsPerTile;
    for (int cb = tci::kMaxCB; cb > 8; cb /= 2)
        if (tiles_r * ((n + cb - 1) / cb) >= kMaxGrid) return cb;
    return 8;
}

// The stop test of _optimizerrlu! (matrixlu.jl:359-368) runs on the device; passes launched after
// it fired return at once. The host learns of it without draining the stream: after each chunk
// of passes the state is copied into one of two pinned slots behind an event, and the host waits
// only for the previous chunk's copy while the current chunk keeps the GPU busy. A stop is seen
// at most one chunk late (<= kMaxChunk empty launches), and no chunk boundary leaves the GPU idle.
// Only the leading (np, done) words of the state are copied: RrluState and the ComplexF64 path's
// CState share that prefix.
static_assert(offsetof(RrluState, done) == 8 && offsetof(tci::CState, done) == 8, "state prefix");
struct StopPoll {
    static constexpr int64_t kMaxChunk = 32;
    static constexpr size_t kPrefix = 16;
    tci_ctx* c;
    const void* dstate;
    int cur = 0;
    bool pending = false;
    StopPoll(tci_ctx* ctx, const void* state) : c(ctx), dstate(state) {}
    // done (optional): the state's done word as copied (1: stop test, 2: a persistent launch gave up)
    int after_chunk(bool* stopped, int* done = nullptr) {
        HIPCHK(c, hipMemcpyAsync(&c->hpoll[cur], dstate, kPrefix, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipEventRecord(c->pollev[cur], c->stream));
        if (pending) {
            HIPCHK(c, hipEventSynchronize(c->pollev[cur ^ 1]));
            *stopped = c->hpoll[cur ^ 1].done != 0;
            if (done) *done = c->hpoll[cur ^ 1].done;
        }
        pending = true;
        cur ^= 1;
        return TCI_OK;
    }
};

// The per-pivot loop of _optimizerrlu! (matrixlu.jl:346-369) on a device matrix (clobbered:
// its trailing values are left stale). Leaves on the device: rowphys/colphys (= rowpermutation /
// colpermutation, 0-based) in c->rowperm / c->colperm, pivot values in c->pivv, L columns in
// physical row order in c->Lp (ld m) and U rows in physical column order in c->Up (ld mr).
// Shadow epochs per fp64 write-back (two-level epoch). A later shadow epoch's read
// passes pay the EXT prologue (exact pending chains up to nb * epochs - 1 long, ~5-10 us each), and
// a refresh replaces a write-back (18 B/element) by the MFMA search's shadow store (4 B/element): the
// trade pays where a write-back streams long, i.e. on large trailing blocks. Measured on MI355X
// (profiles/r04_ab_epochs_shapes.jsonl, r = 256): 2048^2 / 4096^2 fastest at 1, 8192^2 / 16384^2 at
// 3; the break-even (2 write-backs' 14 B/element saved ~ 20 EXT prologues) is near 2.4e7 elements.
// Round 6, 8-bit shadow (refresh 1 + 1 B/element, read-only passes 1 B): the EXT passes' extra start-up
// now weighs more against the write-backs they save, so the middle sizes prefer two shadow epochs
// (profiles/r06_d2_sched_*.jsonl, r06_e2_sched_*.jsonl: 4096^2 fastest at 1 (6.40 vs 6.66 ms), 8192^2
// at 2 (12.05 vs 12.32), 16384^2 2 ~ 3 (36.69 / 36.64), 32768^2 r = 1024 at 3 (508.7 vs 555.9)).
int rrlu_epochs(const tci_ctx* c, int64_t m, int64_t n) {
    if (c->epochs > 0) return c->epochs;
    const double mn = (double)m * (double)n;
    return mn >= 2.0e8 ? 3 : mn >= 2.4e7 ? 2 : 1;
}

// dsrc (optional): the input, ld ldsrc; dA is then the work matrix it is copied into (rrlu's copy,
// matrixlu.jl:462) -- by the pass pipeline's initial argmax pass as it reads (one read of the input,
// not a copy kernel and then the pass), by an explicit copy ahead of the one-launch paths
int rrlu_device(tci_ctx* c, double* dA, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
                double reltol, double abstol, int leftorth, int64_t* np_out, double* err_out,
                const double* dsrc = nullptr, int64_t ldsrc = 0) {
    int st;
    c->sh_valid = 0;  // the shared rrLU buffers are about to be overwritten
    auto copy_input = [&]() -> int {
        if (dsrc && m > 0 && n > 0)
            HIPCHK(c, hipMemcpy2DAsync(dA, lda * sizeof(double), dsrc, ldsrc * sizeof(double), m * sizeof(double),
                                       n, hipMemcpyDeviceToDevice, c->stream));
        dsrc = nullptr;
        return TCI_OK;
    };
    if ((st = ensure(c, &c->rowperm, &c->capPerm, (size_t)m + 1))) return st;
    if ((st = ensure(c, &c->colperm, &c->capColperm, (size_t)n + 1))) return st;
    if ((st = ensure(c, &c->rowpos, &c->capRowpos, (size_t)m + 1))) return st;
    if ((st = ensure(c, &c->colpos, &c->capColpos, (size_t)n + 1))) return st;
    if ((st = ensure(c, &c->cand, &c->capCand, (size_t)kMaxGrid + 8))) return st;  // + the XCD-class candidates
    const int mi = (int)m, ni = (int)n;
    tci::launch_init_state(c->stream, c->st, c->rowpos, c->rowperm, mi, c->colpos, c->colperm, ni);
    int64_t mr = std::min<int64_t>(maxrank, std::min<int64_t>(m, n));
    if (mr < 0) mr = 0;
    c->ldUp = std::max<int64_t>(mr, 1);
    if (m == 0 || n == 0 || mr == 0) {
        if ((st = copy_input())) return st;
        HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        *np_out = 0;
        *err_out = (0 >= std::min(m, n)) ? 0.0 : c->hst->error;
        return TCI_OK;
    }
    if ((st = ensure(c, &c->pivv, &c->capPivv, (size_t)mr + 1))) return st;
    if ((st = ensure(c, &c->Lp, &c->capLp, (size_t)(m * mr)))) return st;
    if ((st = ensure(c, &c->Up, &c->capUp, (size_t)(mr * n)))) return st;
    // the fused copy reads the input as 16-B row pairs (k_pass2's load_chunk): an odd ldsrc or a
    // source not 16-byte aligned would give misaligned loads (and, with an odd m and ldsrc == m, a
    // read 8 B past the last column), so such an input is copied first
    if (dsrc && ((ldsrc & 1) || ((uintptr_t)dsrc & 15)))
        if ((st = copy_input())) return st;
    if (dsrc && ((c->small_path && tci::rrlu_small_fits(m, n)) ||
                 (c->mid_path && !c->mid_faulted && c->ncu > 0 && tci::rrlu_mid_fits(m, n, c->ncu))))
        if ((st = copy_input())) return st;
    if (c->small_path && tci::rrlu_small_fits(m, n)) {
        // the whole factorisation in one workgroup's LDS: one launch instead of one per pivot
        HIPCHK(c, tci::launch_rrlu_small(c->stream, dA, lda, mi, ni, (int)mr, reltol, abstol,
                                         leftorth, c->st, c->rowperm, c->colperm, c->pivv, c->Lp, m,
                                         c->Up, c->ldUp, tci::SmallOut{nullptr, nullptr, nullptr}));
        HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        *np_out = c->hst->np;
        *err_out = (c->hst->np >= std::min(m, n)) ? 0.0 : c->hst->error;  // matrixlu.jl:391-393
        return TCI_OK;
    }
    if (c->mid_path && !c->mid_faulted && c->ncu > 0 && tci::rrlu_mid_fits(m, n, c->ncu)) {
        // the matrix resident in the LDS of a persistent grid: one launch, one barrier per pivot
        const int64_t G = std::min<int64_t>(std::min(c->ncu, 256), n);
        if ((st = ensure(c, &c->colbuf, &c->capColbuf, (size_t)(G * m)))) return st;
        HIPCHK(c, tci::launch_rrlu_mid(c->stream, c->ncu, dA, lda, mi, ni, (int)mr, reltol, abstol,
                                       leftorth, c->st, c->rowperm, c->colperm, c->pivv, c->Lp, m, c->Up,
                                       c->ldUp, c->cand, c->colbuf, c->bar, c->fault));
        HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->hflag, c->fault, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (!*c->hflag) {
            *np_out = c->hst->np;
            *err_out = (c->hst->np >= std::min(m, n)) ? 0.0 : c->hst->error;
            return TCI_OK;
        }
        // the grid barrier timed out (workgroups not co-resident): the input is untouched, so the
        // pass pipeline below recomputes the same factorisation; this context stops trying the
        // persistent grid (the device is evidently shared), so the timeout is paid once
        c->mid_faulted = 1;
    }
    // pending rank-1 updates, slot-major: X[s * ldx + i] (slot s, physical row i), Y[s * ldy + j];
    // ldx >= m + 2 so the 16-B loads of a tile's last odd row stay in bounds
    const int nb = std::max(1, std::min(c->flush_every, tci::kMaxPend));
    const int64_t ldx = round_up(m + 2, 16), ldy = round_up(n + 2, 16);
    if ((st = ensure(c, &c->xbuf, &c->capX, (size_t)(tci::kMaxPendR * ldx)))) return st;
    if ((st = ensure(c, &c->ybuf, &c->capY, (size_t)(tci::kMaxPendR * ldy)))) return st;
    if ((m + tci::kRowsPerTile - 1) / tci::kRowsPerTile > kMaxGrid)
        return set_err(c, TCI_ERR_ARG, "rrlu: more than " +
                                           std::to_string((long long)tci::kRowsPerTile * kMaxGrid) +
                                           " rows is not supported");
    tci::PassArgs g;
    g.A = dA;
    g.lda = lda;
    g.m = mi;
    g.n = ni;
    g.k = -1;
    g.X = c->xbuf;
    g.ldx = ldx;
    g.Y = c->ybuf;
    g.ldy = ldy;
    g.rowpos = c->rowpos;
    g.colpos = c->colpos;
    g.st = c->st;
    g.Lp = c->Lp;
    g.ldl = m;
    g.Up = c->Up;
    g.ldu = c->ldUp;
    g.leftorth = leftorth;
    g.cand = c->cand;
    g.cb = pick_cb(m, n);
    if (const char* e = getenv("TCI_RRLU_CB")) g.cb = std::max(8, std::min(atoi(e) / 8 * 8, tci::kMaxCB));
    g.rev = 0;
    g.rowphys = c->rowperm;
    g.colphys = c->colperm;
    g.pivvals = c->pivv;
    g.reltol = reltol;
    g.abstol = abstol;
    g.ticket = c->ticket;
    g.selk = 0;
    // fp32 shadow for the certified search (4-row lanes need lda, lds multiples of 4)
    const bool shadow = c->shadow && lda % 4 == 0;
    g.S = nullptr;
    g.lds = 0;
    if (shadow) {
        g.lds = round_up(m, 16);
        if ((st = ensure(c, &c->sbuf, &c->capS, (size_t)(g.lds * n)))) return st;
        g.S = c->sbuf;
        if ((st = zero_shadow_pad(c, g.lds, m, n))) return st;
    }
    const int grid = tci::argmax_grid(mi, ni, -1, g.cb,
                                      std::min(std::max(std::max(c->ncu, 1) * c->pass_gridx / c->pass_griddiv, 8), kMaxGrid));
    // two-level epoch: shadow epochs of nb pivots end with a refresh of the fp16
    // shadow by the MFMA search itself, and only every `epochs`-th of them with a write-back of the
    // fp64 values (exact pending updates up to nb * epochs <= kMaxPendR). epochs = 1: every shadow
    // epoch ends with a write-back (round 2's scheme); the exact passes (shadow off) always do.
    // (the refresh is the MFMA search's: shadow epochs of 2 .. 15 pivots -- pass 0 writes the
    // shadow of A and cannot refresh, and the search has at most two K-steps)
    // (the refresh stores address the whole shadow through one 32-bit buffer offset: <= 4 GB)
    const int epochs = (shadow && tci::shadow_two_level() && nb >= 2 && nb <= 15 &&
                        tci::refresh_fits(g.lds, n))
                           ? std::max(1, std::min(rrlu_epochs(c, m, n), tci::kMaxPendR / nb)) : 1;
    const int nbx = nb * epochs;
    g.nbs = nb;
    g.pe = g.ps = 0;
    g.Asrc = dsrc;  // (the initial pass copies the input into A as it reads it)
    g.ldsrc = ldsrc;
    tci::launch_pass(c->stream, 0, false, shadow, g, grid);  // argmax of A, selects pivot 0
    g.Asrc = nullptr;
    // The pass schedule: pass kk applies PE exact / PS shadow pending updates and is a
    // write-back (flush), a refresh, or read-only; te / ts: the first pivot whose update is pending in
    // fp64 / in the shadow. A deterministic function of kk, so a resume can replay it.
    struct Sched {
        int PE, PS;
        bool last, flush, refresh;
    };
    auto sched = [&](int64_t kk, int64_t te, int64_t ts) {
        Sched s;
        s.PE = (int)(kk - te) + 1;
        s.PS = (int)(kk - ts) + 1;
        s.last = kk + 1 >= mr;
        s.flush = s.PE >= nbx && !s.last;
        s.refresh = !s.flush && epochs > 1 && s.PS >= nb && !s.last;
        return s;
    };
    // Persistent epoch launches (tci_rrlu.hip k_pass_mf_epoch): a run of >= 2 read-only MFMA-search
    // passes in one launch, when the grid is one workgroup per CU (all co-resident on an idle device)
    // (persist == 2, a test mode: also when the grid exceeds one workgroup per CU -- it is then NOT
    // co-resident and the launch must give up, after 2 ms instead of 0.5 s, and resume)
    bool persist = c->persist && !c->persist_faulted && shadow && tci::shadow_two_level() && c->ncu > 0 &&
                   ((grid <= c->ncu && c->pass_gridx == 1) || c->persist == 2) && tci::epoch_fits(mi, ni, g.cb, grid) &&
                   2 * grid <= kMaxGrid && grid <= 1024;  // candidates double-buffered by pass parity, reduced by 1024 threads
    const long long ptimeout = c->persist == 2 ? 200000 : 50000000;  // 100 MHz ticks
    int64_t nlaunch = 0;  // persistent launches issued (their sync slots)
    if (persist) {
        const size_t slots = (size_t)mr / 2 + 2;
        if ((st = ensure(c, &c->esync, &c->capEsync, slots * tci::kEpochSlot))) return st;
        HIPCHK(c, hipMemsetAsync(c->esync, 0, slots * tci::kEpochSlot * sizeof(unsigned), c->stream));
    }
    int64_t k = 0, chunk = 2, te = 0, ts = 0;
    StopPoll poll(c, c->st);
    for (;;) {  // once, or again from a resume point after a persistent launch gave up
        while (k < mr) {
            const int64_t kend = std::min<int64_t>(k + chunk, mr);
            int64_t kk = k;
            while (kk < kend) {
                // pass kk: derives x_k / y_k (L column / U row k), applies pending updates 0..P-1 and
                // selects pivot k+1 from the updated block. After the last pivot only x_k / y_k are
                // needed: no selection.
                const Sched s = sched(kk, te, ts);
                const bool ro = !s.flush && !s.refresh && !s.last;
                if (persist && ro && kk >= 1 && s.PS <= tci::kEpochMaxP && (c->persist_kinds & (s.PE > s.PS ? 2 : 1))) {
                    int np = 1;  // the run of read-only passes that follows (te, ts do not move in it)
                    for (; np < c->persist_maxpass; ++np) {
                        const Sched t = sched(kk + np, te, ts);
                        if (t.flush || t.refresh || t.last || t.PS > tci::kEpochMaxP) break;
                    }
                    if (np >= 2) {
                        g.k = (int)kk;
                        g.pe = s.PE;
                        g.ps = s.PS;
                        g.selk = (int)(kk + 1);
                        const bool sampled = nlaunch % 3 == 0;
                        ev_begin(c, s.PE > s.PS ? tci_ctx::kFamEpoch + 1 : tci_ctx::kFamEpoch, sampled, -1, np);
                        tci::launch_pass_epoch(c->stream, g, grid, np, c->serpentine,
                                               c->esync + (size_t)nlaunch * tci::kEpochSlot, ptimeout);
                        ev_end(c, sampled);
                        ++nlaunch;
                        kk += np;
                        continue;
                    }
                }
                g.k = (int)kk;
                g.pe = s.PE;
                g.ps = s.PS;
                g.selk = !s.last ? (int)(kk + 1) : -1;
                g.rev = c->serpentine ? (int)((kk + 1) & 1) : 0;
                const bool sampled = kk % c->timing_stride == 0;
                // pass 0 (shadow on: the exact pass that writes the shadow of A) is a family of its own
                const bool pass0 = kk == 0 && shadow && tci::shadow_elem_bytes() <= 2 && !s.flush;
                ev_begin(c, s.flush ? 0 : s.refresh ? 23 : pass0 ? tci_ctx::kFamPass0 : 2, sampled,
                         s.flush || s.refresh || pass0 ? -1 : (s.PE > s.PS ? 24 : 3) + s.PS);
                tci::launch_pass(c->stream, s.PE, s.flush, shadow, g, grid, s.flush ? 1 : s.refresh ? 2 : 0);
                ev_end(c, sampled);
                if (s.flush) te = ts = kk + 1;
                if (s.refresh) ts = kk + 1;
                ++kk;
            }
            k = kk;
            if (k >= mr) break;
            bool stopped = false;
            if ((st = poll.after_chunk(&stopped))) return st;
            if (stopped) break;
            chunk = std::min<int64_t>(chunk * 2, StopPoll::kMaxChunk);
        }
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (c->hst->done != 2 && c->hst->done != 3) break;
        // A persistent launch ended early: 2 -- it gave up waiting for its grid (another process
        // holds CUs); 3 -- a pass's shadow certificate failed (a rapidly decaying block: the exact
        // bodies are per-pass kernels). Nothing was committed for that pass, every launch after it
        // returned at once, and every pass write is idempotent: resume with per-pass launches at the
        // pass after the last commit (for the rest of this factorisation; after 2 for the context)
        if (c->hst->done == 2) c->persist_faulted = 1;
        persist = false;
        k = c->hst->np - 1;
        te = ts = 0;
        for (int64_t q = 0; q < k; ++q) {  // replay the schedule up to pass k
            const Sched s = sched(q, te, ts);
            if (s.flush) te = ts = q + 1;
            if (s.refresh) ts = q + 1;
        }
        HIPCHK(c, hipMemsetAsync(&c->st->done, 0, sizeof(int32_t), c->stream));
        chunk = 2;
        poll = StopPoll(c, c->st);
    }
    int64_t np = c->hst->np;
    double err = c->hst->error;
    if (np >= std::min(m, n)) err = 0.0;  // matrixlu.jl:391-393
    *np_out = np;
    *err_out = err;
    return TCI_OK;
}

// Position-order L (m x np, ld m) into c->dL and U (np x n, ld np) into c->dU (either skipped when
// want_* is false) with the NaN checks of matrixlu.jl:376-381.
int extract_LU(tci_ctx* c, int64_t m, int64_t n, int64_t np, int leftorth, bool wantL, bool wantU) {
    if (np <= 0) return TCI_OK;
    int st;
    if (wantL && (st = ensure(c, &c->dL, &c->capL, (size_t)(m * np)))) return st;
    if (wantU && (st = ensure(c, &c->dU, &c->capU, (size_t)(np * n)))) return st;
    HIPCHK(c, hipMemsetAsync(c->flag, 0, sizeof(int), c->stream));
    tci::launch_extract(c->stream, c->Lp, m, c->Up, c->ldUp, c->pivv, c->rowperm, c->colperm, (int)m,
                        (int)n, (int)np, leftorth, wantL ? c->dL : nullptr, m, wantU ? c->dU : nullptr,
                        np, c->flag);
    HIPCHK(c, hipMemcpyAsync(c->hflag, c->flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (*c->hflag & 1) return set_err(c, TCI_ERR_NAN, "lu.L contains NaNs");
    if (*c->hflag & 2) return set_err(c, TCI_ERR_NAN, "lu.U contains NaNs");
    return TCI_OK;
}

int fetch_perms(tci_ctx* c, int64_t* rowperm, int64_t* colperm, int64_t nrow, int64_t ncol) {
    if (rowperm && nrow > 0)
        HIPCHK(c, hipMemcpyAsync(rowperm, c->rowperm, nrow * sizeof(int64_t), hipMemcpyDeviceToHost,
                                 c->stream));
    if (colperm && ncol > 0)
        HIPCHK(c, hipMemcpyAsync(colperm, c->colperm, ncol * sizeof(int64_t), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (rowperm)
        for (int64_t i = 0; i < nrow; ++i) rowperm[i] += 1;
    if (colperm)
        for (int64_t j = 0; j < ncol; ++j) colperm[j] += 1;
    return TCI_OK;
}

// pivoterrors (matrixlu.jl:799): |pivot values| then lu.error
int pivot_errors(tci_ctx* c, int64_t np, double err, double* out) {
    if (!out) return TCI_OK;
    if (np > 0) {
        HIPCHK(c, hipMemcpyAsync(out, c->pivv, np * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (int64_t t = 0; t < np; ++t) out[t] = std::fabs(out[t]);
    }
    out[np] = err;
    return TCI_OK;
}

int upload_matrix(tci_ctx* c, const double* A, int64_t m, int64_t n, int64_t lda, int64_t* ld_d) {
    const int64_t ld = round_up(std::max<int64_t>(m, 1), 16);
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(ld * std::max<int64_t>(n, 1))))) return st;
    if (m > 0 && n > 0)
        HIPCHK(c, hipMemcpy2DAsync(c->dA, ld * sizeof(double), A, lda * sizeof(double),
                                   m * sizeof(double), n, hipMemcpyHostToDevice, c->stream));
    *ld_d = ld;
    return TCI_OK;
}

int upload_index(tci_ctx* c, int32_t** d, size_t* cap, const int32_t* h, int64_t count, int32_t w) {
    int st;
    size_t nel = (size_t)std::max<int64_t>(count * w, 1);
    if ((st = ensure(c, d, cap, nel))) return st;
    if (count * w > 0)
        HIPCHK(c, hipMemcpyAsync(*d, h, count * w * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    return TCI_OK;
}

// TCI_F_HOST: the batch is evaluated by the user's callback on this host thread into a pinned
// buffer (the index tables come back from the device first: every caller has uploaded them), then
// uploaded once and its max|.| taken on the device, as for the kernels' fused maxabs. The stream is
// idle while the callback runs, so the pinned buffer is never overwritten under a pending copy.
int host_batcheval(tci_ctx* c, const tci_func* f, const int32_t* dI, int64_t m, int32_t nl,
                   const int32_t* dJ, int64_t n, int32_t nr, int32_t M, int64_t D, double* dout,
                   int64_t ldo) {
    if (m <= 0 || n <= 0) return TCI_OK;
    std::vector<int32_t> hI((size_t)std::max<int64_t>(m * nl, 1)), hJ((size_t)std::max<int64_t>(n * nr, 1));
    if (m * nl > 0)
        HIPCHK(c, hipMemcpyAsync(hI.data(), dI, m * nl * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (n * nr > 0)
        HIPCHK(c, hipMemcpyAsync(hJ.data(), dJ, n * nr * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t mR = m * D;
    int st;
    if ((st = ensure_pinned(c, &c->hfn, &c->capHfn, (size_t)(mR * n) * sizeof(double)))) return st;
    double* hb = reinterpret_cast<double*>(c->hfn);
    if (f->hostfn(f->hostuser, hI.data(), m, nl, hJ.data(), n, nr, M, hb, mR) != 0)
        return set_err(c, TCI_ERR_HOST, "host function evaluation failed");
    ev_begin(c, 1);
    HIPCHK(c, hipMemcpy2DAsync(dout, ldo * sizeof(double), hb, mR * sizeof(double), mR * sizeof(double), n,
                               hipMemcpyHostToDevice, c->stream));
    tci::launch_cache_maxabs(c->stream, dout, mR, n, ldo, c->maxbits);
    ev_end(c);
    HIPCHK(c, hipGetLastError());
    return TCI_OK;
}

// batch evaluation into a device buffer (column-major, ld ldo). *maxabs = max|out|.
// batch evaluation launches only (no synchronisation); c->maxbits receives max|out| bits
// maxbits: where the batch's max |value| bits are folded (atomic max); null = the context's word,
// zeroed first (a running maximum passed in is not)
int batcheval_launch(tci_ctx* c, const tci_func* f, const int32_t* dI, int64_t m, int32_t nl,
                     const int32_t* dJ, int64_t n, int32_t nr, int32_t M, double* dout, int64_t ldo,
                     unsigned long long* maxbits = nullptr) {
    if (nl + M + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    if (M < 0 || M > 1) return set_err(c, TCI_ERR_ARG, "only M = 0 or M = 1 centre legs are supported");
    const int D = M ? f->localdims[nl] : 1;
    if (ldo < m * D) return set_err(c, TCI_ERR_ARG, "ldo < m * prod(centre dims)");
    if (maxbits && f->kind == TCI_F_HOST)
        return set_err(c, TCI_ERR_ARG, "a host integrand (TCI_F_HOST) needs tci_batcheval_d");
    if (!maxbits) {
        maxbits = c->maxbits;
        HIPCHK(c, hipMemsetAsync(c->maxbits, 0, sizeof(unsigned long long), c->stream));
    }
    if (f->kind == TCI_F_C128)
        return set_err(c, TCI_ERR_ARG, "a ComplexF64 integrand needs the ComplexF64 entries (*_c128_*)");
    if (f->kind == TCI_F_HOST) return host_batcheval(c, f, dI, m, nl, dJ, n, nr, M, D, dout, ldo);
    if (m > 0 && n > 0) {
        FuncDev fv = f->view();
        int st;
        int64_t sb = tci::batcheval_scratch_bytes(fv, (int)m, D, (int)n);
        if (sb > 0 && (st = ensure(c, (char**)&c->scratch, &c->capScratch, (size_t)sb))) return st;
        ev_begin(c, 1);
        tci::launch_batcheval(c->stream, fv, dI, (int)m, nl, dJ, (int)n, nr, M, D, dout, ldo,
                              maxbits, c->scratch);
        ev_end(c);
        HIPCHK(c, hipGetLastError());
    }
    return TCI_OK;
}

int batcheval_device(tci_ctx* c, const tci_func* f, const int32_t* dI, int64_t m, int32_t nl,
                     const int32_t* dJ, int64_t n, int32_t nr, int32_t M, double* dout, int64_t ldo,
                     double* maxabs) {
    int st;
    if ((st = batcheval_launch(c, f, dI, m, nl, dJ, n, nr, M, dout, ldo))) return st;
    HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (maxabs) {
        double v;
        unsigned long long b = *c->hmaxbits;
        memcpy(&v, &b, sizeof v);
        *maxabs = v;
    }
    return TCI_OK;
}


// ------------------------------------------------------------------ column-sharded rrLU driver
// The loop of rrlu_device with the selection split across ranks: the passes run unchanged on
// this rank's columns (+ the ghost column) and publish the local winner; then the candidates are
// exchanged, the rank owning the winning column contributes it, and every rank commits the same
// pivot (tci_internal.h, column-sharded rrLU) -- all stream-ordered: the host only polls the stop
// flag in growing chunks, as rrlu_device does. Exchange op 0: all-gather of `words` uint64 per rank
// (rank-major); op 1: element-wise max of `words` uint64 over the ranks.
int shard_exchange(tci_ctx* c, tci_comm* comm, tci_exchange_fn exch, void* user, int op, const void* send,
                   void* recv, int64_t words) {
    if (comm) {
        const ncclResult_t r =
            op == 0 ? ncclAllGather(send, recv, (size_t)words, ncclUint64, comm->nc, c->stream)
                    : ncclAllReduce(send, recv, (size_t)words, ncclUint64, ncclMax, comm->nc, c->stream);
        if (r != ncclSuccess)
            return set_err(c, TCI_ERR_DEVICE, std::string("rrlu_sharded: ") + (op ? "ncclAllReduce" : "ncclAllGather") +
                                                  " failed: " + ncclGetErrorString(r));
        return TCI_OK;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (exch(user, op, send, recv, words) != 0)
        return set_err(c, TCI_ERR_DEVICE, "rrlu_sharded: exchange callback failed");
    return TCI_OK;
}

int rrlu_sharded_device(tci_ctx* c, tci_comm* comm, tci_exchange_fn exch, void* user, int nranks,
                        double* dA, int64_t m, int64_t nloc, int64_t lda, int64_t c0, int64_t n,
                        int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* np_out,
                        double* err_out) {
    int st;
    c->sh_valid = 0;
    if ((st = ensure(c, &c->rowperm, &c->capPerm, (size_t)m + 1))) return st;
    if ((st = ensure(c, &c->colperm, &c->capColperm, (size_t)n + 1))) return st;
    if ((st = ensure(c, &c->rowpos, &c->capRowpos, (size_t)m + 1))) return st;
    if ((st = ensure(c, &c->colpos, &c->capColpos, (size_t)n + 1))) return st;
    if ((st = ensure(c, &c->colposL, &c->capColposL, (size_t)nloc + 2))) return st;
    if ((st = ensure(c, &c->cand, &c->capCand, (size_t)kMaxGrid + 8))) return st;  // + the XCD-class candidates
    // one rank without a communicator: nothing to exchange -- the pass tail commits as in
    // rrlu_device (no candidate record, no ghost column: the pivot column is this rank's own). With a
    // communicator (even of one rank) every pivot goes through the exchange.
    const bool multi = nranks > 1 || comm || exch;
    if (nranks < 1 || (nranks > 1 && !comm && !exch))
        return set_err(c, TCI_ERR_ARG, "rrlu_sharded: more than one rank needs a comm or exchange");
    if (!multi && (c0 != 0 || nloc != n))
        return set_err(c, TCI_ERR_ARG, "rrlu_sharded: a single rank must hold every column");
    if ((st = ensure(c, &c->lout, &c->capLout, (size_t)nranks + 1))) return st;  // [own, all-gathered ...]
    const int64_t cw = tci::shard_col(m);
    // the per-pivot exchange: fused = ONE all-gather of [record | own candidate
    // column] (N x (m + kMaxPendR + 4) words received per rank), two-collective = a 32-B-per-rank
    // all-gather of the records, then an element-wise max of the winner's column (m + kMaxPendR
    // words) as a broadcast from a root no rank knows in advance. By size: fused while the extra
    // bytes it moves stay under kFusedMax (they cost less than the second collective's latency)
    const int64_t fw = tci::kCandWords + cw;
    constexpr int64_t kFusedMax = 4 << 20;
    const bool fused = multi && (c->sh_exchange == 2 || (c->sh_exchange == 0 && (int64_t)(nranks - 1) * fw * 8 <= kFusedMax));
    c->sh_exchange_used = multi ? (fused ? 2 : 1) : 0;
    if (multi) {
        if ((st = ensure(c, &c->shsend, &c->capShSend, (size_t)std::max<int64_t>(fused ? fw : cw, 2)))) return st;
        if ((st = ensure(c, &c->shrecv, &c->capShRecv, (size_t)std::max<int64_t>(fused ? fw * nranks : cw, 2)))) return st;
    }
    // every rank must run the same exchange form (a fused all-gather on one rank against two
    // collectives on another would hang RCCL): the choice follows each rank's own setting
    // (tci_set_shard_exchange / TCI_SHARD_EXCHANGE), so the ranks check that they agree once per
    // factorisation -- one element-wise max of [fused, !fused]: both 1 means they differ, and
    // every rank sees it in the same reduction and fails together
    if (multi && nranks > 1) {
        const uint64_t mine[2] = {fused ? 1u : 0u, fused ? 0u : 1u};
        uint64_t got[2] = {0, 0};
        HIPCHK(c, hipMemcpyAsync(c->shsend, mine, sizeof(mine), hipMemcpyHostToDevice, c->stream));
        if ((st = shard_exchange(c, comm, exch, user, 1, c->shsend, c->shrecv, 2))) return st;
        HIPCHK(c, hipMemcpyAsync(got, c->shrecv, sizeof(got), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (got[0] && got[1])
            return set_err(c, TCI_ERR_ARG, "rrlu_sharded: the ranks chose different exchange forms "
                                           "(tci_set_shard_exchange / TCI_SHARD_EXCHANGE must be uniform)");
    }
    const int mi = (int)m, nl1 = (int)(nloc + 1);  // local columns + the ghost
    tci::launch_init_state(c->stream, c->st, c->rowpos, c->rowperm, mi, c->colpos, c->colperm, (int)n);
    tci::launch_shard_init(c->stream, c->colposL, (int)nloc, c0);
    int64_t mr = std::min<int64_t>(maxrank, std::min<int64_t>(m, n));
    if (mr < 0) mr = 0;
    c->ldUp = std::max<int64_t>(mr, 1);
    if (m == 0 || n == 0 || mr == 0) {
        HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        *np_out = 0;
        *err_out = (0 >= std::min(m, n)) ? 0.0 : c->hst->error;
        return TCI_OK;
    }
    if ((st = ensure(c, &c->pivv, &c->capPivv, (size_t)mr + 1))) return st;
    if ((st = ensure(c, &c->Lp, &c->capLp, (size_t)(m * mr)))) return st;
    if ((st = ensure(c, &c->Up, &c->capUp, (size_t)(mr * nl1)))) return st;
    const int nb = std::max(1, std::min(c->flush_every, tci::kMaxPend));
    const int64_t ldx = round_up(m + 2, 16), ldy = round_up(nl1 + 2, 16);
    if ((st = ensure(c, &c->xbuf, &c->capX, (size_t)(tci::kMaxPendR * ldx)))) return st;
    if ((st = ensure(c, &c->ybuf, &c->capY, (size_t)(tci::kMaxPendR * ldy)))) return st;
    if ((m + tci::kRowsPerTile - 1) / tci::kRowsPerTile > kMaxGrid)
        return set_err(c, TCI_ERR_ARG, "rrlu: too many rows");
    tci::PassArgs g;
    g.A = dA;
    g.lda = lda;
    g.m = mi;
    g.n = nl1;
    g.k = -1;
    g.X = c->xbuf;
    g.ldx = ldx;
    g.Y = c->ybuf;
    g.ldy = ldy;
    g.rowpos = c->rowpos;
    g.colpos = c->colposL;
    g.st = c->st;
    g.Lp = c->Lp;
    g.ldl = m;
    g.Up = c->Up;
    g.ldu = c->ldUp;
    g.leftorth = leftorth;
    g.cand = c->cand;
    g.cb = pick_cb(m, nl1);
    g.rev = 0;
    g.rowphys = c->rowperm;
    g.colphys = c->colperm;
    g.pivvals = c->pivv;
    g.reltol = reltol;
    g.abstol = abstol;
    g.ticket = c->ticket;
    g.selk = 0;
    g.lout = multi ? c->lout : nullptr;
    g.pc_off = c0;
    const bool shadow = c->shadow && lda % 4 == 0;
    g.S = nullptr;
    g.lds = 0;
    if (shadow) {
        g.lds = round_up(m, 16);
        if ((st = ensure(c, &c->sbuf, &c->capS, (size_t)(g.lds * nl1)))) return st;
        g.S = c->sbuf;
        if ((st = zero_shadow_pad(c, g.lds, m, nl1))) return st;
    }
    const int grid = tci::argmax_grid(mi, nl1, -1, g.cb, std::min(std::max(std::max(c->ncu, 1) * c->pass_gridx / c->pass_griddiv, 8), kMaxGrid));
    // candidates: own record at lout[0], the all-gathered ones at lout[1..nranks]
    tci::Cand* recvC = multi ? c->lout + 1 : c->lout;
    uint64_t* colsend = reinterpret_cast<uint64_t*>(c->shsend);
    uint64_t* colrecv = multi ? reinterpret_cast<uint64_t*>(c->shrecv) : nullptr;
    auto select = [&](int selk) -> int {
        if (!multi) return TCI_OK;  // committed by the pass tail
        if (fused) {
            tci::launch_shard_pack(c->stream, c->lout, dA, lda, mi, c->ybuf, ldy, c0, (int)nloc, colsend);
            if (int e = shard_exchange(c, comm, exch, user, 0, colsend, colrecv, fw)) return e;
            tci::launch_shard_commit(c->stream, colrecv, fw, nranks, nullptr, 1, mi, selk, c->st, reltol, abstol,
                                     c->rowpos, c->colpos, c->rowperm, c->colperm, c->pivv, c->colposL, c0,
                                     (int)nloc, dA, lda, c->ybuf, ldy);
            return TCI_OK;
        }
        {
            int e = shard_exchange(c, comm, exch, user, 0, c->lout, recvC, tci::kCandWords);
            if (e) return e;
            tci::launch_shard_pick(c->stream, recvC, nranks, dA, lda, mi, c->ybuf, ldy, c0, (int)nloc, colsend);
            if ((e = shard_exchange(c, comm, exch, user, 1, colsend, colrecv, cw))) return e;
        }
        tci::launch_shard_commit(c->stream, reinterpret_cast<const uint64_t*>(recvC), tci::kCandWords, nranks,
                                 colrecv, 0, mi, selk, c->st, reltol, abstol, c->rowpos, c->colpos, c->rowperm,
                                 c->colperm, c->pivv, c->colposL, c0, (int)nloc, dA, lda, c->ybuf, ldy);
        return TCI_OK;
    };
    // the two-level epoch of rrlu_device, decided by the GLOBAL shape so that every
    // rank runs the same schedule (the ghost column carries all kMaxPendR pending y's of the pivot)
    // (the refresh stores' 32-bit buffer offsets: every rank's shadow <= 4 GB, or no rank refreshes.
    // The test uses the global width n + 1, which bounds every rank's nloc + 1 whatever the split:
    // all ranks reach the same decision without an exchange, and an unbalanced column block cannot
    // exceed it -- ADVICE r4)
    const int epochs = (shadow && tci::shadow_two_level() && nb >= 2 && nb <= 15 &&
                        tci::refresh_fits(round_up(m, 16), n + 1))
                           ? std::max(1, std::min(rrlu_epochs(c, m, n), tci::kMaxPendR / nb)) : 1;
    const int nbx = nb * epochs;
    g.nbs = nb;
    g.pe = g.ps = 0;
    tci::launch_pass(c->stream, 0, false, shadow, g, grid);  // local argmax of A
    if ((st = select(0))) return st;
    int64_t k = 0, chunk = 2, te = 0, ts = 0;  // first pivot pending in fp64 / in the shadow
    StopPoll poll(c, c->st);
    while (k < mr) {
        const int64_t kend = std::min<int64_t>(k + chunk, mr);
        for (int64_t kk = k; kk < kend; ++kk) {
            const int PE = (int)(kk - te) + 1, PS = (int)(kk - ts) + 1;
            const bool last = kk + 1 >= mr;
            const bool flush = PE >= nbx && !last;
            const bool refresh = !flush && epochs > 1 && PS >= nb && !last;
            g.k = (int)kk;
            g.pe = PE;
            g.ps = PS;
            g.selk = !last ? (int)(kk + 1) : -1;
            g.rev = c->serpentine ? (int)((kk + 1) & 1) : 0;
            const bool sampled = kk % c->timing_stride == 0;
            ev_begin(c, flush ? 0 : refresh ? 23 : 2, sampled, flush || refresh ? -1 : (PE > PS ? 24 : 3) + PS);
            tci::launch_pass(c->stream, PE, flush, shadow, g, grid, flush ? 1 : refresh ? 2 : 0);
            ev_end(c, sampled);
            if (g.selk >= 0 && (st = select(g.selk))) return st;
            if (flush) te = ts = kk + 1;
            if (refresh) ts = kk + 1;
        }
        k = kend;
        if (k >= mr) break;
        bool stopped = false;
        if ((st = poll.after_chunk(&stopped))) return st;
        if (stopped) break;
        chunk = std::min<int64_t>(chunk * 2, StopPoll::kMaxChunk);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->hst, c->st, sizeof(RrluState), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int64_t np = c->hst->np;
    double err = c->hst->error;
    if (np >= std::min(m, n)) err = 0.0;  // matrixlu.jl:391-393
    *np_out = np;
    *err_out = err;
    return TCI_OK;
}

}  // namespace

// =================================================================== C ABI
extern "C" {

int tci_ctx_create(int device, tci_ctx** out) {
    if (!out) return TCI_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return TCI_ERR_DEVICE;
    if (device < 0 || device >= ndev) return TCI_ERR_ARG;
    tci_ctx* c = new tci_ctx();
    c->device = device;
    if (const char* e = getenv("TCI_RRLU_NB")) c->flush_every = std::max(1, std::min(atoi(e), tci::kMaxPend));
    if (const char* e = getenv("TCI_RRLU_SERP")) c->serpentine = atoi(e) != 0;
    // 0 = by shape, as tci_set_rrlu_epochs(0)
    if (const char* e = getenv("TCI_RRLU_EPOCHS")) c->epochs = std::max(0, std::min(atoi(e), tci::kMaxPendR));
    if (const char* e = getenv("TCI_RRLU_SHADOW")) c->shadow = atoi(e) != 0;
    if (const char* e = getenv("TCI_PASS_GRIDX")) c->pass_gridx = std::max(1, std::min(atoi(e), 8));
    if (const char* e = getenv("TCI_PASS_GRIDDIV")) c->pass_griddiv = std::max(1, std::min(atoi(e), 16));
    if (const char* e = getenv("TCI_RRLU_SMALL")) c->small_path = atoi(e) != 0;
    if (const char* e = getenv("TCI_SWEEP_SMALL")) c->small_sweep = atoi(e) != 0;
    if (const char* e = getenv("TCI_SW_LUWAVE")) c->sw_lu_wave = atoi(e) != 0;
    if (const char* e = getenv("TCI_SW_LAZYU")) c->sw_lazy_union = atoi(e) != 0;
    if (const char* e = getenv("TCI_RRLU_MID")) c->mid_path = atoi(e) != 0;
    if (const char* e = getenv("TCI_RRLU_PERSIST")) c->persist = tci::kEpochGrid && atoi(e) != 0;
    if (const char* e = getenv("TCI_SHARD_EXCHANGE")) c->sh_exchange = std::max(0, std::min(atoi(e), 2));
    if (const char* e = getenv("TCI_EPOCH_KINDS")) c->persist_kinds = atoi(e);
    if (const char* e = getenv("TCI_EPOCH_MAXPASS")) c->persist_maxpass = std::max(1, atoi(e));
    if (const char* e = getenv("TCI_C128_NB")) c->c128_nb = std::max(0, std::min(atoi(e), tci::kMaxPend - 1));
    if (const char* e = getenv("TCI_C128_SH")) c->c128_sh = atoi(e) != 0;
    if (const char* e = getenv("TCI_DENSE_MFMA")) c->dense = std::max(0, std::min(atoi(e), (int)tci::kDenseAll));
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->ncu = prop.multiProcessorCount;
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return TCI_ERR_DEVICE;
    }
    bool ok = hipMalloc((void**)&c->st, sizeof(RrluState)) == hipSuccess &&
              hipHostMalloc((void**)&c->hst, sizeof(RrluState), 0) == hipSuccess &&
              hipMalloc((void**)&c->flag, sizeof(int)) == hipSuccess &&
              hipMalloc((void**)&c->ticket, 256 * sizeof(unsigned)) == hipSuccess &&
              hipMalloc((void**)&c->bar, sizeof(unsigned)) == hipSuccess &&
              hipMalloc((void**)&c->fault, sizeof(int)) == hipSuccess &&
              hipMemset(c->ticket, 0, 256 * sizeof(unsigned)) == hipSuccess &&
              hipHostMalloc((void**)&c->hflag, sizeof(int), 0) == hipSuccess &&
              hipHostMalloc((void**)&c->hpoll, 2 * sizeof(RrluState), 0) == hipSuccess &&
              hipEventCreateWithFlags(&c->pollev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&c->pollev[1], hipEventDisableTiming) == hipSuccess &&
              hipMalloc((void**)&c->maxbits, sizeof(unsigned long long)) == hipSuccess &&
              hipHostMalloc((void**)&c->hmaxbits, sizeof(unsigned long long), 0) == hipSuccess;
    if (!ok) {
        tci_ctx_destroy(c);
        return TCI_ERR_NOMEM;
    }
    *out = c;
    return TCI_OK;
}

int tci_ctx_destroy(tci_ctx* c) {
    if (!c) return TCI_OK;
    if (c->stream) hipStreamSynchronize(c->stream);
    auto fr = [](void* p) { if (p) hipFree(p); };
    fr(c->dA); fr(c->sbuf); fr(c->cand); fr(c->st); fr(c->rowperm); fr(c->colperm); fr(c->xbuf); fr(c->ybuf); fr(c->flag);
    fr(c->ticket); fr(c->esync); fr(c->bar); fr(c->fault); fr(c->colbuf);
    fr(c->maxbits); fr(c->scratch); fr(c->scratch2); fr(c->dI); fr(c->dJ); fr(c->dI2); fr(c->dF1); fr(c->dF2);
    fr(c->dDiag);
    fr(c->dPiv); fr(c->dPbak); fr(c->rowpos); fr(c->colpos); fr(c->pivv); fr(c->Lp); fr(c->Up); fr(c->dL);
    fr(c->dU); fr(c->cws); fr(c->dRe); fr(c->colposL); fr(c->shsend); fr(c->shrecv); fr(c->lout);
    if (c->hst) hipHostFree(c->hst);
    if (c->hCoop) hipHostFree(c->hCoop);
    if (c->hflag) hipHostFree(c->hflag);
    if (c->hpoll) hipHostFree(c->hpoll);
    for (auto e : c->pollev)
        if (e) hipEventDestroy(e);
    if (c->hmaxbits) hipHostFree(c->hmaxbits);
    if (c->hin) hipHostFree(c->hin);
    if (c->hina) hipHostFree(c->hina);
    fr(c->dIa); fr(c->dJa);
    if (c->ev_ina) hipEventDestroy(c->ev_ina);
    if (c->hout) hipHostFree(c->hout);
    if (c->hd2h) hipHostFree(c->hd2h);
    for (auto e : c->d2h_ev)
        if (e) hipEventDestroy(e);
    if (c->zbuf) hipHostFree(c->zbuf);
    fr(c->sw_ws); fr(c->sw_inbuf); fr(c->sw_tens); fr(c->sw_fmap); fr(c->sw_img[0]); fr(c->sw_img[1]); fr(c->sw_ctl);
    if (c->hctl) hipHostFree(c->hctl);
    if (c->sw_s1t) hipHostFree(c->sw_s1t);
    if (c->sw_fmax) hipHostFree(c->sw_fmax);
    if (c->sw_in) hipHostFree(c->sw_in);
    if (c->sw_out) hipHostFree(c->sw_out);
    if (c->hfn) hipHostFree(c->hfn);
    for (auto e : c->evpool) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return TCI_OK;
}

const char* tci_last_error(const tci_ctx* c) { return c ? c->err.c_str() : "null context"; }
void* tci_ctx_stream(tci_ctx* c) { return c ? (void*)c->stream : nullptr; }
int tci_ctx_synchronize(tci_ctx* c) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}
int tci_set_rrlu_flush(tci_ctx* c, int nb) {
    if (nb < 1 || nb > tci::kMaxPend)
        return set_err(c, TCI_ERR_ARG, "flush interval must be in 1.." + std::to_string(tci::kMaxPend));
    c->flush_every = nb;
    return TCI_OK;
}

int tci_set_rrlu_epochs(tci_ctx* c, int epochs) {
    if (!c || epochs < 0 || epochs > tci::kMaxPendR)
        return set_err(c, TCI_ERR_ARG, "epochs must be in 0 (by shape) .. " + std::to_string(tci::kMaxPendR));
    c->epochs = epochs;
    return TCI_OK;
}

int tci_rrlu_epochs_for(tci_ctx* c, int64_t m, int64_t n) { return c ? rrlu_epochs(c, m, n) : 0; }

int tci_set_rrlu_small(tci_ctx* c, int enabled) {
    c->small_path = enabled != 0;
    return TCI_OK;
}

int tci_set_sweep_small(tci_ctx* c, int enabled) {
    if (!c) return TCI_ERR_ARG;
    c->small_sweep = enabled != 0;
    return TCI_OK;
}

int tci_set_rrlu_shadow(tci_ctx* c, int enabled) {
    c->shadow = enabled != 0;
    return TCI_OK;
}

int tci_rrlu_shadow_bytes(void) { return tci::shadow_elem_bytes(); }

int tci_set_c128_shadow(tci_ctx* c, int enabled) {
    c->c128_sh = enabled != 0;
    return TCI_OK;
}

int tci_set_dense_mfma(tci_ctx* c, int mask) {
    if (!c || mask < 0 || mask > tci::kDenseAll) return TCI_ERR_ARG;
    c->dense = mask;
    return TCI_OK;
}

int tci_set_rrlu_mid(tci_ctx* c, int enabled) {
    c->mid_path = enabled != 0;
    c->mid_faulted = 0;
    return TCI_OK;
}

int tci_set_rrlu_persist(tci_ctx* c, int enabled) {
    if (!c) return TCI_ERR_ARG;
    if (enabled < 0 || enabled > 2) return set_err(c, TCI_ERR_ARG, "persist must be 0, 1 or 2 (test mode)");
    if (enabled && !tci::kEpochGrid)
        return set_err(c, TCI_ERR_ARG, "the persistent epoch grid is not built (default; -DTCI_EPOCH_GRID=1)");
    c->persist = enabled;
    c->persist_faulted = 0;
    return TCI_OK;
}

int tci_rrlu_persist_faulted(tci_ctx* c) { return c ? c->persist_faulted : -1; }

int tci_set_shard_exchange(tci_ctx* c, int mode) {
    if (!c) return TCI_ERR_ARG;
    if (mode < 0 || mode > 2) return set_err(c, TCI_ERR_ARG, "shard exchange must be 0 (by size), 1 or 2");
    c->sh_exchange = mode;
    return TCI_OK;
}

int tci_last_shard_exchange(tci_ctx* c) { return c ? c->sh_exchange_used : -1; }

int tci_set_timing(tci_ctx* c, int enabled) {
    c->timing = enabled > 0;
    c->timing_stride = enabled > 0 ? enabled : 1;
    ev_reset(c);
    return TCI_OK;
}
int tci_last_kernel_stats(tci_ctx* c, int family, double* total_ms, int64_t* launches) {
    return tci_last_kernel_units(c, family, total_ms, launches, nullptr);
}
int tci_last_kernel_units(tci_ctx* c, int family, double* total_ms, int64_t* launches, int64_t* units) {
    if (!c) return TCI_ERR_ARG;
    if (family < 0 || family >= tci_ctx::kFams)
        return set_err(c, TCI_ERR_ARG, "family must be in 0.." + std::to_string(tci_ctx::kFams - 1));
    ev_collect(c);
    if (total_ms) *total_ms = c->fam_ms[family];
    if (launches) *launches = c->fam_n[family];
    if (units) *units = c->fam_u[family];
    return TCI_OK;
}

int tci_func_create(tci_ctx* c, int kind, const double* params, int64_t nparams,
                    const int32_t* localdims, int32_t L, tci_func** out) {
    if (!c || !out) return TCI_ERR_ARG;
    if (kind < TCI_F_SUM || kind > TCI_F_MPO) return set_err(c, TCI_ERR_ARG, "unknown integrand kind");
    if (L < 1) return set_err(c, TCI_ERR_ARG, "L must be >= 1");
    if (L > 62 && (kind == TCI_F_QOSC || kind == TCI_F_QEXP))
        return set_err(c, TCI_ERR_ARG, "quantics integrands support at most 62 legs");
    int32_t cpK = 0, mpoEnv = 0, mpoTmp = 0;
    if (kind == TCI_F_GAUSSMIX || kind == TCI_F_CP) {
        if (nparams < 2 || !params || params[0] < 0) return set_err(c, TCI_ERR_ARG, "params too short");
        cpK = (int32_t)params[0];
        int64_t need = 2 + (int64_t)cpK * L + cpK;  // GAUSSMIX: K, a, centres, weights
        if (kind == TCI_F_CP) {
            const int64_t dmax = (int64_t)params[1];
            for (int t = 0; t < L; ++t)
                if (localdims[t] > dmax) return set_err(c, TCI_ERR_ARG, "CP: localdims exceed dmax");
            need = 2 + (int64_t)cpK * L * dmax;
        }
        if (nparams < need) return set_err(c, TCI_ERR_ARG, "params too short for K terms");
    }
    if (kind == TCI_F_MPO) {
        // Contraction(A, B) (contraction.jl:121-152): matching lengths, shared index d2, bonds
        if (nparams < 1 || !params || (int64_t)params[0] != L)
            return set_err(c, TCI_ERR_ARG, "Tensor trains must have the same length.");
        if (nparams < 1 + 9 * (int64_t)L) return set_err(c, TCI_ERR_ARG, "MPO params too short");
        const int64_t hdr = 1 + 9 * (int64_t)L;
        for (int t = 0; t < L; ++t) {
            const double* q = params + 1 + 9 * t;
            const int64_t ra = (int64_t)q[0], d1 = (int64_t)q[1], d2 = (int64_t)q[2], ra2 = (int64_t)q[3];
            const int64_t rb = (int64_t)q[4], d3 = (int64_t)q[5], rb2 = (int64_t)q[6];
            const int64_t offA = (int64_t)q[7], offB = (int64_t)q[8];
            if (ra < 1 || d1 < 1 || d2 < 1 || ra2 < 1 || rb < 1 || d3 < 1 || rb2 < 1)
                return set_err(c, TCI_ERR_ARG, "MPO: dimensions must be positive");
            if (d1 * d3 != localdims[t]) return set_err(c, TCI_ERR_ARG, "MPO: localdims[t] must be d1 * d3");
            if ((t == 0 && (ra != 1 || rb != 1)) || (t == L - 1 && (ra2 != 1 || rb2 != 1)))
                return set_err(c, TCI_ERR_ARG, "MPO: boundary bond dimensions must be 1");
            if (t + 1 < L) {
                const double* nq = params + 1 + 9 * (t + 1);
                if ((int64_t)nq[0] != ra2 || (int64_t)nq[4] != rb2)
                    return set_err(c, TCI_ERR_ARG, "MPO: bond dimensions do not match");
            }
            if (ra * rb > tci::kMpoEnv || rb * d2 * ra2 > tci::kMpoTmp || ra * d2 * rb2 > tci::kMpoTmp)
                return set_err(c, TCI_ERR_ARG, "MPO: bond dimensions exceed the environment kernel's LDS");
            if (offA < 0 || offB < 0 || hdr + offA + ra * d1 * d2 * ra2 > nparams ||
                hdr + offB + rb * d2 * d3 * rb2 > nparams)
                return set_err(c, TCI_ERR_ARG, "MPO: cores outside params");
            cpK = std::max<int32_t>(cpK, (int32_t)(ra * rb));
            // LDS of k_mpo_env / k_mpo_env_mfma: environments (ra + 1) rb, intermediates
            // (rb d2 + 1) ra' (left chain) / (ra d2 + 1) rb' (right chain)
            mpoEnv = std::max<int32_t>(mpoEnv, (int32_t)std::max((ra + 1) * rb, (ra2 + 1) * rb2));
            mpoTmp = std::max<int32_t>(mpoTmp, (int32_t)std::max((rb * d2 + 1) * ra2, (ra * d2 + 1) * rb2));
        }
    }
    if (kind == TCI_F_TABLE) {
        int64_t cnt = 1;
        for (int t = 0; t < L; ++t) cnt *= localdims[t];
        if (nparams < cnt) return set_err(c, TCI_ERR_ARG, "table smaller than prod(localdims)");
    }
    tci_func* f = new tci_func();
    f->ctx = c;
    f->kind = kind;
    f->cpK = cpK;
    f->mpoEnv = mpoEnv;
    f->mpoTmp = mpoTmp;
    if (kind == TCI_F_LORENTZ) {  // quotient table p0 / (s + 1) for every reachable s
        int64_t smax = 0;
        for (int t = 0; t < L; ++t) smax += (int64_t)localdims[t] * localdims[t];
        f->ntab = smax < (1 << 20) ? smax + 1 : 0;
    }
    f->L = L;
    f->localdims.assign(localdims, localdims + L);
    f->nparams = nparams;
    std::vector<int64_t> strides(L + 1, 1);
    for (int t = 0; t < L; ++t) strides[t + 1] = strides[t] * localdims[t];
    bool ok = hipMalloc((void**)&f->dparams, std::max<int64_t>(nparams, 1) * sizeof(double)) == hipSuccess &&
              hipMalloc((void**)&f->dld, L * sizeof(int32_t)) == hipSuccess &&
              hipMalloc((void**)&f->dstrides, (L + 1) * sizeof(int64_t)) == hipSuccess;
    if (!ok) {
        tci_func_destroy(f);
        return set_err(c, TCI_ERR_NOMEM, "integrand allocation failed");
    }
    if (nparams > 0) hipMemcpy(f->dparams, params, nparams * sizeof(double), hipMemcpyHostToDevice);
    hipMemcpy(f->dld, localdims, L * sizeof(int32_t), hipMemcpyHostToDevice);
    hipMemcpy(f->dstrides, strides.data(), (L + 1) * sizeof(int64_t), hipMemcpyHostToDevice);
    *out = f;
    return TCI_OK;
}

int tci_func_create_host(tci_ctx* c, tci_host_fn fn, void* user, const int32_t* localdims, int32_t L,
                         tci_func** out) {
    if (!c || !out || !fn || !localdims) return TCI_ERR_ARG;
    if (L < 1) return set_err(c, TCI_ERR_ARG, "L must be >= 1");
    for (int t = 0; t < L; ++t)
        if (localdims[t] < 1) return set_err(c, TCI_ERR_ARG, "localdims must be positive");
    tci_func* f = new tci_func();
    f->ctx = c;
    f->kind = TCI_F_HOST;
    f->hostfn = fn;
    f->hostuser = user;
    f->L = L;
    f->localdims.assign(localdims, localdims + L);
    if (hipMalloc((void**)&f->dld, L * sizeof(int32_t)) != hipSuccess) {
        tci_func_destroy(f);
        return set_err(c, TCI_ERR_NOMEM, "integrand allocation failed");
    }
    hipMemcpy(f->dld, localdims, L * sizeof(int32_t), hipMemcpyHostToDevice);
    *out = f;
    return TCI_OK;
}

int tci_func_create_c128(tci_ctx* c, const tci_func* const* re, int32_t nre, const tci_func* const* im,
                         int32_t nim, tci_func** out) {
    if (!c || !out || nre < 0 || nim < 0 || nre + nim < 1 || (nre && !re) || (nim && !im)) return TCI_ERR_ARG;
    const tci_func* first = nre ? re[0] : im[0];
    if (!first) return set_err(c, TCI_ERR_ARG, "complex integrand: parts must be real integrands on the same localdims");
    tci_func* f = new tci_func();
    f->ctx = c;
    f->kind = TCI_F_C128;
    f->L = first->L;
    f->localdims = first->localdims;
    for (int i = 0; i < nre + nim; ++i) {
        const tci_func* p = i < nre ? re[i] : im[i - nre];
        if (!p || p->kind == TCI_F_C128 || p->L != f->L || p->localdims != f->localdims) {
            delete f;
            return set_err(c, TCI_ERR_ARG, "complex integrand: parts must be real integrands on the same localdims");
        }
        f->cparts.push_back(p);
    }
    f->cnre = nre;
    *out = f;
    return TCI_OK;
}

int tci_func_destroy(tci_func* f) {
    if (!f) return TCI_OK;
    if (f->dparams) hipFree(f->dparams);
    if (f->dld) hipFree(f->dld);
    if (f->dstrides) hipFree(f->dstrides);
    delete f;
    return TCI_OK;
}

int tci_batcheval_d(tci_ctx* c, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                    const int32_t* J, int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo,
                    double* maxabs) {
    if (!c || !f) return TCI_ERR_ARG;
    int st;
    // both index tables up through one pinned stage (pageable copies would stage twice)
    const size_t bi = (size_t)std::max<int64_t>(m * nl, 0) * 4, bj = (size_t)std::max<int64_t>(n * nr, 0) * 4;
    if ((st = ensure(c, &c->dI, &c->capI, std::max<size_t>(bi / 4, 1)))) return st;
    if ((st = ensure(c, &c->dJ, &c->capJ, std::max<size_t>(bj / 4, 1)))) return st;
    if ((st = ensure_pinned(c, &c->hin, &c->capHin, bi + bj + 16))) return st;
    if (bi) memcpy(c->hin, I, bi);
    if (bj) memcpy(c->hin + bi, J, bj);
    if (bi) HIPCHK(c, hipMemcpyAsync(c->dI, c->hin, bi, hipMemcpyHostToDevice, c->stream));
    if (bj) HIPCHK(c, hipMemcpyAsync(c->dJ, c->hin + bi, bj, hipMemcpyHostToDevice, c->stream));
    return batcheval_device(c, f, c->dI, m, nl, c->dJ, n, nr, M, d_out, ldo, maxabs);
}

int tci_batcheval_dd(tci_ctx* c, const tci_func* f, const int32_t* dI, int64_t m, int32_t nl, const int32_t* dJ,
                     int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo, uint64_t* d_maxbits) {
    if (!c || !f || !d_maxbits || (m > 0 && nl > 0 && !dI) || (n > 0 && nr > 0 && !dJ)) return TCI_ERR_ARG;
    if (f->kind == TCI_F_C128)
        return set_err(c, TCI_ERR_ARG, "a ComplexF64 integrand needs the ComplexF64 entries (*_c128_*)");
    return batcheval_launch(c, f, dI, m, nl, dJ, n, nr, M, d_out, ldo,
                            reinterpret_cast<unsigned long long*>(d_maxbits));
}

int tci_batcheval_da(tci_ctx* c, const tci_func* f, const int32_t* I, int64_t m, int32_t nl, const int32_t* J,
                     int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo, uint64_t* d_maxbits) {
    if (!c || !f || !d_maxbits || (m > 0 && nl > 0 && !I) || (n > 0 && nr > 0 && !J)) return TCI_ERR_ARG;
    if (f->kind == TCI_F_HOST || f->kind == TCI_F_C128)
        return set_err(c, TCI_ERR_ARG, "tci_batcheval_da: host and ComplexF64 integrands need tci_batcheval_d / *_c128_*");
    int st;
    const size_t bi = (size_t)std::max<int64_t>(m * nl, 0) * 4, bj = (size_t)std::max<int64_t>(n * nr, 0) * 4;
    if ((st = ensure(c, &c->dIa, &c->capIa, std::max<size_t>(bi / 4, 1)))) return st;
    if ((st = ensure(c, &c->dJa, &c->capJa, std::max<size_t>(bj / 4, 1)))) return st;
    if (!c->ev_ina) HIPCHK(c, hipEventCreateWithFlags(&c->ev_ina, hipEventDisableTiming));
    if (c->ev_ina_live) HIPCHK(c, hipEventSynchronize(c->ev_ina));  // the last upload has left the stage
    c->ev_ina_live = false;
    if ((st = ensure_pinned(c, &c->hina, &c->capHina, bi + bj + 16))) return st;
    if (bi) memcpy(c->hina, I, bi);
    if (bj) memcpy(c->hina + bi, J, bj);
    if (bi) HIPCHK(c, hipMemcpyAsync(c->dIa, c->hina, bi, hipMemcpyHostToDevice, c->stream));
    if (bj) HIPCHK(c, hipMemcpyAsync(c->dJa, c->hina + bi, bj, hipMemcpyHostToDevice, c->stream));
    if (bi || bj) {
        HIPCHK(c, hipEventRecord(c->ev_ina, c->stream));
        c->ev_ina_live = true;
    }
    return batcheval_launch(c, f, c->dIa, m, nl, c->dJa, n, nr, M, d_out, ldo,
                            reinterpret_cast<unsigned long long*>(d_maxbits));
}

int tci_batcheval_h(tci_ctx* c, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                    const int32_t* J, int64_t n, int32_t nr, int32_t M, double* out, int64_t ldo,
                    double* maxabs) {
    if (!c || !f) return TCI_ERR_ARG;
    if (nl + M + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    const int64_t D = M ? f->localdims[nl] : 1;
    const int64_t mR = m * D;
    const int64_t ld = round_up(std::max<int64_t>(mR, 1), 2);
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(ld * std::max<int64_t>(n, 1))))) return st;
    if ((st = tci_batcheval_d(c, f, I, m, nl, J, n, nr, M, c->dA, ld, maxabs))) return st;
    if (mR > 0 && n > 0)
        HIPCHK(c, hipMemcpy2DAsync(out, ldo * sizeof(double), c->dA, ld * sizeof(double),
                                   mR * sizeof(double), n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_rrlu_inplace_d(tci_ctx* c, double* dA, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
                       double reltol, double abstol, int leftorth, int64_t* rowperm,
                       int64_t* colperm, int64_t* npivot, double* lasterror, double* pivoterrors) {
    if (!c || !npivot || !lasterror) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || lda < m || (lda & 1) || ((uintptr_t)dA & 15))
        return set_err(c, TCI_ERR_ARG, "rrlu: need lda >= m, lda even and a 16-byte aligned matrix");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int st;
    if ((st = rrlu_device(c, dA, m, n, lda, maxrank, reltol, abstol, leftorth, npivot, lasterror)))
        return st;
    if ((st = extract_LU(c, m, n, *npivot, leftorth, false, false))) return st;  // NaN checks
    if ((st = fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0))) return st;
    return pivot_errors(c, *npivot, *lasterror, pivoterrors);
}

int tci_rrlu_copy_d(tci_ctx* c, const double* d_src, int64_t ldsrc, double* dW, int64_t m, int64_t n, int64_t ldw,
                    int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowperm,
                    int64_t* colperm, int64_t* npivot, double* lasterror, double* pivoterrors) {
    if (!c || !npivot || !lasterror) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || ldw < m || (ldw & 1) || ((uintptr_t)dW & 15) || ldsrc < m || (m > 0 && n > 0 && !d_src))
        return set_err(c, TCI_ERR_ARG, "rrlu: need ld >= m for both matrices, ldw even and a 16-byte aligned work matrix");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    // the two must not overlap: the copy is fused into a pass that reads one while writing the other
    const uintptr_t s0 = (uintptr_t)d_src, s1 = (uintptr_t)(d_src + ldsrc * std::max<int64_t>(n, 1));
    const uintptr_t w0 = (uintptr_t)dW, w1 = (uintptr_t)(dW + ldw * std::max<int64_t>(n, 1));
    if (m > 0 && n > 0 && s0 < w1 && w0 < s1) return set_err(c, TCI_ERR_ARG, "rrlu: input and work matrix overlap");
    int st;
    if ((st = rrlu_device(c, dW, m, n, ldw, maxrank, reltol, abstol, leftorth, npivot, lasterror, d_src, ldsrc)))
        return st;
    if ((st = extract_LU(c, m, n, *npivot, leftorth, false, false))) return st;  // NaN checks
    if ((st = fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0))) return st;
    return pivot_errors(c, *npivot, *lasterror, pivoterrors);
}

int tci_rrlu_h(tci_ctx* c, const double* A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
               double reltol, double abstol, int leftorth, int64_t* rowperm, int64_t* colperm,
               double* L, double* U, int64_t ldu, int64_t* npivot, double* lasterror) {
    if (!c || !npivot || !lasterror || (m > 0 && n > 0 && !A)) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || lda < std::max<int64_t>(m, 1) - (m == 0))
        return set_err(c, TCI_ERR_ARG, "rrlu: invalid dimensions");
    int64_t ld;
    int st;
    if ((st = upload_matrix(c, A, m, n, lda, &ld))) return st;
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    if ((st = rrlu_device(c, c->dA, m, n, ld, maxrank, reltol, abstol, leftorth, npivot, lasterror)))
        return st;
    const int64_t np = *npivot;
    if ((st = extract_LU(c, m, n, np, leftorth, L != nullptr, U != nullptr))) return st;
    if ((st = fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0))) return st;
    if (np > 0 && L)
        HIPCHK(c, hipMemcpyAsync(L, c->dL, m * np * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (np > 0 && U)
        HIPCHK(c, hipMemcpy2DAsync(U, ldu * sizeof(double), c->dU, np * sizeof(double),
                                   np * sizeof(double), n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

// ComplexF64 rrLU on a device matrix (double2, ld >= m): steps, then np / lu.error to the host;
// the pivot column buffer holds the pivot errors afterwards when want_pe
static int crrlu_device(tci_ctx* c, double2* dA, int64_t ld, int64_t m, int64_t n, int64_t mr,
                        double reltol, double abstol, int leftorth, int64_t* np_out,
                        double* err_out, tci::CState** st_out, double2** colbuf_out) {
    c->sh_valid = 0;
    const int mi = (int)m, ni = (int)n;
    const int G = tci::crrlu_grid(mi, ni, 0);
    auto al = [](size_t b) { return (b + 255) / 256 * 256; };
    const size_t oSt = 0, oCand = al(sizeof(tci::CState)), oCol = oCand + al(sizeof(tci::CCand) * G);
    const size_t oRow = oCol + al(16 * (size_t)std::max(mi, 1));
    // deferred updates: pending slots X (kMaxPend x ldx), Y (kMaxPend x ldy), stash
    const int64_t ldx = round_up(std::max<int64_t>(m, 1), 16), ldy = round_up(std::max<int64_t>(n, 1), 16);
    const size_t oX = oRow + al(16 * (size_t)std::max(ni, 1));
    const size_t oY = oX + al(16 * (size_t)(tci::kMaxPend * ldx));
    const size_t oS = oY + al(16 * (size_t)(tci::kMaxPend * ldy));
    // shadow search: |pivot t|, the MFMA fragments (64 halves per row, 128 per column)
    const size_t oPm = oS + al(16 * 4 * tci::kMaxPend);
    const size_t oXA = oPm + al(8 * (size_t)(mr + 1));
    const size_t oYB = oXA + al(128 * (size_t)std::max(mi, 1));
    const size_t bytes = oYB + al(256 * (size_t)std::max(ni, 1));
    int st;
    if ((st = ensure(c, &c->cws, &c->capCws, bytes))) return st;
    if ((st = ensure(c, &c->rowperm, &c->capPerm, (size_t)m + 1))) return st;
    if ((st = ensure(c, &c->colperm, &c->capColperm, (size_t)n + 1))) return st;
    tci::CState* dst = reinterpret_cast<tci::CState*>(c->cws + oSt);
    tci::launch_crrlu_init(c->stream, dst, c->rowperm, c->colperm, mi, ni);
    HIPCHK(c, hipGetLastError());
    tci::CStepArgs g{};
    g.A = dA;
    g.ld = ld;
    g.m = mi;
    g.n = ni;
    g.mr = (int)mr;
    g.leftorth = leftorth;
    g.reltol = reltol;
    g.abstol = abstol;
    g.st = dst;
    g.cand = reinterpret_cast<tci::CCand*>(c->cws + oCand);
    g.colbuf = reinterpret_cast<double2*>(c->cws + oCol);
    g.rowbuf = reinterpret_cast<double2*>(c->cws + oRow);
    g.rowperm = c->rowperm;
    g.colperm = c->colperm;
    g.X = reinterpret_cast<double2*>(c->cws + oX);
    g.ldx = ldx;
    g.Y = reinterpret_cast<double2*>(c->cws + oY);
    g.ldy = ldy;
    g.stash = reinterpret_cast<double2*>(c->cws + oS);
    g.pmod = reinterpret_cast<double*>(c->cws + oPm);
    g.sh = 0;
    if (c->c128_nb != 0 && c->c128_sh && m >= 64 && n >= 64) {
        // certified shadow search (K8): fp16 planes of Re / Im (the Float64 path's shadow buffer,
        // same size), fragments zeroed, shadow padding rows [m, lds) zeroed
        g.lds = round_up(m, 16);
        if ((st = ensure(c, &c->sbuf, &c->capS, (size_t)(g.lds * n)))) return st;
        g.SR = reinterpret_cast<uint16_t*>(c->sbuf);
        g.SI = g.SR + g.lds * n;
        g.XA = reinterpret_cast<uint16_t*>(c->cws + oXA);
        g.YB = reinterpret_cast<uint16_t*>(c->cws + oYB);
        HIPCHK(c, hipMemsetAsync(g.XA, 0, oYB - oXA + 256 * (size_t)std::max(ni, 1), c->stream));
        if (g.lds > m) {
            HIPCHK(c, hipMemset2DAsync(g.SR + m, (size_t)(2 * g.lds), 0, (size_t)(2 * (g.lds - m)), (size_t)n,
                                       c->stream));
            HIPCHK(c, hipMemset2DAsync(g.SI + m, (size_t)(2 * g.lds), 0, (size_t)(2 * (g.lds - m)), (size_t)n,
                                       c->stream));
        }
        g.sh = 1;
    }
    if (c->c128_nb != 0) {
        // deferred updates (K8): pending pivots t0 .. t-1 applied on the fly, written back when
        // nb of them pend; steps after the stop test fired return at once (st->done). With the
        // shadow search, steps with 1..kCShMaxP pending read the fp16 shadow (step 1 is exact and
        // writes the shadow of A's stale values)
        const int nb = std::min(c->c128_nb > 0 ? c->c128_nb : (g.sh ? 11 : 6), tci::kMaxPend - 1);
        const bool check = getenv("TCI_CSH_CHECK") != nullptr;
        int t0 = 0;
        int64_t chunk = 2;
        StopPoll poll(c, dst);  // the host stops launching soon after the device's stop test fired
        for (int t = 0, tend = 0; mr > 0 && t < mr; ++t) {
            if (t == tend && t > 0) {
                bool stopped = false;
                if ((st = poll.after_chunk(&stopped))) return st;
                if (stopped) break;
                chunk = std::min<int64_t>(chunk * 2, StopPoll::kMaxChunk);
            }
            if (t == tend) tend = (int)std::min<int64_t>(t + chunk, mr);
            g.t = t;
            const int P = t - t0;
            const bool flush = P >= nb;
            if (g.sh && !flush && P >= 1 && P <= tci::kCShMaxP) {
                if (t0 == 0 && t == 1)
                    tci::launch_crrlu_step_stale_sh(c->stream, g);
                else if (check)
                    tci::debug_crrlu_check_sh(c->stream, g, P);
                else
                    tci::launch_crrlu_step_sh(c->stream, g, P);
            } else {
                tci::launch_crrlu_step_d(c->stream, g, P, flush);
            }
            if (flush) t0 = t;
            HIPCHK(c, hipGetLastError());
        }
    } else {
        // round 1: one read + write of the trailing block per pivot (A/B switch TCI_C128_NB=0)
        for (int t = 0; mr > 0 && t <= mr; ++t) {
            g.t = t;
            tci::launch_crrlu_step(c->stream, g);
            HIPCHK(c, hipGetLastError());
        }
    }
    tci::CState hs;
    HIPCHK(c, hipMemcpyAsync(&hs, dst, sizeof hs, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *np_out = hs.np;
    *err_out = hs.np >= std::min(m, n) ? 0.0 : hs.err;
    *st_out = dst;
    *colbuf_out = g.colbuf;
    return TCI_OK;
}

// L / U extraction with the NaN checks of matrixlu.jl:376-381 (pivot errors into pe)
static int crrlu_extract(tci_ctx* c, double2* dA, int64_t ld, int64_t m, int64_t n, int64_t np,
                         int leftorth, double2* dL, double2* dU, double* pe, tci::CState* dst) {
    if (np <= 0) return TCI_OK;
    tci::launch_crrlu_extract(c->stream, dA, ld, (int)m, (int)n, (int)np, leftorth, dL, dU, np, pe,
                              &dst->nan);
    HIPCHK(c, hipGetLastError());
    tci::CState hs;
    HIPCHK(c, hipMemcpyAsync(&hs, dst, sizeof hs, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (hs.nan & 1) return set_err(c, TCI_ERR_NAN, "lu.L contains NaNs");
    if (hs.nan & 2) return set_err(c, TCI_ERR_NAN, "lu.U contains NaNs");
    return TCI_OK;
}

int tci_rrlu_c128_h(tci_ctx* c, const double* A, int64_t m, int64_t n, int64_t lda,
                    int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowperm,
                    int64_t* colperm, double* L, double* U, int64_t ldu, int64_t* npivot,
                    double* lasterror, double* pivoterrors) {
    if (!c || !npivot || !lasterror || (m > 0 && n > 0 && !A)) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || (m > 0 && n > 0 && lda < m))
        return set_err(c, TCI_ERR_ARG, "rrlu: invalid dimensions");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int64_t mr = std::min<int64_t>(maxrank, std::min<int64_t>(m, n));
    if (mr < 0) mr = 0;
    if (U && ldu < std::max<int64_t>(mr, 1)) return set_err(c, TCI_ERR_ARG, "rrlu: ldu < maxrank");
    const int64_t ld = std::max<int64_t>(m, 1);
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * ld * std::max<int64_t>(n, 1))))) return st;
    if ((st = ensure(c, &c->dL, &c->capL, (size_t)(2 * std::max<int64_t>(m * mr, 1))))) return st;
    if ((st = ensure(c, &c->dU, &c->capU, (size_t)(2 * std::max<int64_t>(mr * n, 1))))) return st;
    double2* dA = reinterpret_cast<double2*>(c->dA);
    if (m > 0 && n > 0)
        HIPCHK(c, hipMemcpy2DAsync(dA, ld * 16, A, lda * 16, m * 16, n, hipMemcpyHostToDevice,
                                   c->stream));
    int64_t np;
    double err;
    tci::CState* dst;
    double2* colbuf;
    if ((st = crrlu_device(c, dA, ld, m, n, mr, reltol, abstol, leftorth, &np, &err, &dst, &colbuf)))
        return st;
    double2* dL = reinterpret_cast<double2*>(c->dL);
    double2* dU = reinterpret_cast<double2*>(c->dU);
    double* dpe = reinterpret_cast<double*>(colbuf);  // free after the last step
    if ((st = crrlu_extract(c, dA, ld, m, n, np, leftorth, dL, dU, dpe, dst))) return st;
    *npivot = np;
    *lasterror = err;
    if ((st = fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0))) return st;
    if (np > 0 && L)
        HIPCHK(c, hipMemcpyAsync(L, dL, m * np * 16, hipMemcpyDeviceToHost, c->stream));
    if (np > 0 && U)
        HIPCHK(c, hipMemcpy2DAsync(U, ldu * 16, dU, np * 16, np * 16, n, hipMemcpyDeviceToHost,
                                   c->stream));
    if (np > 0 && pivoterrors)
        HIPCHK(c, hipMemcpyAsync(pivoterrors, dpe, np * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (pivoterrors) pivoterrors[np] = *lasterror;
    return TCI_OK;
}

// MatrixLUCI{ComplexF64} of the complex matrix already in c->dA (ld = max(m, 1))
static int cluci_core(tci_ctx* c, int64_t m, int64_t n, int64_t maxrank, double reltol,
                      double abstol, int leftorth, int64_t* rowidx, int64_t* colidx,
                      double* pivoterrors, double* left, double* right, int64_t* npivot) {
    int64_t mr = std::min<int64_t>(maxrank, std::min<int64_t>(m, n));
    if (mr < 0) mr = 0;
    const int64_t ld = std::max<int64_t>(m, 1);
    int st;
    if ((st = ensure(c, &c->dL, &c->capL, (size_t)(2 * std::max<int64_t>(m * mr, 1))))) return st;
    if ((st = ensure(c, &c->dU, &c->capU, (size_t)(2 * std::max<int64_t>(mr * n, 1))))) return st;
    double2* dA = reinterpret_cast<double2*>(c->dA);
    int64_t np;
    double err;
    tci::CState* dst;
    double2* colbuf;
    if ((st = crrlu_device(c, dA, ld, m, n, mr, reltol, abstol, leftorth, &np, &err, &dst, &colbuf)))
        return st;
    double2* dL = reinterpret_cast<double2*>(c->dL);
    double2* dU = reinterpret_cast<double2*>(c->dU);
    double* dpe = reinterpret_cast<double*>(colbuf);
    if ((st = crrlu_extract(c, dA, ld, m, n, np, leftorth, dL, dU, dpe, dst))) return st;
    *npivot = np;
    if (np > 0 && (st = fetch_perms(c, rowidx, colidx, rowidx ? np : 0, colidx ? np : 0))) return st;
    if (np > 0 && pivoterrors) {
        HIPCHK(c, hipMemcpyAsync(pivoterrors, dpe, np * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (pivoterrors) pivoterrors[np] = err;
    if (np > 0 && (left || right)) {
        if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(2 * m * np)))) return st;
        if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(2 * np * n)))) return st;
        tci::launch_cluci_factors(c->stream, dL, dU, (int)m, (int)n, (int)np, leftorth, c->rowperm,
                                  c->colperm, left ? reinterpret_cast<double2*>(c->dF1) : nullptr,
                                  right ? reinterpret_cast<double2*>(c->dF2) : nullptr);
        HIPCHK(c, hipGetLastError());
        if (left)
            HIPCHK(c, hipMemcpyAsync(left, c->dF1, m * np * 16, hipMemcpyDeviceToHost, c->stream));
        if (right)
            HIPCHK(c, hipMemcpyAsync(right, c->dF2, np * n * 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return TCI_OK;
}

int tci_luci_c128_h(tci_ctx* c, const double* A, int64_t m, int64_t n, int64_t lda,
                    int64_t maxrank, double reltol, double abstol, int leftorth, int64_t* rowidx,
                    int64_t* colidx, double* pivoterrors, double* left, double* right,
                    int64_t* npivot) {
    if (!c || !npivot || (m > 0 && n > 0 && !A)) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || (m > 0 && n > 0 && lda < m))
        return set_err(c, TCI_ERR_ARG, "MatrixLUCI: invalid dimensions");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    const int64_t ld = std::max<int64_t>(m, 1);
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * ld * std::max<int64_t>(n, 1))))) return st;
    if (m > 0 && n > 0)
        HIPCHK(c, hipMemcpy2DAsync(c->dA, ld * 16, A, lda * 16, m * 16, n, hipMemcpyHostToDevice,
                                   c->stream));
    return cluci_core(c, m, n, maxrank, reltol, abstol, leftorth, rowidx, colidx, pivoterrors, left,
                      right, npivot);
}

// TCI_F_C128: the complex Pi (interleaved, ld) in c->dA from the real parts (index tables uploaded
// once, each part's real values into c->dRe and added into its component in part order), then
// coeff * Pi and max|.| into c->maxbits. Launches only (the caller synchronises).
static int c128_parts_assemble(tci_ctx* c, const tci_func* f, double cre, double cim, const int32_t* I,
                               int64_t m, int32_t nl, const int32_t* J, int64_t n, int32_t nr, int32_t M,
                               int64_t ld) {
    const int64_t D = M ? f->localdims[nl] : 1, mR = m * D;
    int st;
    const size_t bi = (size_t)std::max<int64_t>(m * nl, 0) * 4, bj = (size_t)std::max<int64_t>(n * nr, 0) * 4;
    if ((st = ensure(c, &c->dI, &c->capI, std::max<size_t>(bi / 4, 1)))) return st;
    if ((st = ensure(c, &c->dJ, &c->capJ, std::max<size_t>(bj / 4, 1)))) return st;
    if ((st = ensure_pinned(c, &c->hin, &c->capHin, bi + bj + 16))) return st;
    if (bi) memcpy(c->hin, I, bi);
    if (bj) memcpy(c->hin + bi, J, bj);
    if (bi) HIPCHK(c, hipMemcpyAsync(c->dI, c->hin, bi, hipMemcpyHostToDevice, c->stream));
    if (bj) HIPCHK(c, hipMemcpyAsync(c->dJ, c->hin + bi, bj, hipMemcpyHostToDevice, c->stream));
    const int64_t ldr = round_up(std::max<int64_t>(mR, 1), 2);
    if ((st = ensure(c, &c->dRe, &c->capRe, (size_t)(ldr * std::max<int64_t>(n, 1))))) return st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * ld * std::max<int64_t>(n, 1))))) return st;
    if (mR > 0 && n > 0) {
        HIPCHK(c, hipMemsetAsync(c->dA, 0, (size_t)(2 * ld * n) * sizeof(double), c->stream));
        for (size_t p = 0; p < f->cparts.size(); ++p) {
            if ((st = batcheval_launch(c, f->cparts[p], c->dI, m, nl, c->dJ, n, nr, M, c->dRe, ldr))) return st;
            tci::launch_c128_accum(c->stream, c->dRe, ldr, (int)mR, (int)n, (int)p >= f->cnre ? 1 : 0,
                                   reinterpret_cast<double2*>(c->dA), ld);
        }
    }
    HIPCHK(c, hipMemsetAsync(c->maxbits, 0, sizeof(unsigned long long), c->stream));
    if (mR > 0 && n > 0)
        tci::launch_c128_finish(c->stream, (int)mR, (int)n, cre, cim, reinterpret_cast<double2*>(c->dA), ld,
                                c->maxbits);
    HIPCHK(c, hipGetLastError());
    return TCI_OK;
}

int tci_batcheval_c128_h(tci_ctx* c, const tci_func* f, double cre, double cim,
                         const int32_t* I, int64_t m, int32_t nl, const int32_t* J, int64_t n,
                         int32_t nr, int32_t M, double* out, double* maxabs) {
    if (c && f && maxabs && f->kind == TCI_F_C128) {
        if (nl + M + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
        if (M < 0 || M > 1) return set_err(c, TCI_ERR_ARG, "only M = 0 or M = 1 centre legs are supported");
        const int64_t mR = m * (M ? f->localdims[nl] : 1), ld = std::max<int64_t>(mR, 1);
        if (mR > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
        int st;
        if ((st = c128_parts_assemble(c, f, cre, cim, I, m, nl, J, n, nr, M, ld))) return st;
        if (out && mR > 0 && n > 0)
            HIPCHK(c, hipMemcpyAsync(out, c->dA, mR * n * 16, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        double mx;
        memcpy(&mx, c->hmaxbits, sizeof mx);
        *maxabs = (mR > 0 && n > 0) ? mx : 0.0;
        return TCI_OK;
    }
    if (!c || !f || !maxabs) return TCI_ERR_ARG;
    if (nl + M + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    const int64_t D = M ? f->localdims[nl] : 1;
    const int64_t mR = m * D;
    const int64_t ld = std::max<int64_t>(mR, 1);
    if (mR > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int st;
    if ((st = ensure(c, &c->dRe, &c->capRe, (size_t)(round_up(ld, 2) * std::max<int64_t>(n, 1)))))
        return st;
    double mxr = 0.0;
    if ((st = tci_batcheval_d(c, f, I, m, nl, J, n, nr, M, c->dRe, round_up(ld, 2), &mxr))) return st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * ld * std::max<int64_t>(n, 1))))) return st;
    HIPCHK(c, hipMemsetAsync(c->maxbits, 0, sizeof(unsigned long long), c->stream));
    tci::launch_c128_scale(c->stream, c->dRe, round_up(ld, 2), (int)mR, (int)n, cre, cim,
                           reinterpret_cast<double2*>(c->dA), ld, c->maxbits);
    HIPCHK(c, hipGetLastError());
    if (out && mR > 0 && n > 0)
        HIPCHK(c, hipMemcpyAsync(out, c->dA, mR * n * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double mx;
    memcpy(&mx, c->hmaxbits, sizeof mx);
    *maxabs = (mR > 0 && n > 0) ? mx : 0.0;
    return TCI_OK;
}

int tci_update_pivots_c128_h(tci_ctx* c, const tci_func* f, double cre, double cim,
                             const int32_t* rows, int64_t m, int32_t nl, const int32_t* cols,
                             int64_t n, int32_t nr, int64_t maxrank, double reltol, double abstol,
                             int leftorth, int want_factors, int64_t* rowidx, int64_t* colidx,
                             double* pivoterrors, int64_t* npivot, double* maxabs, double* left,
                             double* right) {
    if (!c || !f || !npivot || !maxabs) return TCI_ERR_ARG;
    if (nl + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    const int64_t ld = std::max<int64_t>(m, 1);
    int st;
    if (f->kind == TCI_F_C128) {  // Pi from the complex integrand's real parts
        if ((st = c128_parts_assemble(c, f, cre, cim, rows, m, nl, cols, n, nr, 0, ld))) return st;
        HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        double mx;
        memcpy(&mx, c->hmaxbits, sizeof mx);
        *maxabs = (m > 0 && n > 0) ? mx : 0.0;
        return cluci_core(c, m, n, maxrank, reltol, abstol, leftorth, rowidx, colidx, pivoterrors,
                          want_factors ? left : nullptr, want_factors ? right : nullptr, npivot);
    }
    // real values of f on the device, then Pi = coeff * f and max|Pi| (hypot) into c->dA
    if ((st = ensure(c, &c->dRe, &c->capRe, (size_t)(round_up(ld, 2) * std::max<int64_t>(n, 1)))))
        return st;
    double mxr = 0.0;
    if ((st = tci_batcheval_d(c, f, rows, m, nl, cols, n, nr, 0, c->dRe, round_up(ld, 2), &mxr)))
        return st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * ld * std::max<int64_t>(n, 1))))) return st;
    HIPCHK(c, hipMemsetAsync(c->maxbits, 0, sizeof(unsigned long long), c->stream));
    tci::launch_c128_scale(c->stream, c->dRe, round_up(ld, 2), (int)m, (int)n, cre, cim,
                           reinterpret_cast<double2*>(c->dA), ld, c->maxbits);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double mx;
    memcpy(&mx, c->hmaxbits, sizeof mx);
    *maxabs = (m > 0 && n > 0) ? mx : 0.0;
    return cluci_core(c, m, n, maxrank, reltol, abstol, leftorth, rowidx, colidx, pivoterrors,
                      want_factors ? left : nullptr, want_factors ? right : nullptr, npivot);
}

int tci_rrlu_c128_inplace_d(tci_ctx* c, double* d_A, int64_t m, int64_t n, int64_t lda,
                            int64_t maxrank, double reltol, double abstol, int leftorth,
                            int64_t* rowperm, int64_t* colperm, int64_t* npivot,
                            double* lasterror, double* pivoterrors) {
    if (!c || !npivot || !lasterror || (m > 0 && n > 0 && !d_A)) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || (m > 0 && n > 0 && lda < m))
        return set_err(c, TCI_ERR_ARG, "rrlu: invalid dimensions");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    if (reinterpret_cast<uintptr_t>(d_A) % 16)
        return set_err(c, TCI_ERR_ARG, "rrlu: device matrix must be 16-byte aligned");
    int64_t mr = std::min<int64_t>(maxrank, std::min<int64_t>(m, n));
    if (mr < 0) mr = 0;
    int64_t np;
    double err;
    tci::CState* dst;
    double2* colbuf;
    double2* dA = reinterpret_cast<double2*>(d_A);
    int st;
    if ((st = crrlu_device(c, dA, lda, m, n, mr, reltol, abstol, leftorth, &np, &err, &dst, &colbuf)))
        return st;
    // NaN checks need L / U: extract into the context's buffers
    if ((st = ensure(c, &c->dL, &c->capL, (size_t)(2 * std::max<int64_t>(m * np, 1))))) return st;
    if ((st = ensure(c, &c->dU, &c->capU, (size_t)(2 * std::max<int64_t>(np * n, 1))))) return st;
    double* dpe = reinterpret_cast<double*>(colbuf);
    if ((st = crrlu_extract(c, dA, lda, m, n, np, leftorth, reinterpret_cast<double2*>(c->dL),
                            reinterpret_cast<double2*>(c->dU), dpe, dst)))
        return st;
    *npivot = np;
    *lasterror = err;
    if ((st = fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0))) return st;
    if (np > 0 && pivoterrors) {
        HIPCHK(c, hipMemcpyAsync(pivoterrors, dpe, np * sizeof(double), hipMemcpyDeviceToHost,
                                 c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    if (pivoterrors) pivoterrors[np] = err;
    return TCI_OK;
}

// MatrixLUCI outputs after rrlu_device: pivot indices/errors and (optionally) the factors
static int luci_outputs(tci_ctx* c, int64_t m, int64_t n, int leftorth, int64_t np, double err,
                        int64_t* rowidx, int64_t* colidx, double* pivoterrs, double* left,
                        double* right) {
    int st;
    const bool fac = np > 0 && (left || right);
    if ((st = extract_LU(c, m, n, np, leftorth, fac, fac))) return st;
    if ((st = pivot_errors(c, np, err, pivoterrs))) return st;
    if (np > 0 && (st = fetch_perms(c, rowidx, colidx, rowidx ? np : 0, colidx ? np : 0))) return st;
    if (fac) {
        if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(m * np)))) return st;
        if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(np * n)))) return st;
        ev_begin(c, 21);
        tci::launch_luci_factors(c->stream, c->dL, m, c->dU, np, (int)m, (int)n, (int)np, leftorth,
                                 c->rowperm, c->colperm, left ? c->dF1 : nullptr,
                                 right ? c->dF2 : nullptr, c->dense);
        ev_end(c);
        HIPCHK(c, hipGetLastError());
        if (left && (st = d2h_large(c, left, c->dF1, (size_t)(m * np) * sizeof(double)))) return st;
        if (right && (st = d2h_large(c, right, c->dF2, (size_t)(np * n) * sizeof(double)))) return st;
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return TCI_OK;
}

int tci_luci_h(tci_ctx* c, const double* A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
               double reltol, double abstol, int leftorth, int64_t* rowidx, int64_t* colidx,
               double* pivoterrs, double* left, double* right, int64_t* npivot) {
    if (!c || !npivot) return TCI_ERR_ARG;
    int64_t ld, np;
    double err;
    int st;
    if ((st = upload_matrix(c, A, m, n, lda, &ld))) return st;
    if ((st = rrlu_device(c, c->dA, m, n, ld, maxrank, reltol, abstol, leftorth, &np, &err)))
        return st;
    *npivot = np;
    return luci_outputs(c, m, n, leftorth, np, err, rowidx, colidx, pivoterrs, left, right);
}

int tci_luci_inplace_d(tci_ctx* c, double* d_A, int64_t m, int64_t n, int64_t lda, int64_t maxrank,
                       double reltol, double abstol, int leftorth, int64_t* rowidx, int64_t* colidx,
                       double* pivoterrs, double* left, double* right, int64_t* npivot) {
    if (!c || !npivot) return TCI_ERR_ARG;
    if (m < 0 || n < 0 || lda < m || (lda & 1) || ((uintptr_t)d_A & 15))
        return set_err(c, TCI_ERR_ARG, "luci: need lda >= m, lda even and a 16-byte aligned matrix");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int64_t np;
    double err;
    int st;
    if ((st = rrlu_device(c, d_A, m, n, lda, maxrank, reltol, abstol, leftorth, &np, &err))) return st;
    *npivot = np;
    return luci_outputs(c, m, n, leftorth, np, err, rowidx, colidx, pivoterrs, left, right);
}

// The 2-site update of a small Pi (rrlu_small_fits) with one host synchronisation and no
// device-to-host copies: index tables up by one copy from mapped host memory, Pi + maxabs, then
// one workgroup doing rrLU, NaN checks and the MatrixLUCI factors from LDS and writing every
// result straight into the mapped host buffer.
static int update_pivots_small(tci_ctx* c, const tci_func* f, const int32_t* rows, int64_t m,
                               int32_t nl, const int32_t* cols, int64_t n, int32_t nr,
                               int64_t maxrank, double reltol, double abstol, int leftorth,
                               int want_factors, int64_t* rowidx, int64_t* colidx,
                               double* pivoterrs, int64_t* npivot, double* maxabs, double* left,
                               double* right) {
    const int64_t mr = std::min<int64_t>(maxrank, std::min(m, n));
    const int64_t ld = round_up(m, 16);
    const bool wl = want_factors && left, wr = want_factors && right;
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(ld * n)))) return st;
    if ((st = ensure(c, &c->dI, &c->capI, (size_t)(m * nl + n * nr + 8)))) return st;
    // mapped host buffer: rows | cols (uploaded by one copy) | state | flag | maxbits |
    // rowphys[m] | colphys[n] | pivv[mr] | left[m * mr] | right[mr * n] (written by the kernel)
    size_t off[10];
    off[0] = 0;
    off[1] = off[0] + (size_t)round_up((m * nl + n * nr) * 4, 16);
    off[2] = off[1] + (size_t)round_up(sizeof(RrluState), 16);
    off[3] = off[2] + 16;
    off[4] = off[3] + 16;
    off[5] = off[4] + (size_t)round_up(m * 8, 16);
    off[6] = off[5] + (size_t)round_up(n * 8, 16);
    off[7] = off[6] + (size_t)round_up(mr * 8, 16);
    off[8] = off[7] + (wl ? (size_t)(m * mr * 8) : 0);
    off[9] = off[8] + (wr ? (size_t)(mr * n * 8) : 0);
    if ((st = ensure_mapped(c, off[9]))) return st;
    char* h = c->zbuf;
    char* d = c->zdev;
    const size_t bi = (size_t)(m * nl) * 4, bj = (size_t)(n * nr) * 4;
    if (bi) memcpy(h, rows, bi);
    if (bj) memcpy(h + bi, cols, bj);
    if (bi + bj) HIPCHK(c, hipMemcpyAsync(c->dI, d, bi + bj, hipMemcpyHostToDevice, c->stream));
    if ((st = batcheval_launch(c, f, c->dI, m, nl, c->dI + m * nl, n, nr, 0, c->dA, ld))) return st;
    c->ldUp = std::max<int64_t>(mr, 1);
    tci::SmallOut out{wl ? reinterpret_cast<double*>(d + off[7]) : nullptr,
                      wr ? reinterpret_cast<double*>(d + off[8]) : nullptr,
                      reinterpret_cast<int*>(d + off[2]), c->maxbits,
                      reinterpret_cast<unsigned long long*>(d + off[3])};
    HIPCHK(c, tci::launch_rrlu_small(c->stream, c->dA, ld, (int)m, (int)n, (int)mr, reltol, abstol,
                                     leftorth, reinterpret_cast<RrluState*>(d + off[1]),
                                     reinterpret_cast<int64_t*>(d + off[4]),
                                     reinterpret_cast<int64_t*>(d + off[5]),
                                     reinterpret_cast<double*>(d + off[6]), nullptr, m, nullptr,
                                     c->ldUp, out));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const RrluState* hs = reinterpret_cast<const RrluState*>(h + off[1]);
    const int64_t np = hs->np;
    const double err = np >= std::min(m, n) ? 0.0 : hs->error;  // matrixlu.jl:391-393
    if (maxabs) memcpy(maxabs, h + off[3], sizeof(double));
    *npivot = np;
    const int fl = *reinterpret_cast<const int*>(h + off[2]);
    if (fl & 1) return set_err(c, TCI_ERR_NAN, "lu.L contains NaNs");
    if (fl & 2) return set_err(c, TCI_ERR_NAN, "lu.U contains NaNs");
    const int64_t* rp = reinterpret_cast<const int64_t*>(h + off[4]);
    const int64_t* cp = reinterpret_cast<const int64_t*>(h + off[5]);
    const double* pv = reinterpret_cast<const double*>(h + off[6]);
    for (int64_t t = 0; t < np; ++t) {
        if (rowidx) rowidx[t] = rp[t] + 1;
        if (colidx) colidx[t] = cp[t] + 1;
        if (pivoterrs) pivoterrs[t] = std::fabs(pv[t]);
    }
    if (pivoterrs) pivoterrs[np] = err;
    if (wl && np > 0) memcpy(left, h + off[7], (size_t)(m * np * 8));
    if (wr && np > 0) memcpy(right, h + off[8], (size_t)(np * n * 8));
    return TCI_OK;
}

int tci_update_pivots_h(tci_ctx* c, const tci_func* f, const int32_t* rows, int64_t m, int32_t nl,
                        const int32_t* cols, int64_t n, int32_t nr, int64_t maxrank, double reltol,
                        double abstol, int leftorth, int want_factors, int64_t* rowidx,
                        int64_t* colidx, double* pivoterrs, int64_t* npivot, double* maxabs,
                        double* left, double* right) {
    if (!c || !f || !npivot) return TCI_ERR_ARG;
    if (nl + nr != f->L) return set_err(c, TCI_ERR_ARG, "rows/cols widths must add up to L");
    if (c->small_path && tci::rrlu_small_fits(m, n) && maxrank > 0)
        return update_pivots_small(c, f, rows, m, nl, cols, n, nr, maxrank, reltol, abstol, leftorth,
                                   want_factors, rowidx, colidx, pivoterrs, npivot, maxabs, left,
                                   right);
    const int64_t ld = round_up(std::max<int64_t>(m, 1), 16);
    int st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(ld * std::max<int64_t>(n, 1))))) return st;
    if ((st = upload_index(c, &c->dI, &c->capI, rows, m, nl))) return st;
    if ((st = upload_index(c, &c->dJ, &c->capJ, cols, n, nr))) return st;
    if ((st = batcheval_device(c, f, c->dI, m, nl, c->dJ, n, nr, 0, c->dA, ld, maxabs))) return st;
    int64_t np;
    double err;
    if ((st = rrlu_device(c, c->dA, m, n, ld, maxrank, reltol, abstol, leftorth, &np, &err)))
        return st;
    *npivot = np;
    return luci_outputs(c, m, n, leftorth, np, err, rowidx, colidx, pivoterrs,
                        want_factors ? left : nullptr, want_factors ? right : nullptr);
}


// setsitetensor!'s solve on device buffers (piv: c->dPiv, 2 r + 2 ints). The cooperative getrf
// (tci_dense.hip k_getrf_coop) needs its workgroups co-resident; if one of them waited past its
// timeout (another stream or process holding the CUs) every workgroup left and the fault word is
// set: the solve is then redone from a copy of P on the launch-per-panel path. The getrs is launched
// only after the word is read (a getrf that gave up leaves no permutation for it to gather by): one
// host synchronisation more per cooperative solve, ~10 us against ms of solve.
extern "C++" {  // (this file's ABI block is extern "C")
namespace tci {
void launch_sitetensor_solve_parts(hipStream_t s, double* P, int r, double* Pi1, int R, double* T, int* piv,
                                   int dense, int parts);
}
}

static int solve_launch(tci_ctx* c, double* P, int64_t r, double* Pi1, int64_t R, double* T) {
    const int coopmask = tci::kDenseGetrf | tci::kDenseGetrfReg | tci::kDenseGetrfCoop;
    const bool coop = (c->dense & coopmask) == coopmask && tci::getrf_coop_fits((int)r);
    int st;
    if (coop) {
        if ((st = ensure(c, &c->dPbak, &c->capPbak, (size_t)(r * r)))) return st;
        if (!c->hCoop) HIPCHK(c, hipHostMalloc((void**)&c->hCoop, 64, hipHostMallocDefault));
        HIPCHK(c, hipMemcpyAsync(c->dPbak, P, (size_t)(r * r) * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    }
    if (!coop) {
        tci::launch_sitetensor_solve(c->stream, P, (int)r, Pi1, (int)R, T, c->dPiv, c->dense);
        HIPCHK(c, hipGetLastError());
        return TCI_OK;
    }
    tci::launch_sitetensor_solve_parts(c->stream, P, (int)r, Pi1, (int)R, T, c->dPiv, c->dense, 1);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(c->hCoop, c->dPiv + 2 * r + 1, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (*c->hCoop == 0) {  // the permutation is in place: the getrs
        tci::launch_sitetensor_solve_parts(c->stream, P, (int)r, Pi1, (int)R, T, c->dPiv, c->dense, 2);
        HIPCHK(c, hipGetLastError());
        return TCI_OK;
    }
    ++c->coop_faults;
    HIPCHK(c, hipMemcpyAsync(P, c->dPbak, (size_t)(r * r) * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
    tci::launch_sitetensor_solve(c->stream, P, (int)r, Pi1, (int)R, T, c->dPiv, c->dense & ~tci::kDenseGetrfCoop);
    HIPCHK(c, hipGetLastError());
    return TCI_OK;
}

int tci_sitetensor_h(tci_ctx* c, const tci_func* f, const int32_t* Ib, int64_t nIb, int32_t wI,
                     const int32_t* Jb, int64_t nJb, int32_t wJ, const int32_t* Inext,
                     int64_t nInext, double* T, double* maxabs) {
    if (!c || !f || !T) return TCI_ERR_ARG;
    if (wI + 1 + wJ != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    const int64_t d = f->localdims[wI];
    const int64_t R = nIb * d;
    const int64_t ldR = std::max<int64_t>(R, 1);
    if (Inext && nInext != nJb) return set_err(c, TCI_ERR_NONSQ, "Pivot matrix is not square!");
    const int64_t r = nJb;
    int st;
    if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(ldR * std::max<int64_t>(nJb, 1))))) return st;
    if ((st = ensure(c, &c->dI, &c->capI, (size_t)std::max<int64_t>(nIb * wI, 1)))) return st;
    if ((st = ensure(c, &c->dJ, &c->capJ, (size_t)std::max<int64_t>(nJb * wJ, 1)))) return st;
    // index tables up through one pinned stage: Ib | Jb | Inext
    const size_t bi = (size_t)(nIb * wI) * 4, bj = (size_t)(nJb * wJ) * 4;
    const size_t bn = Inext ? (size_t)(nInext * (wI + 1)) * 4 : 0;
    if ((st = ensure_pinned(c, &c->hin, &c->capHin, bi + bj + bn + 16))) return st;
    if (bi) memcpy(c->hin, Ib, bi);
    if (bj) memcpy(c->hin + bi, Jb, bj);
    if (bn) memcpy(c->hin + bi + bj, Inext, bn);
    if (bi) HIPCHK(c, hipMemcpyAsync(c->dI, c->hin, bi, hipMemcpyHostToDevice, c->stream));
    if (bj) HIPCHK(c, hipMemcpyAsync(c->dJ, c->hin + bi, bj, hipMemcpyHostToDevice, c->stream));
    const bool solve = Inext && r > 0 && R > 0;
    if (solve) {
        // P = f(Inext x Jb) (r x r) into dF2 first: maxabs is Pi1's alone (updatemaxsample!(tci,
        // Pi1), tensorci2.jl:609), and each evaluation resets c->maxbits
        if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(r * r)))) return st;
        if ((st = ensure(c, &c->dA, &c->capA, (size_t)(R * r)))) return st;
        if ((st = ensure(c, &c->dPiv, &c->capPiv, (size_t)(2 * r + 2)))) return st;
        if ((st = ensure(c, &c->dI2, &c->capI2, (size_t)std::max<int64_t>(nInext * (wI + 1), 1))))
            return st;
        if (bn)
            HIPCHK(c, hipMemcpyAsync(c->dI2, c->hin + bi + bj, bn, hipMemcpyHostToDevice, c->stream));
        if ((st = batcheval_launch(c, f, c->dI2, nInext, wI + 1, c->dJ, nJb, wJ, 0, c->dF2, r)))
            return st;
    }
    if ((st = batcheval_launch(c, f, c->dI, nIb, wI, c->dJ, nJb, wJ, 1, c->dF1, ldR))) return st;
    if (solve) {
        ev_begin(c, 20);
        if ((st = solve_launch(c, c->dF2, r, c->dF1, R, c->dA))) return st;
        ev_end(c);
    }
    // maxabs through the pinned stage, T by d2h_large (chunked through pinned slots, host copy threaded)
    const size_t bt = (size_t)(R * nJb) * 8;
    if ((st = ensure_pinned(c, &c->hout, &c->capHout, 16))) return st;
    HIPCHK(c, hipMemcpyAsync(c->hout, c->maxbits, 8, hipMemcpyDeviceToHost, c->stream));
    if (bt && (solve || !Inext)) {
        if ((st = d2h_large(c, T, solve ? c->dA : c->dF1, bt))) return st;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (maxabs) memcpy(maxabs, c->hout, 8);
    return TCI_OK;
}

int tci_sitetensor_solve_h(tci_ctx* c, const double* P, int64_t r, const double* Pi1, int64_t R,
                           double* T) {
    if (!c || (r > 0 && (!P || !T)) || (R > 0 && r > 0 && !Pi1) || r < 0 || R < 0)
        return TCI_ERR_ARG;
    if (r == 0 || R == 0) return TCI_OK;
    if (r > INT32_MAX / 2 || R > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int st;
    if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(r * r)))) return st;
    if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(R * r)))) return st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(R * r)))) return st;
    if ((st = ensure(c, &c->dPiv, &c->capPiv, (size_t)(2 * r + 2)))) return st;
    HIPCHK(c, hipMemcpyAsync(c->dF2, P, r * r * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->dF1, Pi1, R * r * sizeof(double), hipMemcpyHostToDevice, c->stream));
    ev_begin(c, 20);
    if ((st = solve_launch(c, c->dF2, r, c->dF1, R, c->dA))) return st;
    ev_end(c);
    HIPCHK(c, hipMemcpyAsync(T, c->dA, R * r * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_diag_mfma_f64(tci_ctx* c, double* tflops) {
    if (!c || !tflops) return TCI_ERR_ARG;
    int st;
    if ((st = ensure(c, &c->dF2, &c->capF2, 64))) return st;
    const int grid = std::max(c->ncu, 1) * 4, iters = 4096;  // one wave per SIMD
    tci::launch_mfma_f64_probe(c->stream, grid, 64, c->dF2);   // warm
    hipEvent_t e0, e1;
    HIPCHK(c, hipEventCreate(&e0));
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventRecord(e0, c->stream));
    tci::launch_mfma_f64_probe(c->stream, grid, iters, c->dF2);
    HIPCHK(c, hipEventRecord(e1, c->stream));
    HIPCHK(c, hipEventSynchronize(e1));
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    const double flops = (double)grid * 4 /* waves */ * iters * 8 * (16.0 * 16 * 4 * 2);
    *tflops = flops / (ms * 1e-3) / 1e12;
    return TCI_OK;
}

int tci_sitetensor_solve_d(tci_ctx* c, double* d_P, int64_t r, const double* d_Pi1, int64_t R,
                           double* d_T) {
    if (!c || r < 0 || R < 0 || (r > 0 && R > 0 && (!d_P || !d_Pi1 || !d_T))) return TCI_ERR_ARG;
    if (r == 0 || R == 0) return TCI_OK;
    if (r > INT32_MAX / 2 || R > INT32_MAX / 2 || r * R > INT32_MAX * 64LL)
        return set_err(c, TCI_ERR_ARG, "matrix too large");
    int st;
    if ((st = ensure(c, &c->dPiv, &c->capPiv, (size_t)(2 * r + 2)))) return st;
    ev_begin(c, 20);
    if ((st = solve_launch(c, d_P, r, const_cast<double*>(d_Pi1), R, d_T))) return st;
    ev_end(c);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_dgemm_d(tci_ctx* c, int transb, int64_t m, int64_t n, int64_t k, double alpha,
                const double* d_A, int64_t lda, const double* d_B, int64_t ldb, double beta,
                double* d_C, int64_t ldc) {
    if (!c || m < 0 || n < 0 || k < 0) return TCI_ERR_ARG;
    if (m == 0 || n == 0) return TCI_OK;
    if (!d_C || (k > 0 && (!d_A || !d_B)) || lda < std::max<int64_t>(m, 1) ||
        ldb < std::max<int64_t>(transb ? n : k, 1) || ldc < m)
        return set_err(c, TCI_ERR_ARG, "dgemm: bad pointer or leading dimension");
    if (m > INT32_MAX || n > INT32_MAX || k > INT32_MAX) return set_err(c, TCI_ERR_ARG, "matrix too large");
    ev_begin(c, 22);
    tci::launch_dgemm(c->stream, transb != 0, (int)m, (int)n, (int)k, alpha, d_A, lda, d_B, ldb, beta, d_C,
                      ldc, d_C, ldc, nullptr, nullptr);
    ev_end(c);
    HIPCHK(c, hipGetLastError());
    return TCI_OK;
}

int tci_schur_update_d(tci_ctx* c, double* d_C, int64_t m, int64_t n, int64_t ldc,
                       const double* d_W, int64_t ldw, const double* d_V, int64_t ldv, int64_t k) {
    return tci_dgemm_d(c, 0, m, n, k, -1.0, d_W, ldw, d_V, ldv, 1.0, d_C, ldc);
}

int tci_diag_mfma_f64_ex(tci_ctx* c, int waves_per_simd, double* tflops, double* ghz) {
    if (!c || !tflops || waves_per_simd < 1 || waves_per_simd > 4) return TCI_ERR_ARG;
    const int w = waves_per_simd == 3 ? 2 : waves_per_simd;
    const int grid = std::max(c->ncu, 1), iters = 2048;
    int st;
    if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(64 + grid)))) return st;
    long long* cyc = reinterpret_cast<long long*>(c->dF2 + 64);
    tci::launch_mfma_probe2(c->stream, w, grid, 64, c->dF2, cyc);  // warm
    hipEvent_t e0, e1;
    HIPCHK(c, hipEventCreate(&e0));
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipEventRecord(e0, c->stream));
    tci::launch_mfma_probe2(c->stream, w, grid, iters, c->dF2, cyc);
    HIPCHK(c, hipEventRecord(e1, c->stream));
    HIPCHK(c, hipEventSynchronize(e1));
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    std::vector<long long> h(grid);
    HIPCHK(c, hipMemcpy(h.data(), cyc, grid * sizeof(long long), hipMemcpyDeviceToHost));
    double mean = 0;
    for (long long v : h) mean += (double)v;
    mean /= grid;
    const double flops = (double)grid * 4 * w * iters * 8 * (16.0 * 16 * 4 * 2);
    *tflops = flops / (ms * 1e-3) / 1e12;
    // clock64 counts shader-clock cycles: cycles of the loop / its wall time ~ the clock held
    if (ghz) *ghz = mean / (ms * 1e-3) / 1e9;
    return TCI_OK;
}

int tci_tt_evaluate_h(tci_ctx* c, int32_t L, const int32_t* dims, const int32_t* bonddims,
                      const double* cores, int64_t ncore, const int32_t* X, int64_t npts, double* out) {
    if (!c || L < 1 || !dims || !bonddims || !cores || (npts > 0 && (!X || !out)))
        return TCI_ERR_ARG;
    if (bonddims[0] != 1 || bonddims[L] != 1)
        return set_err(c, TCI_ERR_ARG, "tt: the first and last bond dimensions must be 1");
    std::vector<int64_t> off(L + 1, 0);
    int rmax = 1;
    for (int t = 0; t < L; ++t) {
        off[t + 1] = off[t] + (int64_t)bonddims[t] * dims[t] * bonddims[t + 1];
        rmax = std::max(rmax, (int)bonddims[t + 1]);
    }
    if (off[L] > ncore) return set_err(c, TCI_ERR_ARG, "tt: core buffer smaller than the bond dimensions imply");
    if (rmax > 1024) return set_err(c, TCI_ERR_ARG, "tt: bond dimension above 1024");
    if (npts == 0) return TCI_OK;
    // one device block: cores | X | dims, bonddims | offsets | out
    const size_t bc = (size_t)off[L] * 8, bx = (size_t)(npts * L) * 4, bm = (size_t)(2 * L + 1) * 4,
                 bo = (size_t)(L + 1) * 8, bout = (size_t)npts * 8;
    const size_t o1 = round_up(bc, 16), o2 = o1 + round_up(bx, 16), o3 = o2 + round_up(bm, 16),
                 o4 = o3 + round_up(bo, 16), total = o4 + bout;
    int st;
    if ((st = ensure(c, (char**)&c->scratch2, &c->capScratch2, total))) return st;
    if ((st = ensure_pinned(c, &c->hin, &c->capHin, o4))) return st;
    memcpy(c->hin, cores, bc);
    memcpy(c->hin + o1, X, bx);
    memcpy(c->hin + o2, dims, (size_t)L * 4);
    memcpy(c->hin + o2 + (size_t)L * 4, bonddims, (size_t)(L + 1) * 4);
    memcpy(c->hin + o3, off.data(), bo);
    char* d = c->scratch2;
    HIPCHK(c, hipMemcpyAsync(d, c->hin, o4, hipMemcpyHostToDevice, c->stream));
    tci::launch_tt_eval(c->stream, reinterpret_cast<const double*>(d), reinterpret_cast<const int64_t*>(d + o3),
                        reinterpret_cast<const int32_t*>(d + o2 + (size_t)L * 4),
                        reinterpret_cast<const int32_t*>(d + o2), L, reinterpret_cast<const int32_t*>(d + o1),
                        (int)npts, reinterpret_cast<double*>(d + o4), rmax);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out, d + o4, bout, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_tt_evaluate_c128_h(tci_ctx* c, int32_t L, const int32_t* dims, const int32_t* bonddims,
                           const double* cores, int64_t ncore, const int32_t* X, int64_t npts,
                           double* out) {
    if (!c || L < 1 || !dims || !bonddims || !cores || (npts > 0 && (!X || !out)))
        return TCI_ERR_ARG;
    if (bonddims[0] != 1 || bonddims[L] != 1)
        return set_err(c, TCI_ERR_ARG, "tt: the first and last bond dimensions must be 1");
    std::vector<int64_t> off(L + 1, 0);
    int rmax = 1;
    for (int t = 0; t < L; ++t) {
        off[t + 1] = off[t] + (int64_t)bonddims[t] * dims[t] * bonddims[t + 1];
        rmax = std::max(rmax, (int)bonddims[t + 1]);
    }
    if (off[L] > ncore) return set_err(c, TCI_ERR_ARG, "tt: core buffer smaller than the bond dimensions imply");
    if (rmax > 1024) return set_err(c, TCI_ERR_ARG, "tt: bond dimension above 1024");
    for (int64_t e = 0; e < npts * L; ++e)
        if (X[e] < 1 || X[e] > dims[e % L]) return set_err(c, TCI_ERR_ARG, "tt: index out of range");
    if (npts == 0) return TCI_OK;
    if (npts > INT32_MAX) return set_err(c, TCI_ERR_ARG, "tt: too many points");
    const size_t bc = (size_t)off[L] * 16, bx = (size_t)(npts * L) * 4, bm = (size_t)(2 * L + 1) * 4,
                 bo = (size_t)(L + 1) * 8, bout = (size_t)npts * 16;
    const size_t o1 = round_up(bc, 16), o2 = o1 + round_up(bx, 16), o3 = o2 + round_up(bm, 16),
                 o4 = o3 + round_up(bo, 16), total = o4 + bout;
    int st;
    if ((st = ensure(c, (char**)&c->scratch2, &c->capScratch2, total))) return st;
    if ((st = ensure_pinned(c, &c->hin, &c->capHin, o4))) return st;
    memcpy(c->hin, cores, bc);
    memcpy(c->hin + o1, X, bx);
    memcpy(c->hin + o2, dims, (size_t)L * 4);
    memcpy(c->hin + o2 + (size_t)L * 4, bonddims, (size_t)(L + 1) * 4);
    memcpy(c->hin + o3, off.data(), bo);
    char* d = c->scratch2;
    HIPCHK(c, hipMemcpyAsync(d, c->hin, o4, hipMemcpyHostToDevice, c->stream));
    tci::launch_ctt_eval(c->stream, reinterpret_cast<const double2*>(d),
                         reinterpret_cast<const int64_t*>(d + o3),
                         reinterpret_cast<const int32_t*>(d + o2 + (size_t)L * 4),
                         reinterpret_cast<const int32_t*>(d + o2), L,
                         reinterpret_cast<const int32_t*>(d + o1), (int)npts,
                         reinterpret_cast<double2*>(d + o4));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(out, d + o4, bout, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_sitetensor_solve_c128_h(tci_ctx* c, const double* P, int64_t r, const double* Pi1,
                                int64_t R, double* T) {
    if (!c || (r > 0 && (!P || !T)) || (R > 0 && r > 0 && !Pi1) || r < 0 || R < 0)
        return TCI_ERR_ARG;
    if (r == 0 || R == 0) return TCI_OK;
    if (r > 8192 || R > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int st;
    if ((st = ensure(c, &c->dF2, &c->capF2, (size_t)(2 * r * r)))) return st;
    if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(2 * R * r)))) return st;
    if ((st = ensure(c, &c->dA, &c->capA, (size_t)(2 * (R * r + r * r))))) return st;
    if ((st = ensure(c, &c->dPiv, &c->capPiv, (size_t)(2 * r + 2)))) return st;
    HIPCHK(c, hipMemcpyAsync(c->dF2, P, r * r * 16, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->dF1, Pi1, R * r * 16, hipMemcpyHostToDevice, c->stream));
    double2* dT = reinterpret_cast<double2*>(c->dA);
    double2* work = dT + R * r;
    tci::launch_csitetensor_solve(c->stream, reinterpret_cast<const double2*>(c->dF2), (int)r,
                                  reinterpret_cast<const double2*>(c->dF1), (int)R, dT, work,
                                  c->dPiv);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(T, dT, R * r * 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_fill_uniform_d(tci_ctx* c, double* d_A, int64_t m, int64_t n, int64_t lda, uint64_t seed) {
    if (!c || lda < m) return TCI_ERR_ARG;
    tci::launch_fill_uniform(c->stream, d_A, m, n, lda, seed);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_fill_uniform_block_d(tci_ctx* c, double* d_A, int64_t m, int64_t n, int64_t lda, uint64_t seed,
                             uint64_t offset) {
    if (!c || lda < m) return TCI_ERR_ARG;
    tci::launch_fill_uniform(c->stream, d_A, m, n, lda, seed, offset);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_diag_stream_d(tci_ctx* c, const double* d_a, double* d_b, int64_t n, int reps, int grid,
                      double* ms_read, double* ms_copy) {
    if (!c || !d_a || n < 2 || reps < 1) return TCI_ERR_ARG;
    hipEvent_t e0, e1;
    HIPCHK(c, hipEventCreate(&e0));
    HIPCHK(c, hipEventCreate(&e1));
    HIPCHK(c, hipMemsetAsync(c->maxbits, 0, sizeof(unsigned long long), c->stream));
    tci::launch_stream_read(c->stream, d_a, n, c->maxbits, grid);  // warm
    float ms = 0;
    HIPCHK(c, hipEventRecord(e0, c->stream));
    for (int r = 0; r < reps; ++r) tci::launch_stream_read(c->stream, d_a, n, c->maxbits, grid);
    HIPCHK(c, hipEventRecord(e1, c->stream));
    HIPCHK(c, hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
    if (ms_read) *ms_read = ms / reps;
    if (d_b && ms_copy) {
        tci::launch_stream_copy(c->stream, d_a, d_b, n, grid);
        HIPCHK(c, hipEventRecord(e0, c->stream));
        for (int r = 0; r < reps; ++r) tci::launch_stream_copy(c->stream, d_a, d_b, n, grid);
        HIPCHK(c, hipEventRecord(e1, c->stream));
        HIPCHK(c, hipEventSynchronize(e1));
        hipEventElapsedTime(&ms, e0, e1);
        *ms_copy = ms / reps;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return TCI_OK;
}

int tci_malloc_d(tci_ctx* c, void** p, int64_t bytes) {
    if (hipMalloc(p, (size_t)std::max<int64_t>(bytes, 16)) != hipSuccess)
        return set_err(c, TCI_ERR_NOMEM, "hipMalloc failed");
    return TCI_OK;
}
int tci_free_d(tci_ctx* c, void* p) {
    if (p) HIPCHK(c, hipFree(p));
    return TCI_OK;
}
int tci_memcpy_h2d(tci_ctx* c, void* dst, const void* src, int64_t bytes) {
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}
int tci_memset_d(tci_ctx* c, void* dst, int value, int64_t bytes) {
    if (!c || (bytes > 0 && !dst) || bytes < 0) return TCI_ERR_ARG;
    if (bytes > 0) HIPCHK(c, hipMemsetAsync(dst, value, (size_t)bytes, c->stream));
    return TCI_OK;
}
int tci_memcpy_d2h(tci_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c || bytes < 0 || (bytes > 0 && (!dst || !src))) return TCI_ERR_ARG;
    if (bytes == 0) return TCI_OK;
    return d2h_large(c, dst, src, (size_t)bytes);  // (synchronous; chunked through pinned slots when large)
}
int tci_memcpy_d2d(tci_ctx* c, void* dst, const void* src, int64_t bytes) {
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_memcpy2d_d2d(tci_ctx* c, void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                     int64_t height) {
    if (!c || width < 0 || height < 0 || dpitch < width || spitch < width) return TCI_ERR_ARG;
    if (width == 0 || height == 0) return TCI_OK;
    HIPCHK(c, hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)height,
                               hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

}  // extern "C"

extern "C" {

int tci_comm_unique_id(void* id, int64_t* nbytes) {
    if (nbytes) *nbytes = NCCL_UNIQUE_ID_BYTES;
    if (!id) return nbytes ? TCI_OK : TCI_ERR_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return TCI_ERR_DEVICE;
    memcpy(id, &u, sizeof u);
    return TCI_OK;
}

int tci_comm_create(tci_ctx* c, int nranks, int rank, const void* id, tci_comm** out) {
    if (!c || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return TCI_ERR_ARG;
    *out = nullptr;
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    tci_comm* cm = new tci_comm();
    cm->ctx = c;
    cm->nranks = nranks;
    cm->rank = rank;
    const ncclResult_t r = ncclCommInitRank(&cm->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        delete cm;
        return set_err(c, TCI_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = cm;
    return TCI_OK;
}

int tci_comm_destroy(tci_comm* cm) {
    if (!cm) return TCI_OK;
    if (cm->ctx && cm->ctx->stream) hipStreamSynchronize(cm->ctx->stream);
    if (cm->nc) ncclCommDestroy(cm->nc);
    delete cm;
    return TCI_OK;
}

int tci_comm_allgather_d(tci_comm* cm, const void* d_send, void* d_recv, int64_t bytes) {
    if (!cm || bytes < 0 || (bytes > 0 && (!d_send || !d_recv))) return TCI_ERR_ARG;
    tci_ctx* c = cm->ctx;
    if (bytes == 0) return TCI_OK;
    const ncclResult_t r = ncclAllGather(d_send, d_recv, (size_t)bytes, ncclUint8, cm->nc, c->stream);
    if (r != ncclSuccess) return set_err(c, TCI_ERR_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    return TCI_OK;
}

int tci_comm_allreduce_max_u64_d(tci_comm* cm, void* d_buf, int64_t count) {
    if (!cm || count < 0 || (count > 0 && !d_buf)) return TCI_ERR_ARG;
    tci_ctx* c = cm->ctx;
    if (count == 0) return TCI_OK;
    const ncclResult_t r = ncclAllReduce(d_buf, d_buf, (size_t)count, ncclUint64, ncclMax, cm->nc, c->stream);
    if (r != ncclSuccess) return set_err(c, TCI_ERR_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return TCI_OK;
}

int tci_rrlu_sharded_d(tci_ctx* c, tci_comm* comm, tci_exchange_fn exch, void* user, int nranks, double* d_A,
                       int64_t m, int64_t nloc, int64_t lda, int64_t c0, int64_t n, int64_t maxrank,
                       double reltol, double abstol, int leftorth, int64_t* rowperm, int64_t* colperm,
                       int64_t* npivot, double* lasterror, double* pivoterrors) {
    if (!c || !npivot || !lasterror || m < 0 || nloc < 0 || n < 0 || c0 < 0 || c0 + nloc > n || nranks < 1)
        return TCI_ERR_ARG;
    if (comm && comm->nranks != nranks) return set_err(c, TCI_ERR_ARG, "rrlu_sharded: nranks != comm size");
    if (m > 0 && (!d_A || lda < m || lda % 2)) return set_err(c, TCI_ERR_ARG, "rrlu_sharded: bad matrix / lda");
    if (m > INT32_MAX / 2 || n > INT32_MAX / 2) return set_err(c, TCI_ERR_ARG, "matrix too large");
    int64_t np;
    double err;
    int st = rrlu_sharded_device(c, comm, exch, user, nranks, d_A, m, nloc, lda, c0, n, maxrank, reltol, abstol,
                                 leftorth, &np, &err);
    if (st) return st;
    c->sh_np = np;
    c->sh_valid = 1;
    c->sh_nloc = nloc;
    c->sh_c0 = c0;
    c->sh_m = m;
    c->sh_n = n;
    c->sh_leftorth = leftorth;
    *npivot = np;
    *lasterror = err;
    if ((st = pivot_errors(c, np, err, pivoterrors))) return st;
    return fetch_perms(c, rowperm, colperm, rowperm ? m : 0, colperm ? n : 0);
}

int tci_rrlu_sharded_factors_h(tci_ctx* c, double* L, double* U, int64_t ldu) {
    if (!c) return TCI_ERR_ARG;
    if (!c->sh_valid)
        return set_err(c, TCI_ERR_ARG, "rrlu_sharded_factors: no current tci_rrlu_sharded_d result on this "
                                        "context (another factorisation ran since)");
    const int64_t m = c->sh_m, n = c->sh_n, np = c->sh_np;
    if (np <= 0) return TCI_OK;
    if (U && ldu < np) return set_err(c, TCI_ERR_ARG, "ldu < npivot");
    int st;
    if ((st = ensure(c, &c->dL, &c->capL, (size_t)(m * np)))) return st;
    if ((st = ensure(c, &c->dU, &c->capU, (size_t)(np * n)))) return st;
    if (U) HIPCHK(c, hipMemcpy2DAsync(c->dU, np * sizeof(double), U, ldu * sizeof(double), np * sizeof(double), n,
                                      hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->flag, 0, sizeof(int), c->stream));
    tci::launch_extract_shard(c->stream, c->Lp, m, c->Up, c->ldUp, c->pivv, c->rowperm, c->colperm, (int)m, (int)n,
                              (int)np, c->sh_leftorth, L ? c->dL : nullptr, m, U ? c->dU : nullptr, np, c->flag,
                              c->sh_c0, (int)c->sh_nloc);
    HIPCHK(c, hipMemcpyAsync(c->hflag, c->flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (L) HIPCHK(c, hipMemcpyAsync(L, c->dL, m * np * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (U) HIPCHK(c, hipMemcpy2DAsync(U, ldu * sizeof(double), c->dU, np * sizeof(double), np * sizeof(double), n,
                                      hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (*c->hflag & 1) return set_err(c, TCI_ERR_NAN, "lu.L contains NaNs");
    if (*c->hflag & 2) return set_err(c, TCI_ERR_NAN, "lu.U contains NaNs");
    return TCI_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ CachedFunction device memo
namespace {

int cache_alloc_table(tci_cache* h, int64_t cap) {
    tci_ctx* c = h->ctx;
    unsigned long long* k = nullptr;
    double* v = nullptr;
    unsigned* st = nullptr;
    if (hipMalloc((void**)&k, cap * 8) != hipSuccess || hipMalloc((void**)&v, cap * 8) != hipSuccess ||
        hipMalloc((void**)&st, cap * 4) != hipSuccess) {
        if (k) hipFree(k);
        if (v) hipFree(v);
        return set_err(c, TCI_ERR_NOMEM, "cache: table allocation failed");
    }
    HIPCHK(c, hipMemsetAsync(k, 0xff, cap * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(st, 0, cap * 4, c->stream));
    if (h->keys) {  // rehash the ready entries
        tci::launch_cache_rehash(c->stream, h->keys, h->vals, h->cap, k, v, st, cap);
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hipFree(h->keys);
        hipFree(h->vals);
        hipFree(h->state);
    }
    h->keys = k;
    h->vals = v;
    h->state = st;
    h->cap = cap;
    return TCI_OK;
}

}  // namespace

extern "C" {

int tci_cache_create(tci_ctx* c, const int32_t* localdims, int32_t L, int64_t capacity, tci_cache** out) {
    if (!c || !out || L <= 0 || !localdims) return TCI_ERR_ARG;
    *out = nullptr;
    double log2space = 0;
    for (int t = 0; t < L; ++t) {
        if (localdims[t] <= 0) return set_err(c, TCI_ERR_ARG, "cache: localdims must be positive");
        log2space += std::log2((double)localdims[t]);
    }
    if (log2space >= 62.5) return set_err(c, TCI_ERR_ARG, "cache: index space beyond 2^62 keys (use a host cache)");
    tci_cache* h = new tci_cache();
    h->ctx = c;
    h->L = L;
    h->coeffs.assign(L, 1);
    for (int t = 1; t < L; ++t) h->coeffs[t] = h->coeffs[t - 1] * localdims[t - 1];
    int64_t cap = 1024;
    while (cap < 2 * capacity) cap <<= 1;
    int st;
    if (hipMalloc((void**)&h->dcoeff, L * 8) != hipSuccess || hipMalloc((void**)&h->counts, 24) != hipSuccess ||
        hipHostMalloc((void**)&h->hcounts, 24, 0) != hipSuccess) {
        tci_cache_destroy(h);
        return TCI_ERR_NOMEM;
    }
    if (hipMemcpy(h->dcoeff, h->coeffs.data(), L * 8, hipMemcpyHostToDevice) != hipSuccess ||
        (st = cache_alloc_table(h, cap))) {
        tci_cache_destroy(h);
        return TCI_ERR_DEVICE;
    }
    *out = h;
    return TCI_OK;
}

int tci_cache_destroy(tci_cache* h) {
    if (!h) return TCI_OK;
    if (h->ctx && h->ctx->stream) hipStreamSynchronize(h->ctx->stream);
    for (void* p : {(void*)h->dcoeff, (void*)h->keys, (void*)h->vals, (void*)h->state, (void*)h->kI, (void*)h->kJ,
                    (void*)h->miss, (void*)h->dup, (void*)h->X, (void*)h->mv, (void*)h->counts})
        if (p) hipFree(p);
    if (h->hcounts) hipHostFree(h->hcounts);
    delete h;
    return TCI_OK;
}

int tci_cache_clear(tci_cache* h) {
    if (!h) return TCI_ERR_ARG;
    tci_ctx* c = h->ctx;
    HIPCHK(c, hipMemsetAsync(h->keys, 0xff, h->cap * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(h->state, 0, h->cap * 4, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    h->size = 0;
    return TCI_OK;
}

int tci_cache_size(tci_cache* h, int64_t* n) {
    if (!h || !n) return TCI_ERR_ARG;
    *n = h->size;
    return TCI_OK;
}

int tci_cache_dump_h(tci_cache* h, int64_t* keys, double* vals, int64_t capacity, int64_t* n) {
    if (!h || !n) return TCI_ERR_ARG;
    tci_ctx* c = h->ctx;
    std::vector<unsigned long long> k(h->cap);
    std::vector<double> v(h->cap);
    HIPCHK(c, hipMemcpyAsync(k.data(), h->keys, h->cap * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(v.data(), h->vals, h->cap * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    int64_t q = 0;
    for (int64_t s = 0; s < h->cap; ++s) {
        if (k[s] == ~0ull) continue;
        if (keys && vals && q < capacity) {
            keys[q] = (int64_t)k[s];
            vals[q] = v[s];
        }
        ++q;
    }
    *n = q;
    return TCI_OK;
}

int tci_cache_batcheval_d(tci_ctx* c, tci_cache* h, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                          const int32_t* J, int64_t n, int32_t nr, int32_t M, double* d_out, int64_t ldo,
                          double* maxabs, int64_t* nmiss) {
    if (!c || !h || !f || h->ctx != c || m < 0 || n < 0) return TCI_ERR_ARG;
    if (f->L != h->L) return set_err(c, TCI_ERR_ARG, "cache: the integrand's leg count differs from the cache's");
    if (nl + M + nr != f->L) return set_err(c, TCI_ERR_ARG, "Invalid number of central indices");
    if (M < 0 || M > 1) return set_err(c, TCI_ERR_ARG, "only M = 0 or M = 1 centre legs are supported");
    const int64_t D = M ? f->localdims[nl] : 1, mR = m * D, tot = mR * n;
    if (ldo < mR) return set_err(c, TCI_ERR_ARG, "ldo < m * prod(centre dims)");
    if (nmiss) *nmiss = 0;
    if (maxabs) *maxabs = 0.0;
    if (tot == 0) return TCI_OK;
    int st;
    if ((st = upload_index(c, &c->dI, &c->capI, I, m, nl))) return st;
    if ((st = upload_index(c, &c->dJ, &c->capJ, J, n, nr))) return st;
    if (2 * (h->size + tot) > h->cap) {
        int64_t cap = h->cap;
        while (2 * (h->size + tot) > cap) cap <<= 1;
        if ((st = cache_alloc_table(h, cap))) return st;
    }
    if ((st = ensure(c, &h->kI, &h->capKI, (size_t)m))) return st;
    if ((st = ensure(c, &h->kJ, &h->capKJ, (size_t)n))) return st;
    if ((st = ensure(c, &h->miss, &h->capMiss, (size_t)(2 * tot)))) return st;
    if ((st = ensure(c, &h->dup, &h->capDup, (size_t)tot))) return st;
    tci::launch_cache_partial_keys(c->stream, c->dI, (int)m, nl, h->dcoeff, 0, h->kI);
    tci::launch_cache_partial_keys(c->stream, c->dJ, (int)n, nr, h->dcoeff, f->L - nr, h->kJ);
    HIPCHK(c, hipMemsetAsync(h->counts, 0, 24, c->stream));
    tci::CacheProbeArgs a{h->keys, h->vals, h->state, h->cap, h->kI, h->kJ, M ? h->coeffs[nl] : 0, m, mR, n, d_out,
                          ldo, h->miss, h->dup, h->counts};
    if (m == 0 || nl == 0) HIPCHK(c, hipMemsetAsync(h->kI, 0, 8 * std::max<int64_t>(m, 1), c->stream));
    if (n == 0 || nr == 0) HIPCHK(c, hipMemsetAsync(h->kJ, 0, 8 * std::max<int64_t>(n, 1), c->stream));
    tci::launch_cache_probe(c->stream, a);
    HIPCHK(c, hipMemcpyAsync(h->hcounts, h->counts, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t nm = (int64_t)h->hcounts[0], nd = (int64_t)h->hcounts[1];
    // the probe claimed nm empty slots (state 1); until they are filled a failure must give them
    // back, or later batches would take them for pending values
    auto rollback = [&](int code) {
        const std::string msg = c->err;
        tci::launch_cache_unclaim(c->stream, h->miss, nm, h->keys, h->state);
        hipStreamSynchronize(c->stream);
        c->err = msg;
        return code;
    };
    if (nm > 0) {
        if ((st = ensure(c, &h->X, &h->capX, (size_t)(nm * f->L)))) return rollback(st);
        if ((st = ensure(c, &h->mv, &h->capMv, (size_t)nm))) return rollback(st);
        tci::launch_cache_gather_points(c->stream, h->miss, nm, c->dI, nl, c->dJ, nr, M, m, mR, h->X);
        // the misses as ONE batch evaluation: no left legs, the points as columns
        if ((st = batcheval_launch(c, f, c->dI, 1, 0, h->X, nm, f->L, 0, h->mv, 1))) return rollback(st);
        tci::launch_cache_fill(c->stream, h->miss, nm, h->mv, h->vals, h->state, mR, d_out, ldo);
    }
    tci::launch_cache_dups(c->stream, a, nd);
    HIPCHK(c, hipMemsetAsync(c->maxbits, 0, 8, c->stream));
    tci::launch_cache_maxabs(c->stream, d_out, mR, n, ldo, c->maxbits);
    HIPCHK(c, hipMemcpyAsync(c->hmaxbits, c->maxbits, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(h->hcounts + 2, h->counts + 2, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));
    h->size += nm;
    if (h->hcounts[2]) return set_err(c, TCI_ERR_DEVICE, "cache: a repeated point found no ready value");
    if (nmiss) *nmiss = nm;
    if (maxabs) {
        double v;
        unsigned long long b = *c->hmaxbits;
        memcpy(&v, &b, sizeof v);
        *maxabs = v;
    }
    return TCI_OK;
}

int tci_cache_lookup_h(tci_cache* h, const int32_t* X, int64_t npts, int32_t* found, double* vals) {
    if (!h || npts < 0 || (npts > 0 && (!X || !found || !vals))) return TCI_ERR_ARG;
    if (npts == 0) return TCI_OK;
    tci_ctx* c = h->ctx;
    int st;
    const size_t bx = (size_t)(npts * h->L) * 4;
    if ((st = ensure(c, &h->X, &h->capX, (size_t)(npts * h->L)))) return st;
    if ((st = ensure(c, &h->mv, &h->capMv, (size_t)(2 * npts)))) return st;
    HIPCHK(c, hipMemcpyAsync(h->X, X, bx, hipMemcpyHostToDevice, c->stream));
    int32_t* dfound = reinterpret_cast<int32_t*>(h->mv + npts);
    tci::launch_cache_lookup(c->stream, h->X, npts, h->L, h->dcoeff, h->keys, h->vals, h->state, h->cap, dfound,
                             h->mv);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(vals, h->mv, npts * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(found, dfound, npts * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return TCI_OK;
}

int tci_cache_batcheval_h(tci_ctx* c, tci_cache* h, const tci_func* f, const int32_t* I, int64_t m, int32_t nl,
                          const int32_t* J, int64_t n, int32_t nr, int32_t M, double* out, int64_t ldo,
                          double* maxabs, int64_t* nmiss) {
    if (!c || !f) return TCI_ERR_ARG;
    const int64_t D = (M && nl < f->L) ? f->localdims[nl] : 1, mR = m * D;
    const int64_t ld = round_up(std::max<int64_t>(mR, 1), 2);
    int st;
    if ((st = ensure(c, &c->dF1, &c->capF1, (size_t)(ld * std::max<int64_t>(n, 1))))) return st;
    if ((st = tci_cache_batcheval_d(c, h, f, I, m, nl, J, n, nr, M, c->dF1, ld, maxabs, nmiss))) return st;
    if (out && mR > 0 && n > 0) {
        HIPCHK(c, hipMemcpy2DAsync(out, ldo * sizeof(double), c->dF1, ld * sizeof(double), mR * sizeof(double), n,
                                   hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return TCI_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- device-resident small sweeps
// Called by tci_sweep.cpp (C++ linkage): whether f / L can take the path, one launch of
// k_sweep_small on the SwIO images (tci_internal.h), and the reference's message for a status.
bool tci_sweep_small_ok(tci_ctx* c, const tci_func* f, int L) {
    return c && f && c->small_path && c->small_sweep && L >= 2 && L <= tci::kSwMaxL && !f->hostfn &&
           tci::sweep_small_kind(f->kind);
}

int tci_sweep_small_run(tci_ctx* c, const tci_func* f, int L, int64_t cap, const char* in, size_t inbytes,
                        int mode, int fill, int niter, int iter1, int strategy, int strictlynested, double abstol,
                        int64_t maxbonddim, std::vector<char>& out, const tci::SwSweep1* s1) {
    auto width = [&](int bank, int p) { return (bank & 1) ? L - 1 - p : p; };
    const int64_t tot = 6 * cap * ((int64_t)L * (L - 1) / 2);  // six banks (tci_sweep_small.hip)
    const tci::SwIO io = tci::sw_io(L);
    const size_t outcap = io.sets + (size_t)tot * 4;
    int st;
    if ((st = ensure(c, &c->sw_ws, &c->capSwWs, (size_t)std::max<int64_t>(tot, 1)))) return st;
    if ((st = ensure(c, &c->sw_inbuf, &c->capSwInbuf, inbytes))) return st;
    if ((st = ensure_mapped_pair(c, &c->sw_in, &c->sw_in_d, &c->capSwIn, inbytes))) return st;
    if ((st = ensure_mapped_pair(c, &c->sw_out, &c->sw_out_d, &c->capSwOut, outcap))) return st;
    memcpy(c->sw_in, in, inbytes);
    HIPCHK(c, hipMemcpyAsync(c->sw_inbuf, c->sw_in, inbytes, hipMemcpyHostToDevice, c->stream));
    tci::SweepSmallArgs a;
    a.f = f->view();
    a.L = L;
    a.ws = c->sw_ws;
    a.cap = cap;
    a.inbuf = c->sw_inbuf;
    a.out = c->sw_out_d;
    a.niter = niter;
    a.iter1 = iter1;
    a.strategy = strategy;
    a.strictlynested = strictlynested;
    a.abstol = abstol;
    a.maxbonddim = maxbonddim;
    a.mode = mode;
    a.fill = fill;
    a.s1fwd = s1 ? s1->forward : 0;
    a.s1tens = s1 ? s1->tensors : 0;
    a.reltol = s1 ? s1->reltol : 1e-14;
    a.lu_wave = c->sw_lu_wave;
    a.lazy_union = c->sw_lazy_union;
    a.tens = nullptr;
    a.tcap = 0;
    a.fsolve = mode != 2 && s1 && s1->tensors ? 1 : 0;  // a fill that also solves the site tensors
    if (s1 && s1->tensors) {  // the site tensors in HBM: [site] (offset, count), then the data
        if ((st = ensure(c, &c->sw_tens, &c->capSwTens, (size_t)(2 * L + s1->tcap)))) return st;
        a.tens = c->sw_tens;
        a.tcap = s1->tcap;
    }
    // the fill (mode 0 with fill, mode 1): k_sweep_small checks and maps the sets, then
    // k_fill_sites evaluates every site in parallel (one workgroup per site)
    const bool filling = (mode == 0 && fill) || mode == 1;
    if (filling) {
        if ((st = ensure(c, &c->sw_fmap, &c->capSwFmap, (size_t)(4 * L + 4)))) return st;
        if ((st = ensure_mapped_pair(c, &c->sw_fmax, &c->sw_fmax_d, &c->capSwFmax, (size_t)L * 8))) return st;
        a.fmap = c->sw_fmap;
    }
    HIPCHK(c, tci::launch_sweep_small(c->stream, a));
    if (filling)
        HIPCHK(c, tci::launch_fill_sites(c->stream, a, reinterpret_cast<unsigned long long*>(c->sw_fmax_d)));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int64_t* hdr = reinterpret_cast<const int64_t*>(c->sw_out);
    if (filling && hdr[0] == 0 && hdr[8] == 0) {
        // updatemaxsample! over the sites: max of |Pi1| bits (Julia's NaN-propagating max, order-free
        // on non-negative values) folded into the header's maxsample
        unsigned long long b = (unsigned long long)reinterpret_cast<const int64_t*>(c->sw_out)[6] & 0x7fffffffffffffffull;
        const unsigned long long* fm = reinterpret_cast<const unsigned long long*>(c->sw_fmax);
        for (int q = 0; q < L; ++q) b = std::max(b, fm[q]);
        reinterpret_cast<int64_t*>(c->sw_out)[6] = (int64_t)b;
    }
    const int64_t* cn = reinterpret_cast<const int64_t*>(c->sw_out + io.counts);
    size_t bytes = io.sets;
    const int nb = (hdr[0] == 1 && hdr[4]) ? 6 : 4;
    for (int b = 0; b < nb; ++b)
        for (int p = 0; p < L; ++p) bytes += (size_t)cn[(size_t)b * L + p] * width(b, p) * 4;
    if (bytes > outcap) return set_err(c, TCI_ERR_DEVICE, "device sweep: output image overflow");
    out.assign(c->sw_out, c->sw_out + bytes);
    // the tensors the sweep (mode 2) or the solving fill wrote (fill status hdr[8] == 0), one copy
    if (s1 && s1->tensors && hdr[0] == 0 && s1->table && (mode == 2 || hdr[8] == 0)) {
        const int64_t used = hdr[10];
        if (used < 0 || used > s1->tcap) return set_err(c, TCI_ERR_DEVICE, "device sweep: tensor overflow");
        HIPCHK(c, hipMemcpyAsync(s1->table, c->sw_tens, (size_t)(2 * L) * 8, hipMemcpyDeviceToHost, c->stream));
        if (used > 0)
            HIPCHK(c, hipMemcpyAsync(s1->data, c->sw_tens + 2 * L, (size_t)used * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    return TCI_OK;
}

// Chained optimize! for the device-resident small sweep: the iterations of optimize!
// (tensorci2.jl:1018-1172 with no global pivot search) as back-to-back launches that hand the state
// over in device memory -- iteration i reads iteration i-1's output image, folds its fill maxima and
// derives its abstol on the device, and records pivoterror / rank / the convergence test in ctl
// (SweepSmallArgs) -- with one host synchronisation per chunk of iterations (the first chunk is
// ncheckhistory long: no earlier iteration can converge), then the closing sweep1site! launch.
// Launches after the stop return at once. Results:
//   *ended = 1: the loop ended on the device at iteration *niter (converged or maxiter); with
//     *s1done the closing sweep ran too (out = its image, tensors as tci_sweep_small_run mode 2;
//     *errnorm = the maxsample it normalised with), else out = iteration *niter's image.
//   *ended = 0: iteration *niter + 1 could not run on the device (a bond outgrew the workgroup, a NaN,
//     a fill that does not fit): out = iteration *niter's image (empty when *niter = 0); the caller
//     continues from there on the ordinary path, which raises the reference's errors.
//   errors[i] / ranks[i], i = 1 .. *niter: pivoterror and rank after iteration i.
// Iteration images carry the sweep's maxsample; the fill maxima are folded into `out`'s header here.
int tci_sweep_small_optimize(tci_ctx* c, const tci_func* f, int L, int64_t cap, const char* in, size_t inbytes,
                             double tol, int norm, int maxiter, int ncheck, int strictlynested, int64_t maxbonddim,
                             int fsolve, int64_t fill_tcap, const tci::SwSweep1* s1, std::vector<char>& out,
                             int* niter, int* ended, int* s1done, double* errors, int64_t* ranks, double* errnorm) {
    auto width = [&](int bank, int p) { return (bank & 1) ? L - 1 - p : p; };
    const int64_t tot = 6 * cap * ((int64_t)L * (L - 1) / 2);
    const tci::SwIO io = tci::sw_io(L);
    const size_t outcap = io.sets + (size_t)tot * 4;
    const size_t nctl = 8 + 2 * (size_t)tci::kSwOptMax;
    *niter = 0;
    *ended = 0;
    *s1done = 0;
    out.clear();
    if (maxiter < 1 || maxiter >= tci::kSwOptMax || ncheck < 1) return set_err(c, TCI_ERR_ARG, "optimize chain: maxiter");
    int st;
    if ((st = ensure(c, &c->sw_ws, &c->capSwWs, (size_t)std::max<int64_t>(tot, 1)))) return st;
    if ((st = ensure(c, &c->sw_inbuf, &c->capSwInbuf, inbytes))) return st;
    for (int i = 0; i < 2; ++i)
        if ((st = ensure(c, &c->sw_img[i], &c->capSwImg[i], outcap))) return st;
    if ((st = ensure(c, &c->sw_ctl, &c->capSwCtl, nctl))) return st;
    if ((st = ensure_pinned(c, &c->hctl, &c->capHctl, nctl * 8))) return st;
    if ((st = ensure_mapped_pair(c, &c->sw_in, &c->sw_in_d, &c->capSwIn, inbytes))) return st;
    if ((st = ensure_mapped_pair(c, &c->sw_out, &c->sw_out_d, &c->capSwOut, outcap))) return st;
    if ((st = ensure(c, &c->sw_fmap, &c->capSwFmap, (size_t)(4 * L + 4)))) return st;
    if ((st = ensure_mapped_pair(c, &c->sw_fmax, &c->sw_fmax_d, &c->capSwFmax, (size_t)L * 8))) return st;
    if (fsolve && fill_tcap > 0 && (st = ensure(c, &c->sw_tens, &c->capSwTens, (size_t)(2 * L + fill_tcap))))
        return st;
    // the closing sweep writes its (small) site tensors straight into mapped host memory: no copy
    // and no second synchronisation after the chain
    if (s1 && s1->tensors &&
        (st = ensure_mapped_pair(c, &c->sw_s1t, &c->sw_s1t_d, &c->capSwS1t, (size_t)(2 * L + s1->tcap) * 8)))
        return st;
    memcpy(c->sw_in, in, inbytes);
    HIPCHK(c, hipMemcpyAsync(c->sw_inbuf, c->sw_in, inbytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemsetAsync(c->sw_ctl, 0, nctl * 8, c->stream));
    unsigned long long* fmax_d = reinterpret_cast<unsigned long long*>(c->sw_fmax_d);
    tci::SweepSmallArgs a;
    a.f = f->view();
    a.L = L;
    a.ws = c->sw_ws;
    a.cap = cap;
    a.niter = 2;  // sweep2site!(tci, f, 2; iter1 = 1): one back-and-forth pair per iteration
    a.iter1 = 1;
    a.strategy = 0;
    a.strictlynested = strictlynested;
    a.abstol = 0.0;  // (derived on the device)
    a.maxbonddim = maxbonddim;
    a.mode = 0;
    a.fill = 1;
    a.fsolve = fsolve ? 1 : 0;
    a.fmap = c->sw_fmap;
    a.s1fwd = 0;
    a.s1tens = 0;
    a.reltol = 1e-14;
    a.tens = fsolve ? c->sw_tens : nullptr;
    a.tcap = fsolve ? fill_tcap : 0;
    a.lu_wave = c->sw_lu_wave;
    a.lazy_union = c->sw_lazy_union;
    a.ctl = c->sw_ctl;
    a.opt_maxiter = maxiter;
    a.opt_ncheck = ncheck;
    a.opt_norm = norm ? 1 : 0;
    a.opt_tol = tol;
    const unsigned long long* hc = reinterpret_cast<const unsigned long long*>(c->hctl);
    // the closing sweep1site! (mode 2), enqueued after every chunk: it runs only once the loop has
    // ended (ctl[0] = 1), from the stop iteration's image, with that iteration's fill folded on the
    // device -- so a loop that ends inside a chunk costs no further round trip
    tci::SweepSmallArgs z = a;
    if (s1) {
        z.mode = 2;
        z.fill = 0;
        z.fsolve = 0;
        z.fmap = nullptr;
        z.opt_it = -1;
        z.inbuf = c->sw_img[0];
        z.img_sel[0] = c->sw_img[0];
        z.img_sel[1] = c->sw_img[1];
        z.out = c->sw_out_d;
        z.fmax_in = fmax_d;
        z.s1fwd = s1->forward;
        z.s1tens = s1->tensors;
        z.reltol = s1->reltol;
        z.tens = s1->tensors ? reinterpret_cast<double*>(c->sw_s1t_d) : nullptr;
        z.tcap = s1->tensors ? s1->tcap : 0;
    }
    const char* prev = c->sw_inbuf;
    int it = 1;
    unsigned long long stop = 0, stop_it = 0;
    while (it <= maxiter) {
        const int chunk = it == 1 ? std::min(ncheck, maxiter) : std::min(2, maxiter - it + 1);
        for (int j = 0; j < chunk; ++j, ++it) {
            a.opt_it = it;
            a.inbuf = prev;
            a.out = c->sw_img[it & 1];
            a.fmax_in = it > 1 ? fmax_d : nullptr;
            HIPCHK(c, tci::launch_sweep_small(c->stream, a));
            HIPCHK(c, tci::launch_fill_sites(c->stream, a, fmax_d));
            prev = c->sw_img[it & 1];
        }
        if (s1) HIPCHK(c, tci::launch_sweep_small(c->stream, z));
        HIPCHK(c, hipMemcpyAsync(c->hctl, c->sw_ctl, nctl * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        stop = hc[0];
        stop_it = hc[1];
        if (stop) break;
    }
    if (stop != 1 && stop != 2) return set_err(c, TCI_ERR_DEVICE, "optimize chain: no stop after maxiter");
    const int n = stop == 1 ? (int)stop_it : (int)stop_it - 1;  // iterations completed on the device
    for (int i = 1; i <= n; ++i) {
        errors[i] = __builtin_bit_cast(double, hc[8 + i]);
        ranks[i] = (int64_t)hc[8 + tci::kSwOptMax + i];
    }
    *niter = n;
    // iteration n's image (device) -> out, with its fill's maxima folded into the header
    auto take_iteration = [&]() -> int {
        if (n == 0) return TCI_OK;
        const char* img = c->sw_img[n & 1];
        std::vector<char> head(io.sets);
        HIPCHK(c, hipMemcpyAsync(head.data(), img, io.sets, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        const int64_t* cn = reinterpret_cast<const int64_t*>(head.data() + io.counts);
        size_t bytes = io.sets;
        for (int b = 0; b < 4; ++b)
            for (int p = 0; p < L; ++p) bytes += (size_t)cn[(size_t)b * L + p] * width(b, p) * 4;
        if (bytes > outcap) return set_err(c, TCI_ERR_DEVICE, "optimize chain: image overflow");
        out.assign(head.begin(), head.end());
        out.resize(bytes);
        if (bytes > io.sets)
            HIPCHK(c, hipMemcpyAsync(out.data() + io.sets, img + io.sets, bytes - io.sets, hipMemcpyDeviceToHost,
                                     c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        int64_t* hdr = reinterpret_cast<int64_t*>(out.data());
        unsigned long long b = (unsigned long long)hdr[6] & 0x7fffffffffffffffull;
        const unsigned long long* fm = reinterpret_cast<const unsigned long long*>(c->sw_fmax);
        for (int q = 0; q < L; ++q) b = std::max(b, fm[q]);
        hdr[6] = (int64_t)b;
        return TCI_OK;
    };
    if (stop == 2) return take_iteration();
    *ended = 1;
    if (!s1) return take_iteration();
    // (the closing sweep ran behind the chunk that stopped the loop)
    *errnorm = __builtin_bit_cast(double, hc[2]);
    const int64_t* hdr = reinterpret_cast<const int64_t*>(c->sw_out);
    if (hdr[0] != 0) return take_iteration();  // the host loop runs sweep1site! (and raises its errors)
    const int64_t* cn = reinterpret_cast<const int64_t*>(c->sw_out + io.counts);
    size_t bytes = io.sets;
    for (int b = 0; b < 4; ++b)
        for (int p = 0; p < L; ++p) bytes += (size_t)cn[(size_t)b * L + p] * width(b, p) * 4;
    if (bytes > outcap) return set_err(c, TCI_ERR_DEVICE, "device sweep: output image overflow");
    out.assign(c->sw_out, c->sw_out + bytes);
    if (s1->tensors && s1->table) {
        const int64_t used = hdr[10];
        if (used < 0 || used > s1->tcap) return set_err(c, TCI_ERR_DEVICE, "device sweep: tensor overflow");
        const double* tm = reinterpret_cast<const double*>(c->sw_s1t);
        memcpy(s1->table, tm, (size_t)(2 * L) * 8);
        if (used > 0) memcpy(s1->data, tm + 2 * L, (size_t)used * 8);
    }
    *s1done = 1;
    return TCI_OK;
}

int tci_sweep_small_error(tci_ctx* c, int status, int64_t bond) {
    if (status == 2) return set_err(c, TCI_ERR_NAN, "lu.L contains NaNs");
    if (status == 3) return set_err(c, TCI_ERR_NAN, "lu.U contains NaNs");
    if (status == 4) return set_err(c, TCI_ERR_NONSQ, "Pivot matrix at bond " + std::to_string(bond) + " is not square!");
    return set_err(c, TCI_ERR_DEVICE, "device sweep: status " + std::to_string(status));
}
