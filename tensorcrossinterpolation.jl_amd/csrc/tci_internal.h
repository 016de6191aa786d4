// tci_internal.h -- shared declarations between the device code (tci_device.hip) and the
// C-ABI host layer (tci_abi.cpp). Not part of the public ABI (include/tci_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tci {

// Argmax candidate: abs2 value, column and row in the *current permuted* coordinates.
// Sentinel (no finite candidate): v = -1, col = row = INT32_MAX.
struct Cand {
    double v;
    int32_t col;
    int32_t row;
};

// Device-resident rrLU state (mirrors rrLU.npivot / rrLU.error and the loop-local maxerror of
// _optimizerrlu!, matrixlu.jl:353-369). Written only by the single-block select kernel.
struct RrluState {
    int64_t np;      // pivots accepted so far
    int32_t done;    // stop test fired (matrixlu.jl:363-365)
    int32_t pad;
    double maxerror;
    double error;    // lu.error (last |A[p,q]| examined)
    int64_t p, q;    // accepted pivot position (0-based, permuted coordinates)
    double pval;     // A[p,q]
};

// Device view of an integrand (tci_func).
struct FuncDev {
    int32_t kind;
    int32_t L;
    const int32_t* localdims;  // device
    const double* params;      // device
    int64_t nparams;
    const int64_t* strides;    // device, column-major strides for TCI_F_TABLE
};

constexpr int kUpdThreads = 256;   // fused Schur update: 4 waves
constexpr int kRowsPerTile = 512;  // 256 lanes x double2
constexpr int kSelThreads = 1024;

// ---- launchers (tci_device.hip)
void launch_argmax_update(hipStream_t s, bool update, double* A, int64_t lda, int m, int n, int k,
                          const double* ybuf, const RrluState* st, Cand* cand, int grid, int cb);
int argmax_grid(int m, int n, int k, int cb, int max_grid);
void launch_select(hipStream_t s, const double* A, int64_t lda, int m, int n, int k,
                   const Cand* cand, int ncand, RrluState* st, double reltol, double abstol);
void launch_swap(hipStream_t s, double* A, int64_t lda, int m, int n, int k, const RrluState* st,
                 int64_t* rowperm, int64_t* colperm, double* ybuf, int leftorth);
void launch_init_state(hipStream_t s, RrluState* st, int64_t* rowperm, int m, int64_t* colperm, int n);
void launch_nan_check(hipStream_t s, const double* A, int64_t lda, int m, int n, int np,
                      int* flag);
void launch_gather_diag(hipStream_t s, const double* A, int64_t lda, int np, double* out);
void launch_extract_LU(hipStream_t s, const double* A, int64_t lda, int m, int n, int np,
                       int leftorth, double* L, int64_t ldl, double* U, int64_t ldu);
void launch_luci_factors(hipStream_t s, double* A, int64_t lda, int m, int n, int np,
                         int leftorth, const int64_t* rowperm, const int64_t* colperm,
                         double* left, double* right);
void launch_fill_uniform(hipStream_t s, double* A, int64_t m, int64_t n, int64_t lda, uint64_t seed);

// batch evaluation: I (m x nl) and J (n x nr) device int32 tables, row-major entries.
// scratch must hold batcheval_scratch_bytes() bytes. maxbits: device uint64, zeroed.
// D = prod of the M centre local dims (1 when M == 0).
void launch_batcheval(hipStream_t s, const FuncDev& f, const int32_t* I, int m, int nl,
                      const int32_t* J, int n, int nr, int M, int D, double* out, int64_t ldo,
                      unsigned long long* maxbits, void* scratch);
int64_t batcheval_scratch_bytes(const FuncDev& f, int m, int D, int n);

// site-tensor solve: T (R x r) = Pi1 (R x r) * P^-1; P overwritten by its LU (partial pivot of P^T)
void launch_sitetensor_solve(hipStream_t s, double* P, int r, double* Pi1, int R, double* T,
                             int* piv);

}  // namespace tci
