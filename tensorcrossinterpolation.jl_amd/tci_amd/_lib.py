"""ctypes binding of libtci_hip.so (include/tci_hip.h).

The HIP library is the only compute path: if it is missing or no GPU is visible, every entry
point raises -- there is no CPU fallback.
"""
import atexit
import ctypes as C
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TCI_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libtci_hip.so"))

TCI_OK, TCI_ERR_ARG, TCI_ERR_NAN, TCI_ERR_NONSQ, TCI_ERR_DEVICE, TCI_ERR_NOMEM, TCI_ERR_HOST = range(7)

i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
vp = C.c_void_p
dbl = C.c_double
i64 = C.c_int64
i32 = C.c_int32
pi64 = C.POINTER(C.c_int64)
pdbl = C.POINTER(C.c_double)


class TCIError(RuntimeError):
    """Raised for TCI_ERR_* codes; the message follows the reference's exception text."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class TCIArgumentError(TCIError, ValueError):
    pass


class TCIDeviceError(TCIError):
    pass


# optional pointers (NULL allowed) use c_void_p and are passed via _ptr()
SIGNATURES = {
    "tci_ctx_create": ([C.c_int, C.POINTER(vp)], C.c_int),
    "tci_ctx_destroy": ([vp], C.c_int),
    "tci_last_error": ([vp], C.c_char_p),
    "tci_ctx_stream": ([vp], vp),
    "tci_ctx_synchronize": ([vp], C.c_int),
    "tci_last_kernel_stats": ([vp, C.c_int, pdbl, pi64], C.c_int),
    "tci_last_kernel_units": ([vp, C.c_int, pdbl, pi64, pi64], C.c_int),
    "tci_set_rrlu_persist": ([vp, C.c_int], C.c_int),
    "tci_rrlu_persist_faulted": ([vp], C.c_int),
    "tci_set_shard_exchange": ([vp, C.c_int], C.c_int),
    "tci_last_shard_exchange": ([vp], C.c_int),
    "tci_set_timing": ([vp, C.c_int], C.c_int),
    "tci_set_rrlu_flush": ([vp, C.c_int], C.c_int),
    "tci_set_rrlu_epochs": ([vp, C.c_int], C.c_int),
    "tci_rrlu_epochs_for": ([vp, i64, i64], C.c_int),
    "tci_set_rrlu_small": ([vp, C.c_int], C.c_int),
    "tci_set_rrlu_mid": ([vp, C.c_int], C.c_int),
    "tci_set_rrlu_shadow": ([vp, C.c_int], C.c_int),
    "tci_rrlu_shadow_bytes": ([], C.c_int),
    "tci_set_c128_shadow": ([vp, C.c_int], C.c_int),
    "tci_set_dense_mfma": ([vp, C.c_int], C.c_int),
    "tci_func_create": ([vp, C.c_int, vp, i64, i32p, i32, C.POINTER(vp)], C.c_int),
    "tci_func_destroy": ([vp], C.c_int),
    "tci_func_create_host": ([vp, vp, vp, i32p, i32, C.POINTER(vp)], C.c_int),
    "tci_func_create_c128": ([vp, vp, i32, vp, i32, C.POINTER(vp)], C.c_int),
    "tci_batcheval_h": ([vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, pdbl], C.c_int),
    "tci_batcheval_d": ([vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, pdbl], C.c_int),
    "tci_batcheval_dd": ([vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, vp], C.c_int),
    "tci_batcheval_da": ([vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, vp], C.c_int),
    "tci_rrlu_h": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, vp, vp, i64, pi64, pdbl],
                   C.c_int),
    "tci_rrlu_c128_h": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, vp, vp, i64, pi64, pdbl,
                         vp], C.c_int),
    "tci_rrlu_c128_inplace_d": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, pi64, pdbl, vp],
                                C.c_int),
    "tci_luci_c128_h": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, vp, vp, vp, pi64], C.c_int),
    "tci_batcheval_c128_h": ([vp, vp, dbl, dbl, vp, i64, C.c_int32, vp, i64, C.c_int32, C.c_int32, vp, pdbl],
                             C.c_int),
    "tci_update_pivots_c128_h": ([vp, vp, dbl, dbl, vp, i64, C.c_int32, vp, i64, C.c_int32, i64, dbl, dbl,
                                  C.c_int, C.c_int, vp, vp, vp, pi64, pdbl, vp, vp], C.c_int),
    "tci_sitetensor_solve_c128_h": ([vp, vp, i64, vp, i64, vp], C.c_int),
    "tci_tt_evaluate_c128_h": ([vp, C.c_int32, vp, vp, vp, i64, vp, i64, vp], C.c_int),
    "tci_rrlu_inplace_d": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, pi64, pdbl, vp],
                           C.c_int),
    "tci_rrlu_copy_d": ([vp, vp, i64, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, pi64, pdbl, vp],
                        C.c_int),
    "tci_luci_h": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, vp, vp, vp, pi64], C.c_int),
    "tci_luci_inplace_d": ([vp, vp, i64, i64, i64, i64, dbl, dbl, C.c_int, vp, vp, vp, vp, vp, pi64], C.c_int),
    "tci_update_pivots_h": ([vp, vp, vp, i64, i32, vp, i64, i32, i64, dbl, dbl, C.c_int, C.c_int, vp,
                             vp, vp, pi64, pdbl, vp, vp], C.c_int),
    "tci_sitetensor_h": ([vp, vp, vp, i64, i32, vp, i64, i32, vp, i64, vp, pdbl], C.c_int),
    "tci_sitetensor_solve_h": ([vp, vp, i64, vp, i64, vp], C.c_int),
    "tci_tt_evaluate_h": ([vp, i32, vp, vp, vp, i64, vp, i64, vp], C.c_int),
    "tci_fill_uniform_d": ([vp, vp, i64, i64, i64, C.c_uint64], C.c_int),
    "tci_fill_uniform_block_d": ([vp, vp, i64, i64, i64, C.c_uint64, C.c_uint64], C.c_int),
    "tci_diag_stream_d": ([vp, vp, vp, i64, C.c_int, C.c_int, pdbl, pdbl], C.c_int),
    "tci_diag_mfma_f64": ([vp, pdbl], C.c_int),
    "tci_diag_mfma_f64_ex": ([vp, C.c_int, pdbl, pdbl], C.c_int),
    "tci_sitetensor_solve_d": ([vp, vp, i64, vp, i64, vp], C.c_int),
    "tci_dgemm_d": ([vp, C.c_int, i64, i64, i64, dbl, vp, i64, vp, i64, dbl, vp, i64], C.c_int),
    "tci_schur_update_d": ([vp, vp, i64, i64, i64, vp, i64, vp, i64, i64], C.c_int),
    "tci_tci2_create": ([vp, i32, i32p, C.POINTER(vp)], C.c_int),
    "tci_tci2_destroy": ([vp], C.c_int),
    "tci_tci2_set_set": ([vp, C.c_int, i32, vp, i64], C.c_int),
    "tci_tci2_get_set": ([vp, C.c_int, i32, vp, i64, pi64], C.c_int),
    "tci_tci2_clear_history": ([vp], C.c_int),
    "tci_tci2_set_errors": ([vp, dbl, vp, vp, i64], C.c_int),
    "tci_tci2_errors": ([vp, pdbl, vp, vp, i64, pi64], C.c_int),
    "tci_tci2_sweep2site": ([vp, vp, i32, i32, dbl, i64, i32, i32], C.c_int),
    "tci_tci2_set_sets": ([vp, C.c_int, vp, vp], C.c_int),
    "tci_tci2_get_sets": ([vp, C.c_int, vp, vp, i64], C.c_int),
    "tci_tci2_fill_maxsample": ([vp, vp, C.POINTER(C.c_int)], C.c_int),
    "tci_tci2_fill_solve": ([vp, vp, vp, i64, vp, C.POINTER(C.c_int)], C.c_int),
    "tci_tci2_optimize_small": ([vp, vp, dbl, i64, i32, i32, i32, i32, i32, vp, i64, vp, vp, vp,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                 C.POINTER(C.c_double), C.POINTER(C.c_int)], C.c_int),
    "tci_tci2_sweep2site_fillsolve": ([vp, vp, i32, i32, dbl, i64, i32, i32, vp, i64, vp, C.POINTER(C.c_int)],
                                      C.c_int),
    "tci_tci2_sweep2site_fill": ([vp, vp, i32, i32, dbl, i64, i32, i32, C.POINTER(C.c_int)], C.c_int),
    "tci_tci2_sweep1site": ([vp, vp, i32, dbl, dbl, i64, i32, vp, i64, vp, C.POINTER(C.c_int)], C.c_int),
    "tci_set_sweep_small": ([vp, C.c_int], C.c_int),
    "tci_cache_create": ([vp, i32p, i32, i64, C.POINTER(vp)], C.c_int),
    "tci_cache_destroy": ([vp], C.c_int),
    "tci_cache_clear": ([vp], C.c_int),
    "tci_cache_size": ([vp, pi64], C.c_int),
    "tci_cache_dump_h": ([vp, vp, vp, i64, pi64], C.c_int),
    "tci_cache_lookup_h": ([vp, vp, i64, vp, vp], C.c_int),
    "tci_cache_batcheval_d": ([vp, vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, pdbl, pi64], C.c_int),
    "tci_cache_batcheval_h": ([vp, vp, vp, vp, i64, i32, vp, i64, i32, i32, vp, i64, pdbl, pi64], C.c_int),
    "tci_comm_unique_id": ([vp, pi64], C.c_int),
    "tci_comm_create": ([vp, C.c_int, C.c_int, vp, C.POINTER(vp)], C.c_int),
    "tci_comm_destroy": ([vp], C.c_int),
    "tci_comm_allgather_d": ([vp, vp, vp, i64], C.c_int),
    "tci_comm_allreduce_max_u64_d": ([vp, vp, i64], C.c_int),
    "tci_rrlu_sharded_d": ([vp, vp, vp, vp, C.c_int, vp, i64, i64, i64, i64, i64, i64, dbl, dbl, C.c_int,
                            vp, vp, pi64, pdbl, vp], C.c_int),
    "tci_rrlu_sharded_factors_h": ([vp, vp, vp, i64], C.c_int),
    "tci_malloc_d": ([vp, C.POINTER(vp), i64], C.c_int),
    "tci_free_d": ([vp, vp], C.c_int),
    "tci_memcpy_h2d": ([vp, vp, vp, i64], C.c_int),
    "tci_memset_d": ([vp, vp, C.c_int, i64], C.c_int),
    "tci_memcpy_d2h": ([vp, vp, vp, i64], C.c_int),
    "tci_memcpy_d2d": ([vp, vp, vp, i64], C.c_int),
    "tci_memcpy2d_d2d": ([vp, vp, i64, vp, i64, i64, i64], C.c_int),
}

# tci_exchange_fn (include/tci_hip.h): int (*)(void* user, int op, const void* d_send, void* d_recv,
# int64 count) -- op 0 all-gather, op 1 element-wise uint64 max, count 8-byte words
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, vp, C.c_int, vp, vp, i64)

_lib = None
_lock = threading.Lock()


def load():
    """Loads libtci_hip.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise TCIDeviceError(TCI_ERR_DEVICE,
                                     f"libtci_hip.so not found at {LIB_PATH}: build it with "
                                     "`python -c 'import __graft_entry__ as g; g.build()'` "
                                     "(no CPU fallback exists)")
            lib = C.CDLL(LIB_PATH)
            for name, (args, res) in SIGNATURES.items():
                try:
                    fn = getattr(lib, name)
                except AttributeError:
                    # an A/B build of an earlier commit (TCI_HIP_LIB): the entries it predates stay
                    # unbound; the in-tree library must export every one
                    if "TCI_HIP_LIB" in os.environ:
                        continue
                    raise
                fn.argtypes = args
                fn.restype = res
            _lib = lib
    return _lib


_host_exc = threading.local()


def set_host_exception(e):
    """Records the exception a host callback (tci_func_create_host) raised; Context.check re-raises
    it when the library returns TCI_ERR_HOST, so an error inside the user's f propagates as it
    would from f in the reference."""
    _host_exc.e = e


def ptr(a):
    """ctypes pointer of a numpy array (or None -> NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(vp)


# Teardown order (SIGSEGV inside exit() after rocprofv3 finalisation): every
# context and every device object it owns is released by an atexit hook, i.e. while the
# interpreter and the HIP runtime are both still intact. After that, __del__ methods and
# interpreter finalisation make no HIP calls at all.
_live_contexts = weakref.WeakSet()
_shutting_down = False


def shutting_down():
    return _shutting_down


@atexit.register
def _shutdown():
    global _shutting_down, _lib
    for c in list(_live_contexts):
        try:
            c.close()
        except Exception:
            pass
    _shutting_down = True
    # The compiler-generated module destructor of libtci_hip.so (it unregisters the embedded code
    # objects from the HIP runtime) is a C atexit handler of the library; left to exit(), it would
    # run after the C-level shutdown of whatever registered later (rocprofv3's tool finalisation is
    # one). Unloading the library here runs it now, while the runtime and any profiler are intact.
    # (The exit-time SIGSEGV of VERDICT r2 #6 itself was HIP's cooperative queue, see
    # tci_rrlu.hip launch_rrlu_mid.) Nothing calls into the library after this point: every
    # release()/__del__ checks Context.alive, which is False from here on.
    diag = os.environ.get("TCI_EXIT_DIAG")
    if diag:  # the process map before the unload, to resolve frames of an exit-time fault
        with open("/proc/self/maps") as src, open(diag, "w") as dst:
            dst.write(src.read())
    if _lib is not None and os.environ.get("TCI_UNLOAD_AT_EXIT", "1") == "1":
        try:
            import _ctypes
            handle, _lib = _lib._handle, None
            _ctypes.dlclose(handle)
        except Exception:
            pass
    if diag:
        import sys
        print(f"[tci_amd] atexit teardown done (unloaded: {_lib is None}); maps in {diag}",
              file=sys.stderr, flush=True)


class Context:
    """One tci_ctx (device stream + workspaces). Use `context()` for the per-thread default.

    Device objects created on a context (integrands, DeviceMatrix) register with `own()`; `close()`
    releases them before the context itself, and nothing touches HIP after the atexit hook."""

    def __init__(self, device=0):
        self.lib = load()
        h = vp()
        st = self.lib.tci_ctx_create(device, C.byref(h))
        if st != TCI_OK:
            raise TCIDeviceError(st, f"tci_ctx_create(device={device}) failed with code {st} "
                                     "(no visible MI355X / HIP runtime?)")
        self.h = h
        self.device = device
        self._owned = weakref.WeakSet()
        _live_contexts.add(self)

    def own(self, obj):
        """Registers a device object with a `release()` method, freed before the context."""
        self._owned.add(obj)
        return obj

    @property
    def alive(self):
        return bool(getattr(self, "h", None)) and not _shutting_down

    def check(self, st):
        if st == TCI_OK:
            return
        msg = self.lib.tci_last_error(self.h).decode(errors="replace")
        if st == TCI_ERR_HOST:
            e = getattr(_host_exc, "e", None)
            _host_exc.e = None
            if e is not None:
                raise e
        if st == TCI_ERR_ARG:
            raise TCIArgumentError(st, msg)
        if st == TCI_ERR_DEVICE or st == TCI_ERR_NOMEM:
            raise TCIDeviceError(st, msg)
        raise TCIError(st, msg)

    def close(self):
        if getattr(self, "h", None) and not _shutting_down:
            for obj in list(getattr(self, "_owned", ())):
                try:
                    obj.release()
                except Exception:
                    pass
            self.lib.tci_ctx_synchronize(self.h)
            self.lib.tci_ctx_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timing(self, on, stride=1):
        """HIP-event kernel timing on/off; rrLU passes are sampled every `stride`-th pivot."""
        self.check(self.lib.tci_set_timing(self.h, max(1, int(stride)) if on else 0))

    def kernel_stats(self, family):
        ms = C.c_double()
        n = C.c_int64()
        self.check(self.lib.tci_last_kernel_stats(self.h, family, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def kernel_units(self, family):
        """(total ms, launches, units) of a timing family; units = passes for the persistent epoch
        launches (families 41 / 42), launches otherwise."""
        ms = C.c_double()
        n = C.c_int64()
        u = C.c_int64()
        self.check(self.lib.tci_last_kernel_units(self.h, family, C.byref(ms), C.byref(n), C.byref(u)))
        return ms.value, n.value, u.value

    @property
    def stream(self):
        return self.lib.tci_ctx_stream(self.h)

    def synchronize(self):
        self.check(self.lib.tci_ctx_synchronize(self.h))


_tls = threading.local()


def context(device=None):
    """Default per-thread context on `device` (LOCAL_RANK or 0)."""
    if device is None:
        device = int(os.environ.get("TCI_DEVICE", "0"))
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]
