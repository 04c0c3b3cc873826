"""ctypes binding of libpsk.so (include/psk.h), the gfx950 Krylov engine.

There is no CPU fallback: if the library is missing or cannot be loaded this
module raises ImportError, and every solve goes through the HIP kernels.
"""
import atexit
import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSK_LIBRARY", os.path.join(_HERE, "_lib", "libpsk.so"))

PSK_OK = 0
PSK_ERR_ARG, PSK_ERR_HIP, PSK_ERR_RCCL, PSK_ERR_ALLOC, PSK_ERR_UNSUPPORTED = -1, -2, -3, -4, -5
ABI_VERSION = 4          # include/psk.h PSK_ABI_VERSION (psk_ctl.norm_b in 2, psk_result.exit in 3, comm timing in 4)
PSK_CONVERGED, PSK_MAXITER, PSK_BREAKDOWN, PSK_TRUE_RESID_FAIL = 0, 1, 2, 3
PSK_EXIT_NONE, PSK_EXIT_TOLERANCE, PSK_EXIT_ARNOLDI_BREAKDOWN, PSK_EXIT_MAXITER, PSK_EXIT_DOT_BREAKDOWN = 0, 1, 2, 3, 4
PSK_HOST, PSK_DEVICE = 0, 1
PSK_PREC_IDENTITY, PSK_PREC_JACOBI, PSK_PREC_ILU, PSK_PREC_AMG, PSK_PREC_DENSE = 0, 1, 2, 3, 4
PSK_LAYOUT_CSR, PSK_LAYOUT_SLICED, PSK_LAYOUT_SLICED_WIDE, PSK_LAYOUT_SLICED_DICT, PSK_LAYOUT_DIAG = 0, 1, 2, 3, 4
PSK_UNIQUE_ID_BYTES = 128

STATUS_NAMES = {PSK_CONVERGED: "converged", PSK_MAXITER: "maxiter", PSK_BREAKDOWN: "breakdown",
                PSK_TRUE_RESID_FAIL: "true residual above tolerance"}


class PskCtl(ctypes.Structure):
    _fields_ = [("maxiter", ctypes.c_int64), ("tau", ctypes.c_double),
                ("fail_on_maxiter", ctypes.c_int32), ("restart", ctypes.c_int32),
                ("check_every", ctypes.c_int32), ("time_kernels", ctypes.c_int32), ("norm_b", ctypes.c_double)]


class PskResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("success", ctypes.c_int32), ("iters", ctypes.c_int64),
                ("resid", ctypes.c_double), ("resid_recursive", ctypes.c_double),
                ("norm_b", ctypes.c_double), ("loop_ms", ctypes.c_double), ("spmv_ms", ctypes.c_double),
                ("spmv_launches", ctypes.c_int64), ("hist_len", ctypes.c_int64), ("msg", ctypes.c_char * 256),
                ("exit", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("gather_ms", ctypes.c_double), ("halo_ms", ctypes.c_double), ("comm_samples", ctypes.c_int64)]


# name -> (restype, argtypes); this is the full list of symbols include/psk.h declares
P = ctypes.c_void_p
I32, I64, F64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_double
PP = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = {
    "psk_abi_version": (ctypes.c_int, []),
    "psk_last_error": (ctypes.c_char_p, []),
    "psk_device_count": (ctypes.c_int, [ctypes.POINTER(I32)]),
    "psk_set_device": (ctypes.c_int, [I32]),
    "psk_synchronize": (ctypes.c_int, []),
    "psk_shutdown": (ctypes.c_int, []),
    "psk_shutdown_ex": (ctypes.c_int, [ctypes.c_int32]),
    "psk_dmalloc": (ctypes.c_int, [I64, PP]),
    "psk_dfree": (ctypes.c_int, [P]),
    "psk_h2d": (ctypes.c_int, [P, P, I64]),
    "psk_d2h": (ctypes.c_int, [P, P, I64]),
    "psk_dmemset0": (ctypes.c_int, [P, I64]),
    "psk_csr_create": (ctypes.c_int, [I64, I64, P, P, P, I32, PP]),
    "psk_csr_create_fd2d": (ctypes.c_int, [F64, F64, I64, PP]),
    "psk_csr_create_rect": (ctypes.c_int, [I64, I64, I64, P, P, P, I32, PP]),
    "psk_csr_info": (ctypes.c_int, [P, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
    "psk_csr_layout": (ctypes.c_int, [P, I32, ctypes.POINTER(I32)] + [ctypes.POINTER(I64)] * 3),
    "psk_csr_download": (ctypes.c_int, [P, P, P, P]),
    "psk_csr_destroy": (ctypes.c_int, [P]),
    "psk_spmv": (ctypes.c_int, [P, P, P, I32]),
    "psk_spmv_timed": (ctypes.c_int, [P, P, P, I32, ctypes.POINTER(F64)]),
    "psk_dot": (ctypes.c_int, [I64, P, P, I32, ctypes.POINTER(F64)]),
    "psk_nrm2": (ctypes.c_int, [I64, P, I32, ctypes.POINTER(F64)]),
    "psk_axpy": (ctypes.c_int, [I64, F64, P, P, I32]),
    "psk_prec_create": (ctypes.c_int, [P, I32, PP]),
    "psk_prec_apply": (ctypes.c_int, [P, I64, P, P, I32]),
    "psk_prec_jacobi_uniform": (ctypes.c_int, [P, ctypes.POINTER(I32), ctypes.POINTER(ctypes.c_double)]),
    "psk_prec_create_ilu": (ctypes.c_int, [I64, P, P, P, P, P, P, P, P, PP]),
    "psk_prec_destroy": (ctypes.c_int, [P]),
    "psk_prec_create_trisolve": (ctypes.c_int, [I64, P, P, P, I32, P, P, P, I32, P, P, PP]),
    "psk_prec_create_amg": (ctypes.c_int, [I32, PP, PP, PP, PP, P, I32, I32, I32, F64, PP]),
    "psk_prec_create_dense_inverse": (ctypes.c_int, [P, I32, PP]),
    "psk_prec_trisolve_schedule": (ctypes.c_int, [P, I32, I32, ctypes.POINTER(I32), ctypes.POINTER(I64),
                                                   ctypes.POINTER(I32), ctypes.POINTER(F64), ctypes.POINTER(F64)]),
    "psk_prec_trisolve_grid_info": (ctypes.c_int, [P, I32, ctypes.POINTER(I64)]),
    "psk_trisolve_grid_plan": (ctypes.c_int, [I64, P, P, P, I32, ctypes.POINTER(I64)]),
    "psk_prec_info": (ctypes.c_int, [P, ctypes.POINTER(I32)] + [ctypes.POINTER(I64)] * 5),
    "psk_mm_info": (ctypes.c_int, [ctypes.c_char_p] + [ctypes.POINTER(I64)] * 3),
    "psk_mm_read": (ctypes.c_int, [ctypes.c_char_p, P, P, P, ctypes.POINTER(I64)]),
    "psk_csr_create_mm": (ctypes.c_int, [ctypes.c_char_p, PP]),
    "psk_sa_aggregate": (ctypes.c_int, [I64, P, P, P, F64, P, ctypes.POINTER(I64), P]),
    "psk_pcg": (ctypes.c_int, [P, P, P, P, ctypes.POINTER(PskCtl), ctypes.POINTER(PskResult), P, I32]),
    "psk_gmres": (ctypes.c_int, [P, P, P, P, ctypes.POINTER(PskCtl), ctypes.POINTER(PskResult), P, I32]),
    "psk_comm_unique_id": (ctypes.c_int, [P]),
    "psk_comm_init": (ctypes.c_int, [I32, I32, P, PP]),
    "psk_comm_destroy": (ctypes.c_int, [P]),
    "psk_comm_init_dry": (ctypes.c_int, [I32, I32, PP]),
    "psk_comm_init_host": (ctypes.c_int, [I32, I32, ctypes.c_char_p, PP]),
    "psk_comm_mailbox": (ctypes.c_int, [P, ctypes.c_char_p]),
    "psk_comm_mailbox_check": (ctypes.c_int, [P, I32]),
    "psk_csr_create_fd2d_dist": (ctypes.c_int, [F64, F64, I64, P, PP, ctypes.POINTER(I64),
                                                ctypes.POINTER(I64)]),
    "psk_csr_create_dist": (ctypes.c_int, [I64, P, P, P, P, P, PP]),
    "psk_csr_halo_cols": (ctypes.c_int, [P, P, ctypes.POINTER(I64)]),
    "psk_csr_halo_peers": (ctypes.c_int, [P, P, P, P, P, ctypes.POINTER(I32)]),
    "psk_csr_halo_pack": (ctypes.c_int, [P, P, P]),
    "psk_fd2d_dist_plan": (ctypes.c_int, [I64, I32, I32] + [ctypes.POINTER(I64)] * 5),
}


# include/psk_lab.h: libpsk_lab.so (tests / lab tools only; not part of the product library)
LAB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libpsk_lab.so")
LAB_SIGNATURES = {
    "psk_lab_occupy_begin": (ctypes.c_int, [I32, I32, F64]),
    "psk_lab_occupy_end": (ctypes.c_int, [ctypes.POINTER(I32)]),
    "psk_lab_occupy_xcc": (ctypes.c_int, [ctypes.POINTER(I32)]),
    "psk_lab_dispatch_probe": (ctypes.c_int, [I32, I32, F64, P]),
    "psk_lab_trisolve_workers": (ctypes.c_int, [P, I32, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
    "psk_lab_amg_gs_pair": (ctypes.c_int, [P, I32, ctypes.POINTER(I32), ctypes.POINTER(I32)]),
    "psk_lab_spmv_rotate": (ctypes.c_int, [P, ctypes.POINTER(P), ctypes.POINTER(P), I32, I32, I32, ctypes.POINTER(F64)]),
    "psk_lab_spmv_after_write": (ctypes.c_int, [P, P, P, P, P, I32, I32, I32, ctypes.POINTER(F64)]),
}
_lab = None


def load_lab():
    """libpsk_lab.so (include/psk_lab.h), loaded once: a separate library linked against the libpsk.so this
    module loaded (it shares libpsk's device context, streams and handles)."""
    global _lab
    if _lab is None:
        if not os.path.exists(LAB_PATH):
            raise ImportError("libpsk_lab.so not found at %s (make -C pysolvers_amd/csrc)" % LAB_PATH)
        lab = ctypes.CDLL(LAB_PATH)
        for name, (res, args) in LAB_SIGNATURES.items():
            fn = getattr(lab, name)
            fn.restype = res
            fn.argtypes = args
        _lab = lab
    return _lab


def prec_info(h):
    """dict(kind, n, nnz_l, nnz_u, levels_l, levels_u) of a psk_prec handle."""
    k = I32()
    v = [I64() for _ in range(5)]
    check(lib.psk_prec_info(h, ctypes.byref(k), *[ctypes.byref(x) for x in v]), "psk_prec_info")
    return dict(kind=k.value, n=v[0].value, nnz_l=v[1].value, nnz_u=v[2].value, levels_l=v[3].value,
                levels_u=v[4].value)


def handle_array(hs):
    """ctypes void*[] of handles (None -> NULL)."""
    arr = (ctypes.c_void_p * max(len(hs), 1))()
    for i, h in enumerate(hs):
        arr[i] = h.value if isinstance(h, ctypes.c_void_p) else h
    return ctypes.cast(arr, PP), arr


def fd2d_dist_plan(m, nranks, rank):
    """(row_begin, row_end, ncols, halo_lo, halo_hi) of `rank` (host-only, no GPU needed)."""
    v = [I64() for _ in range(5)]
    check(lib.psk_fd2d_dist_plan(m, nranks, rank, *[ctypes.byref(x) for x in v]), "psk_fd2d_dist_plan")
    return tuple(x.value for x in v)


class PskError(RuntimeError):
    """A negative return code from libpsk (API/HIP/RCCL error, not a numerical failure)."""

    def __init__(self, code, where, text):
        super().__init__("%s failed (%d): %s" % (where, code, text))
        self.code = code


def _pin_runtime():
    """Make sure the process ends up with ONE HIP/HSA/RCCL runtime.

    PyTorch-ROCm wheels ship their own HIP/HSA/RCCL and load them by UNVERSIONED names; libpsk
    asks by SONAME (libamdhip64.so.7, librccl.so.1). If libpsk were loaded first, a later
    `import torch` would map a second HIP runtime into the process (measured here: duplicate
    libamdhip64/libhsa-runtime64/librccl and a heap corruption at exit). So when torch is
    installed it is imported FIRST and libpsk binds to the runtime torch loaded (same sonames);
    without torch, or with PSK_NO_TORCH=1 (a process that will never import torch, e.g. a one-GPU
    bench.py), the system ROCm runtime is used.
    """
    import importlib.util
    if os.environ.get("PSK_NO_TORCH") == "1":   # the caller never imports torch: the system ROCm runtime
        return
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libpsk.so not found at %s — build it with `python -c 'import __graft_entry__ as "
                          "g; g.build()'` (make -C pysolvers_amd/csrc)" % LIB_PATH)
    _pin_runtime()
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.psk_abi_version() != ABI_VERSION:
        raise ImportError("libpsk ABI version mismatch (library %d, bindings %d)" % (lib.psk_abi_version(), ABI_VERSION))
    return lib


PSK_SHUTDOWN_RESET_DEVICE = 1
lib = _load()
shut_down = False


def _shutdown():
    """atexit: release libpsk's streams, events and host-mapped memory while the HIP runtime is still
    alive (psk_shutdown). Registered at import, so it runs after every atexit handler registered
    later (a caller's own cleanup still has the library); objects collected afterwards find their
    destroy entry points turned into no-ops."""
    global shut_down
    if not shut_down:
        shut_down = True
        # The exit fault under rocprofv3 (profiles/r4_exit_fault.txt) was fixed by launching the triangular
        # solves without hipLaunchCooperativeKernel and by keeping torch's bundled HIP runtime out of a one-rank
        # bench; a device reset did not change it. It would also destroy every other HIP user's allocations
        # in the process, so it is opt-in (PSK_SHUTDOWN_RESET=1).
        reset = os.environ.get("PSK_SHUTDOWN_RESET") == "1"
        lib.psk_shutdown_ex(PSK_SHUTDOWN_RESET_DEVICE if reset else 0)


atexit.register(_shutdown)


def check(rc, where):
    if rc != PSK_OK:
        raise PskError(rc, where, lib.psk_last_error().decode(errors="replace"))


def ptr(a):
    """Data pointer of a numpy array, a torch tensor or a raw int address."""
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    raise TypeError("cannot take the address of %r" % type(a))


def device_count():
    n = I32(0)
    check(lib.psk_device_count(ctypes.byref(n)), "psk_device_count")
    return n.value
