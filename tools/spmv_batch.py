#!/usr/bin/env python3
"""Back-to-back SpMV launch time on FDLaplacian2D(-1, 1, m) (lab tool; psk_spmv_timed).

    PSK_SPMV_TIMED_MODE=1 python tools/spmv_batch.py [m] [reps]

Mode 0 (default): plain y = A x; mode 1: the PCG loop's kSpmvDot launch (dot epilogue + gridsum).
PSK_LIBRARY selects a libpsk build (A/B of experiment builds on one box)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pysolvers_amd import _native as N  # noqa: E402


def main(m=3163, reps=200):
    n = m * m
    A, dx, dy = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    N.check(N.lib.psk_set_device(0), "dev")
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "fd2d")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dx)), "alloc")
    N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dy)), "alloc")
    xe = np.random.default_rng(12345).random(n)
    N.check(N.lib.psk_h2d(dx, N.ptr(xe), n * 8), "h2d")
    ms = ctypes.c_double()
    out = []
    for _ in range(3):
        N.check(N.lib.psk_spmv_timed(A, dx, dy, reps, ctypes.byref(ms)), "timed")
        out.append(ms.value)
    print("m=%d mode=%s lib=%s avg_ms %s" % (m, os.environ.get("PSK_SPMV_TIMED_MODE", "0"),
                                             os.path.basename(os.path.dirname(N.LIB_PATH)),
                                             " ".join("%.4f" % v for v in out)))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
