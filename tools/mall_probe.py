#!/usr/bin/env python3
"""Is the in-loop SpMV's "loop context" the Infinity Cache? (lab tool, psk_lab_spmv_rotate)

The back-to-back SpMV batch re-reads ONE x (80 MB at N = 10M) and its 10 MB presence bytes, writing one y: ~170 MB,
which the 256 MB Infinity Cache (MALL) can hold across launches. In the PCG loop every SpMV reads a p that K3 has
just written while ~650 MB stream per iteration. This times back-to-back launches cycling through nbuf (x, y)
pairs: nbuf = 1 is the batch; at nbuf >= 2 the x of a launch was last read nbuf launches earlier, with
nbuf * 160 MB streamed in between.

A second probe times the SpMV launch alone (dispatch-recorded events) when every launch follows a streaming write of
n doubles: into nothing, into the SpMV's own x (as K3 writes the p the next SpMV gathers), or into another buffer.

    python tools/mall_probe.py [m] [reps]
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pysolvers_amd import _native as N  # noqa: E402


def main(m=3163, reps=120):
    n = m * m
    lab = N.load_lab()
    N.check(N.lib.psk_set_device(0), "dev")
    A = ctypes.c_void_p()
    N.check(N.lib.psk_csr_create_fd2d(-1.0, 1.0, m, ctypes.byref(A)), "fd2d")
    xe = np.random.default_rng(12345).random(n)
    bufs = []
    for _ in range(8):
        dx, dy = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dx)), "alloc")
        N.check(N.lib.psk_dmalloc(n * 8, ctypes.byref(dy)), "alloc")
        N.check(N.lib.psk_h2d(dx, N.ptr(xe), n * 8), "h2d")
        bufs.append((dx, dy))
    out = {"m": m, "reps": reps, "layout_bytes_per_launch": 17 * n}
    for dot in (0, 1):
        for nbuf in (1, 2, 4, 8):
            xs = (ctypes.c_void_p * nbuf)(*[b[0].value for b in bufs[:nbuf]])
            ys = (ctypes.c_void_p * nbuf)(*[b[1].value for b in bufs[:nbuf]])
            vals = []
            for _ in range(3):
                ms = ctypes.c_double()
                N.check(lab.psk_lab_spmv_rotate(A, ctypes.cast(xs, ctypes.POINTER(ctypes.c_void_p)),
                                                ctypes.cast(ys, ctypes.POINTER(ctypes.c_void_p)), nbuf, reps, dot,
                                                ctypes.byref(ms)), "rotate")
                vals.append(ms.value)
            key = "%s_nbuf%d" % ("dot" if dot else "plain", nbuf)
            out[key] = {"avg_ms": vals, "frac_of_8TBps": [17 * n / (v * 1e-3) / 8e12 for v in vals]}
            print(key, " ".join("%.4f" % v for v in vals), flush=True)
    # each SpMV after a streaming write kernel (16-B copy of n doubles): none / into the SpMV's x / into another buffer
    src, scr = bufs[6][1], bufs[7][1]
    x, y = bufs[0]
    for dot in (0, 1):
        for target, tname in ((0, "none"), (1, "x"), (2, "other")):
            vals = []
            for _ in range(3):
                ms = ctypes.c_double()
                N.check(lab.psk_lab_spmv_after_write(A, x, y, src, scr, target, min(reps, 200), dot, ctypes.byref(ms)),
                        "after_write")
                vals.append(ms.value)
            key = "%s_after_write_%s" % ("dot" if dot else "plain", tname)
            out[key] = {"avg_ms": vals}
            print(key, " ".join("%.4f" % v for v in vals), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
