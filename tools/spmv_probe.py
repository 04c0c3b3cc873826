#!/usr/bin/env python3
"""Per-workgroup timeline of the diagonal-layout SpMV at the bench's N = 10M (lab tool; needs a
-DPSK_SPMV_PROF build: scripts/build_variant.sh sprof -DPSK_SPMV_PROF, then PSK_LIBRARY=tools/bin/ab_sprof/libpsk.so).

For the last SpMV of a short PCG solve (kSpmvDot, in the loop) and for one plain SpMV: the kernel span
(first entry to last exit, s_memrealtime at 100 MHz), how workgroup starts spread over it, the time from
the last workgroup's sums to its exit, the group reductions and the final reduction (the dot epilogue's
tail).
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
WG, GRP, FIN = 32768, 3 * 32768, 3 * 32768 + 2 * 4096


def read(N):
    buf = (ctypes.c_ulonglong * (FIN + 2))()
    fn = N.lib.psk_spmv_prof_read
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf) == 0
    return np.frombuffer(buf, dtype=np.uint64).astype(np.int64)


def summarize(p, nwg, label):
    w = p[:3 * nwg].reshape(nwg, 3)
    t0 = w[:, 0].min()
    ent, mid, end = (w[:, 0] - t0) * 10.0, (w[:, 1] - t0) * 10.0, (w[:, 2] - t0) * 10.0   # ns
    g = p[GRP:GRP + 2 * 4096].reshape(4096, 2)
    gv = g[(g[:, 0] >= t0) & (g[:, 1] >= g[:, 0])]
    out = {"label": label, "workgroups": int(nwg), "span_us": float(end.max() / 1e3),
           "entry_us_pct": [float(np.percentile(ent, q) / 1e3) for q in (0, 10, 50, 90, 99, 100)],
           "wg_dur_us_pct": [float(np.percentile(end - ent, q) / 1e3) for q in (10, 50, 90, 99)],
           "sums_to_exit_us_pct": [float(np.percentile(end - mid, q) / 1e3) for q in (10, 50, 90, 99, 100)],
           "last_sums_us": float(mid.max() / 1e3), "last_exit_us": float(end.max() / 1e3)}
    if len(gv):
        gs_, ge = (gv[:, 0] - t0) * 10.0, (gv[:, 1] - t0) * 10.0
        out.update(groups=int(len(gv)), group_red_us_pct=[float(np.percentile(ge - gs_, q) / 1e3) for q in (50, 90, 100)],
                   group_start_us_pct=[float(np.percentile(gs_, q) / 1e3) for q in (0, 50, 90, 100)],
                   last_group_end_us=float(ge.max() / 1e3))
    if p[FIN] >= t0:
        out.update(final_start_us=float((p[FIN] - t0) * 10.0 / 1e3), final_end_us=float((p[FIN + 1] - t0) * 10.0 / 1e3))
    return out


def main():
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import bench
    from pysolvers_amd import _native as N
    N.check(N.lib.psk_set_device(0), "set_device")
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 3163
    s = bench.PcgSystem(N, m, None, 1)
    tpw = int(os.environ.get("PSK_PROBE_TPW", "2"))   # slices per workgroup of the probed build
    nwg = ((s.nloc + 255) // 256 + tpw - 1) // tpw
    for it in (3, 20):
        s.run(it, False)
        print(json.dumps(summarize(read(N), nwg, "pcg_last_spmv_dot_%d" % it)), flush=True)
    ms = ctypes.c_double()
    N.check(N.lib.psk_spmv_timed(s.A, s.db, s.dsol, 1, ctypes.byref(ms)), "spmv_timed")
    print(json.dumps(summarize(read(N), nwg, "plain_spmv")), flush=True)
    s.free()


if __name__ == "__main__":
    main()
