"""Per-band timeline of the AMG smoother's paired Gauss-Seidel launch (amg.hip gs_pair_kernel) from a profile build:
    bash scripts/build_variant.sh gpprof -DPSK_GP_PROF
    PSK_LIBRARY=tools/bin/ab_gpprof/libpsk.so python tools/gp_prof.py [--m 8192]
Runs AMG applies on -FD m^2 (5 levels) and reads the last launch's per-band records: start lag between
consecutive bands, per-step time of each sweep, and the cycles each wave spent waiting. One JSON line."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--levels", type=int, default=5)
    a = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    m = a.m
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, m).to_scipy()
    dA = psk.DeviceCSR.from_scipy(A)
    M = psk.AMG(numIters=2, numLevels=a.levels).form(dA)
    v = psk.DeviceVector.from_numpy(np.random.default_rng(1).standard_normal(m * m))
    for _ in range(2):
        M.apply(v)
    N.check(N.lib.psk_synchronize(), "sync")
    nb = (m + 62) // 63
    buf = (ctypes.c_ulonglong * (16 * nb))()
    rd = N.lib.psk_gp_prof_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert rd(buf, nb) == 0
    r = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 16).astype(np.float64)
    t0 = r[:, 0].min()
    start, e0, e1 = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0, (r[:, 2] - t0) / 100.0   # us
    S = m + 63
    out = {"m": m, "nbands": nb, "launch_us": float(max(e0.max(), e1.max())),
           "band_start_lag_us_median": float(np.median(np.diff(start))),
           "band_start_lag_us_p10_p90": [float(np.percentile(np.diff(start), 10)), float(np.percentile(np.diff(start), 90))],
           "sweep1_us_per_step_median": float(np.median((e0 - start) / S)),
           "sweep2_end_after_sweep1_us_median": float(np.median(e1 - e0)),
           "wait_cycles_median": {k: float(np.median(r[:, i])) for k, i in
                                  (("ring", 3), ("ext_dx1", 4), ("sweep1_progress", 5), ("ext_dx2", 6))},
           "residual_wave": {"busy_frac_median": float(np.median(1 - (r[:, 11] + r[:, 12]) / np.maximum(r[:, 10], 1))),
                             "wait_sweep1_cycles_median": float(np.median(r[:, 11])),
                             "wait_ext_cycles_median": float(np.median(r[:, 12]))},
           "sweep1_busy_frac_band0": float(1 - (r[0, 3] + r[0, 4]) / max(r[0, 8], 1)),
           "sweep2_busy_frac_band0": float(1 - (r[0, 5] + r[0, 6]) / max(r[0, 9], 1)),
           "residual_busy_frac_band0": float(1 - (r[0, 11] + r[0, 12]) / max(r[0, 10], 1)),
           "xcd_counts": np.bincount(r[:, 7].astype(int), minlength=8).tolist(),
           "band0_raw": [int(x) for x in r[0]], "band1_raw": [int(x) for x in r[1]],
           "first_bands": [[round(float(x), 1) for x in (start[i], e0[i], e1[i])] for i in range(min(6, nb))]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
