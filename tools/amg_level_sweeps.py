"""Per-level smoother sweep times of configs[4]'s AMG hierarchy (-FD m^2, 5 levels): each level's Gauss-Seidel
operator applied alone (median of 5), with its schedule. Used with a probe build (PSK_LIBRARY=...) to see what the
grid schedule's per-step memory operations cost. One JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    a = ap.parse_args()
    import pysolvers_amd as psk
    from pysolvers_amd import _native as N
    A = -psk.DeviceCSR.fd_laplacian_2d(-1.0, 1.0, a.m).to_scipy()
    dA = psk.DeviceCSR.from_scipy(A)
    M = psk.AMG(numIters=2, numLevels=5).form(dA)
    out = {"m": a.m, "levels": {}}
    for k in range(1, 5):
        S = M._S[k].operator
        n = M.levels()[k]
        v = psk.DeviceVector.from_numpy(np.random.default_rng(k).standard_normal(n))
        S.apply(v)
        ts = []
        for _ in range(5):
            N.check(N.lib.psk_synchronize(), "sync")
            t = time.perf_counter()
            S.apply(v)
            N.check(N.lib.psk_synchronize(), "sync")
            ts.append((time.perf_counter() - t) * 1e3)
        info = S.device_info()
        out["levels"][k] = {"n": n, "schedule": S.schedule("U")["schedule"], "ms": float(np.median(ts)),
                            "dep_levels": info["levels_u"],
                            "us_per_level": float(np.median(ts)) * 1e3 / max(1, info["levels_u"])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
