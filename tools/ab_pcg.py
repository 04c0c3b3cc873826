#!/usr/bin/env python3
"""Same-box A/B of libpsk variants on the bench's PCG+Jacobi systems (lab tool, not the bench).

    python tools/ab_pcg.py --sides 3163,16384 --rounds 2 \
        base= tpw2=PSK_SPMV_TPW=2 k3pnt=@tools/bin/ab_k3pnt/libpsk.so

Each VARIANT is NAME=[@LIBPATH][,ENV=VALUE...]; every (round, variant) runs in a fresh process (the
library reads its switches once), interleaved, and prints one JSON line per run: PCG it/s (median of
3 regions of --steps iterations, sampled dispatch events), in-loop SpMV ms, 50 back-to-back plain SpMV
launches, and bit-checks (the final recursive residual and a solution checksum) so variants that
change the arithmetic show up.
"""
import argparse
import ctypes
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(sides, steps):
    sys.path.insert(0, REPO)
    import numpy as np
    import bench
    from pysolvers_amd import _native as N
    N.check(N.lib.psk_set_device(0), "set_device")
    out = {}
    for m in sides:
        s = bench.PcgSystem(N, m, None, 1)
        regs = s.regions(steps, 20, 3, lambda: None, None)
        regs.sort()
        dt, sms, _ = regs[len(regs) // 2]
        bms = ctypes.c_double()
        N.check(N.lib.psk_spmv_timed(s.A, s.db, s.dsol, 50, ctypes.byref(bms)), "spmv_timed")
        res = s.run(steps, False)
        x = np.empty(s.nloc)
        N.check(N.lib.psk_d2h(N.ptr(x), s.dsol, s.nloc * 8), "d2h")
        blay, _, _ = s.layout()
        out[str(m)] = {"it_s": steps / dt, "regions_it_s": [steps / r[0] for r in regs], "spmv_ms": sms,
                       "spmv_frac": blay / (sms * 1e-3) / 8e12, "plain_ms": bms.value,
                       "resid_bits": float(res.resid_recursive).hex(),
                       "x_sha": hashlib.sha256(x.tobytes()).hexdigest()[:16]}
        s.free()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sides", default="3163")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    sides = [int(v) for v in a.sides.split(",")]
    if a.child:
        child(sides, a.steps)
        return
    for r in range(a.rounds):
        for v in a.variants:
            name, _, spec = v.partition("=")
            env = dict(os.environ)
            for item in filter(None, spec.split(",")):
                if item.startswith("@"):
                    env["PSK_LIBRARY"] = os.path.join(REPO, item[1:])
                else:
                    k, _, val = item.partition("=")
                    env[k] = val
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--sides", a.sides,
                                "--steps", str(a.steps)], env=env, capture_output=True, text=True, timeout=600)
            line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 and p.stdout.strip() else None
            print(json.dumps({"round": r, "variant": name, "rc": p.returncode,
                              "result": json.loads(line) if line else p.stderr[-800:]}), flush=True)
            if p.returncode != 0:
                sys.exit(p.returncode)


if __name__ == "__main__":
    main()
