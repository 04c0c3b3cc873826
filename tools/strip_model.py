#!/usr/bin/env python3
"""Host model of the strip triangular-solve schedule (lab tool; restates ilu.hip plan_strip):
strips of the natural index, rows in ASAP order packed greedily into steps of <= 64 independent
rows, then an event simulation of the solve (a step starts when its strip's previous step ended
and every external dependency was published + the cross-CU hand-off). Checks that every local
dependency sits in an earlier step and that the simulation never deadlocks.

    python tools/strip_model.py M [step_us entry_us remote_us]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ilu_dag import factors, strict  # noqa: E402


def plan(T, lower, nat, P, prio_step=0.25, prio_remote=1.5, chunk=1024):
    n = T.shape[0]
    ip, ix = T.indptr, T.indices
    s = (nat.astype(np.int64) * P) // n
    per = max(1, P // 8)
    wg = ((s % 8) * per + s // 8) if P % 8 == 0 else s
    order = range(n) if lower else range(n - 1, -1, -1)
    fin = np.zeros(n)
    for i in order:
        t = 0.0
        for j in ix[ip[i]:ip[i + 1]]:
            c = prio_step if wg[j] == wg[i] else prio_remote
            if fin[j] + c > t:
                t = fin[j] + c
        fin[i] = t
    pos = np.arange(n) if lower else n - 1 - np.arange(n)
    idx = np.lexsort((pos, fin, wg))
    stepid = np.full(n, -1, dtype=np.int64)
    steps = []   # (strip, rows, E)
    cur = None
    lo = 0.0
    for i in idx:
        w = wg[i]
        ln = ip[i + 1] - ip[i]
        deps = ix[ip[i]:ip[i + 1]]
        if cur is None or cur[0] != w or len(cur[1]) == 64 or max(cur[2], ln) * (len(cur[1]) + 1) > chunk or \
                any(stepid[j] == len(steps) - 1 and wg[j] == w for j in deps) or \
                any(wg[j] != w and fin[j] >= lo for j in deps):
            cur = [w, [], 0]
            steps.append(cur)
            lo = fin[i]
        cur[1].append(i)
        cur[2] = max(cur[2], ln)
        stepid[i] = len(steps) - 1
    for k, (w, rows, E) in enumerate(steps):   # local dependencies in earlier steps
        for i in rows:
            for j in ix[ip[i]:ip[i + 1]]:
                assert wg[j] != w or stepid[j] < k
    return wg, fin, steps, stepid


def simulate(T, wg, steps, stepid, P, step_us, entry_us, remote_us):
    n = T.shape[0]
    ip, ix = T.indptr, T.indices
    done = np.full(n, np.nan)
    by_strip = [[] for _ in range(P)]
    for k, st in enumerate(steps):
        by_strip[st[0]].append(k)
    head = [0] * P
    tfree = [0.0] * P
    left = len(steps)
    while left:
        progressed = False
        for w in range(P):
            while head[w] < len(by_strip[w]):
                k = by_strip[w][head[w]]
                _, rows, E = steps[k]
                t = tfree[w]
                ok = True
                for i in rows:
                    for j in ix[ip[i]:ip[i + 1]]:
                        if wg[j] != w:
                            if np.isnan(done[j]):
                                ok = False
                                break
                            t = max(t, done[j] + remote_us)
                    if not ok:
                        break
                if not ok:
                    break
                t += step_us + E * entry_us
                for i in rows:
                    done[i] = t
                tfree[w] = t
                head[w] += 1
                left -= 1
                progressed = True
        assert progressed, "deadlock"
    return float(np.nanmax(done))


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    step_us, entry_us, remote_us = [float(a) for a in sys.argv[2:5]] if len(sys.argv) > 4 else (0.12, 0.012, 1.2)
    L, U, pr, pc = factors(m)
    n = m * m
    nat_l = np.empty(n, dtype=np.int64)
    nat_l[pr] = np.arange(n)   # L row k <-> equation perm_r^-1 ... (row of the permuted system)
    nat_u = np.empty(n, dtype=np.int64)
    nat_u[pc] = np.arange(n)
    for name, T, lower, nat in (("L", strict(L, True), True, nat_l), ("U", strict(U, False), False, nat_u)):
        P = 256
        wg, fin, steps, stepid = plan(T, lower, nat, P)
        nst = np.bincount([s[0] for s in steps], minlength=P)
        t = simulate(T, wg, steps, stepid, P, step_us, entry_us, remote_us)
        rows_per_step = n / len(steps)
        print("%s m=%d: steps %d (per strip max %d mean %.0f), rows/step %.1f, simulated %.2f ms" %
              (name, m, len(steps), nst.max(), nst.mean(), rows_per_step, t / 1e3))


if __name__ == "__main__":
    main()
