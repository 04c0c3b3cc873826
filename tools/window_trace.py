#!/usr/bin/env python3
"""Kernel time inside one window of a rocprofv3 --kernel-trace CSV (development tool).

    python tools/window_trace.py run_kernel_trace.csv MARKER [run_memory_copy_trace.csv]

The window starts at the LAST launch whose kernel name contains MARKER (e.g. `pcg_gen_init` for the
last PCG solve of tools/bench_amg.py) and runs to the end of the trace. Prints the window's wall
span, busy time (union of kernel and copy intervals), idle gaps, and per-(kernel, workgroups) sums.
"""
import collections
import csv
import sys


def rows(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        if kind == "kernel":
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            name = "%s [%d wg]" % (r["Kernel_Name"][:110], grid // max(wg, 1))
        else:
            name = "copy %s" % r.get("Direction", r.get("Operation", "?"))
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return out


def main(path, marker, copies=None):
    ks = sorted(rows(path, "kernel"))
    starts = [i for i, k in enumerate(ks) if marker in k[2]]
    if not starts:
        raise SystemExit("marker %r not found" % marker)
    t0 = ks[starts[-1]][0]
    ev = [k for k in ks if k[0] >= t0]
    if copies:
        ev += [c for c in rows(copies, "copy") if c[0] >= t0]
    ev.sort()
    t1 = max(e[1] for e in ev)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print("window %.3f ms, busy %.3f ms, idle %.3f ms in %d gaps (largest %.3f ms), %d events" %
          ((t1 - t0) / 1e6, busy / 1e6, sum(gaps) / 1e6, len(gaps), max(gaps or [0]) / 1e6, len(ev)))
    agg = collections.defaultdict(list)
    for s, e, n in ev:
        agg[n].append(e - s)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print("%9.3f ms %5d x %8.1f us  %s" % (sum(v) / 1e6, len(v), sum(v) / len(v) / 1e3, n))
    big = sorted(gaps, reverse=True)[:10]
    print("largest gaps (us):", ["%.1f" % (g / 1e3) for g in big])


if __name__ == "__main__":
    main(*sys.argv[1:4])
