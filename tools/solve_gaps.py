#!/usr/bin/env python3
"""Kernel timeline of each PCG solve in a rocprofv3 --kernel-trace CSV (lab tool).

    python tools/solve_gaps.py run_kernel_trace.csv [--iters 20] [--min-grid 1000]

Splits the trace at every pcg_init_kernel launch, keeps the solves with exactly --iters SpMV launches of
a large grid, and prints per solve: the GPU span from the init's start to the last kernel's end, the sum
of kernel durations by kernel family, and the idle time between consecutive kernels (the first gaps and
the tail separately: what a short solve pays beyond its iterations).
"""
import argparse
import csv
import json
import re
import statistics


def family(name):
    for key in ("pcg_init_kernel", "spmv_", "pcg_update_kernel", "pcg_direction_kernel", "gridsum_counter_check",
                "pcg_flush", "pcg_init_finish", "pcg_finish_kernel"):
        if key in name:
            return key.rstrip("_")
    m = re.match(r"(?:void )?(?:psk::)?([A-Za-z0-9_]+)", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"])))
    rows.sort()
    solves, cur = [], None
    for r in rows:
        if r[2] == "pcg_init_kernel":
            cur = [r]
            solves.append(cur)
        elif cur is not None:
            cur.append(r)
    res = []
    for sv in solves:
        # the solve ends at its finish kernel (state + gridsum checks; round 4: the counter check kernel)
        end = next((i for i, r in enumerate(sv) if r[2] in ("pcg_finish_kernel", "gridsum_counter_check")), None)
        if end is None:
            continue
        sv = sv[:end + 1]
        if sum(1 for r in sv if r[2] == "spmv") != a.iters:
            continue
        gaps = [sv[i + 1][0] - sv[i][1] for i in range(len(sv) - 1)]
        fam = {}
        for s, e, f in sv:
            fam[f] = fam.get(f, 0) + (e - s)
        res.append({"span_us": (sv[-1][1] - sv[0][0]) / 1e3, "kernels_us": sum(e - s for s, e, _ in sv) / 1e3,
                    "gaps_us": sum(gaps) / 1e3, "first_gaps_us": [g / 1e3 for g in gaps[:6]],
                    "last_gaps_us": [g / 1e3 for g in gaps[-4:]],
                    "by_kernel_us": {k: v / 1e3 for k, v in fam.items()}})
    out = {"solves": len(res)}
    if res:
        for key in ("span_us", "kernels_us", "gaps_us"):
            out["median_" + key] = statistics.median(r[key] for r in res)
        out["median_solve"] = sorted(res, key=lambda r: r["span_us"])[len(res) // 2]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
