#!/usr/bin/env python3
"""The headline regions' SpMV launches in a rocprofv3 --kernel-trace CSV of `bench.py` (evidence tool).

    python tools/region_trace.py run_kernel_trace.csv [--kernel spmv_diag_kernel<1] \
        [--workgroups 19541] [--settle 1999] [--warmup 5] [--steps 20] [--regions 5] [--init-fused 1]

bench.py's first launches of the in-loop SpMV at the headline size are the warmup solve's (`--warmup`
iterations) and the settle solve's (`--settle` iterations: PcgSystem.settle_iters, 1999 at N = 10M), then the
timed regions (`--regions` x `--steps`). With the init fused into the first SpMV (the diagonal layout,
`--init-fused 1`, round 5) a solve of K iterations launches this kernel K - 1 times. Prints the mean duration over exactly those
timed launches, per region, and over every launch of the kernel at that grid in the whole run (what a
`--stats` summary averages), so the bench line's `roofline.avg_launch_ms` (HIP events on every 8th launch of
the median region) can be compared with the profiler on the same launches.
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="spmv_diagp_kernel<1,")
    ap.add_argument("--workgroups", type=int, default=9771)
    ap.add_argument("--settle", type=int, default=1999)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--regions", type=int, default=5)
    ap.add_argument("--init-fused", type=int, default=1)
    a = ap.parse_args()
    launches = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].replace(" ", "")
        if a.kernel.replace(" ", "") not in name:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        if grid // max(wg, 1) != a.workgroups:
            continue
        launches.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    launches.sort()
    durs = [d for _, d in launches]
    f = 1 if a.init_fused else 0
    skip = (a.settle - f) + (a.warmup - f)
    per = a.steps - f   # launches per timed region
    timed = durs[skip:skip + per * a.regions]
    per_region = [statistics.mean(timed[i * per:(i + 1) * per]) / 1e3 for i in range(a.regions)
                  if timed[i * per:(i + 1) * per]]
    print(json.dumps({"kernel": a.kernel, "workgroups": a.workgroups, "launches_in_trace": len(durs),
                      "timed_launches": len(timed),
                      "timed_mean_us": statistics.mean(timed) / 1e3 if timed else None,
                      "timed_per_region_mean_us": per_region,
                      "median_region_mean_us": statistics.median(per_region) if per_region else None,
                      "all_launches_mean_us": statistics.mean(durs) / 1e3 if durs else None}))


if __name__ == "__main__":
    main()
