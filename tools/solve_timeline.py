#!/usr/bin/env python3
"""Where a short psk_pcg call's wall time goes (lab tool, round 6): host monotonic-ns marks around each call of a
few solves at N = 10M, to be read against a `rocprofv3 --runtime-trace --kernel-trace` of the same run (same
CLOCK_MONOTONIC clock): the HIP API calls and kernels inside each mark pair.

    rocprofv3 --runtime-trace --kernel-trace -d OUT -o run --output-format csv -- python tools/solve_timeline.py
    python tools/solve_timeline.py --analyze OUT/.../run_hip_api_trace.csv OUT/.../run_kernel_trace.csv marks.json
"""
import argparse
import csv
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(out, side, iters, reps):
    os.environ.setdefault("PSK_NO_TORCH", "1")
    import bench
    from pysolvers_amd import _native as N
    N.check(N.lib.psk_set_device(0), "set_device")
    s = bench.PcgSystem(N, side, None, 1)
    s.run(20, False)
    s.run(s.settle_iters(), False)
    marks = []
    for k in iters:
        for _ in range(reps):
            N.check(N.lib.psk_synchronize(), "sync")
            t0 = time.monotonic_ns()
            s.run(k, False)
            t1 = time.monotonic_ns()
            N.check(N.lib.psk_synchronize(), "sync")
            t2 = time.monotonic_ns()
            marks.append({"iters": k, "t0": t0, "t1": t1, "t2": t2})
    s.free()
    json.dump(marks, open(out, "w"))


def analyze(api_csv, kern_csv, marks_json):
    marks = json.load(open(marks_json))
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(api_csv))]
    ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kern_csv))]
    rows = []
    for m in marks:
        a = sorted(x for x in api if m["t0"] <= x[0] <= m["t2"])
        k = sorted(x for x in ker if m["t0"] <= x[0] <= m["t2"])
        if not k:
            continue
        first_launch = next((x for x in a if "Launch" in x[2]), None)
        syncs = [x for x in a if "Synchronize" in x[2]]
        rows.append({
            "iters": m["iters"], "call_us": (m["t1"] - m["t0"]) / 1e3, "call_plus_sync_us": (m["t2"] - m["t0"]) / 1e3,
            "to_first_launch_api_us": (first_launch[0] - m["t0"]) / 1e3 if first_launch else None,
            "to_first_kernel_start_us": (k[0][0] - m["t0"]) / 1e3,
            "gpu_span_us": (k[-1][1] - k[0][0]) / 1e3,
            "kernels_busy_us": sum(e - s for s, e, _ in k) / 1e3,
            "last_kernel_end_to_call_return_us": (m["t1"] - k[-1][1]) / 1e3,
            "last_kernels": [x[2].split("(")[0][-40:] for x in k[-3:]],
            "sync_calls_us": [round((e - s) / 1e3, 1) for s, e, f in syncs],
            "api_calls": len(a),
            "first_api": [(x[2], round((x[0] - m["t0"]) / 1e3, 1), round((x[1] - x[0]) / 1e3, 1)) for x in a[:8]],
            "last_api": [(x[2], round((x[0] - m["t0"]) / 1e3, 1), round((x[1] - x[0]) / 1e3, 1)) for x in a[-6:]],
            "kernels": [(x[2].split("(")[0].replace("void ", "")[-44:], round((x[0] - m["t0"]) / 1e3, 1),
                         round((x[1] - x[0]) / 1e3, 1)) for x in (k[:5] + k[-4:])],
        })
    by = {}
    for r in rows:
        by.setdefault(r["iters"], []).append(r)
    for k, rs in by.items():
        med = lambda key: sorted(x[key] for x in rs if x[key] is not None)[len(rs) // 2]
        print(json.dumps({"iters": k, "solves": len(rs), **{key: med(key) for key in (
            "call_us", "call_plus_sync_us", "to_first_launch_api_us", "to_first_kernel_start_us", "gpu_span_us",
            "kernels_busy_us", "last_kernel_end_to_call_return_us", "api_calls")}, "example": rs[len(rs) // 2]}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", nargs=3)
    ap.add_argument("--out", default="gpurun_out/solve_timeline_marks.json")
    ap.add_argument("--side", type=int, default=3163)
    ap.add_argument("--iters", default="0,1,20")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    if a.analyze:
        analyze(*a.analyze)
    else:
        run(a.out, a.side, [int(v) for v in a.iters.split(",")], a.reps)
