#!/usr/bin/env python3
"""Per-(kernel, grid) durations from a rocprofv3 --kernel-trace CSV.

rocprofv3's --stats summary averages every launch of a kernel name, so a bench that runs the same
kernel at several sizes (bench.py: 16384^2 PCG, the N = 10M SpMV, configs[1] 4096^2) mixes them.
This splits the trace by grid size, the form bench.py's HIP-event averages are compared against:

    python tools/trace_stats.py gpurun_out/prof_TAG/run_kernel_trace.csv > profiles/TAG_kernel_trace_stats.csv
"""
import collections
import csv
import sys


def main(path, top=40):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        agg[(name, grid // max(wg, 1))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in agg.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Workgroups", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs",
                "Percentage"])
    for (name, nwg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        s = sorted(v)
        w.writerow([name, nwg, len(v), sum(v), "%.1f" % (sum(v) / len(v)), s[len(s) // 2], s[0], s[-1],
                    "%.3f" % (100.0 * sum(v) / total)])


if __name__ == "__main__":
    main(sys.argv[1])
