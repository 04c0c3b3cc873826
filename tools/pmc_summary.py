#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc passes (scripts/gpu_pmc.sh), with the gfx950
corrections of MI355X_MICROARCH.md §HBM, verified by tools/pmc_calib.hip:

  read bytes  = FETCH_SIZE[KB] * 1024 * (calibrated read factor; 2.0 = "FETCH reads 1/2")
  write bytes = WRITE_SIZE[KB] * 1024 * (calibrated write factor; 1.0)

    python tools/pmc_summary.py gpurun_out/pmc_TAG_FETCH_SIZE gpurun_out/pmc_TAG_WRITE_SIZE \
        gpurun_out/pmc_TAG_calib_FETCH_SIZE gpurun_out/pmc_TAG_calib_WRITE_SIZE [SIDE "BENCH ARGS" SHA_FILE] > profiles/x.json

SHA_FILE: the `sha256sum` line of the libpsk.so the passes ran with (scripts/gpu_pmc.sh writes it);
bench.py uses a profile only when it matches the library it loaded.
"""
import collections
import csv
import glob
import json
import os
import sys

CALIB_BYTES = 1 << 30


def per_kernel(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main(fetch_dir, write_dir, cal_fetch, cal_write, side=None, bench_args=None, sha_file=None):
    cf, cw = per_kernel(cal_fetch), per_kernel(cal_write)
    rfac = {k.split("(")[0]: CALIB_BYTES / (sum(v) / len(v)) for k, v in cf.items() if k.startswith(("void rd", "rd16"))}
    wfac = {k.split("(")[0]: CALIB_BYTES / (sum(v) / len(v)) for k, v in cw.items() if k.startswith("wr8")}
    read_factor = sum(rfac.values()) / len(rfac)
    write_factor = sum(wfac.values()) / len(wfac)
    fe, wr = per_kernel(fetch_dir), per_kernel(write_dir)
    out = {"read_factor": read_factor, "write_factor": write_factor, "calibration_read": rfac,
           "calibration_write": wfac, "kernels": {}}
    for k in fe:
        rb = sum(fe[k]) / len(fe[k]) * read_factor
        wb = (sum(wr[k]) / len(wr[k]) * write_factor) if k in wr else None
        out["kernels"][k] = {"launches": len(fe[k]), "read_bytes_per_launch": rb,
                             "write_bytes_per_launch": wb,
                             "hbm_bytes_per_launch": rb + (wb or 0.0)}
    if side is not None:
        out["config"] = {"side": int(side), "bench_args": bench_args,
                         "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_pmc.sh), corrected "
                                 "with tools/pmc_calib.hip factors"}
    if sha_file is not None:
        out["libpsk_sha256"] = open(sha_file).read().split()[0]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:8])
