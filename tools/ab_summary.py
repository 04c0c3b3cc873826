#!/usr/bin/env python3
"""Print tools/ab_pcg.py's JSON lines as one row per (round, variant, side)."""
import json
import sys

for line in open(sys.argv[1]):
    d = json.loads(line)
    r = d["result"]
    if not isinstance(r, dict):
        print(d["round"], d["variant"], "rc", d["rc"], str(r)[-400:])
        continue
    for side, v in r.items():
        print("%d %-8s %6s: %8.1f it/s  spmv %.4f ms (%.3f)  plain %.4f ms  bits %s/%s" % (
            d["round"], d["variant"], side, v["it_s"], v["spmv_ms"], v["spmv_frac"], v["plain_ms"],
            v["resid_bits"][-6:], v["x_sha"][:6]))
