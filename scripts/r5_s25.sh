#!/bin/bash
# Round-5 session 25: slices per workgroup of the diagonal-layout SpMV (kDiagTpw 2, in-tree) vs 1 and 3
# (PSK_DIAG_TPW builds), same-box A/B at N = 10M and 16384^2 (20- and 200-iteration regions).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s25}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 tpw2= tpw1=@tools/bin/ab_tpw1/libpsk.so tpw3=@tools/bin/ab_tpw3/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
exit $c
