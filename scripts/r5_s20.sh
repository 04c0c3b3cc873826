#!/bin/bash
# Round-5 session 20: cache policy of the PCG loop's Ap (the SpMV's dot-mode y store and K2's Ap load):
# non-temporal (in-tree) vs default policy, same-box A/B at N = 10M and 16384^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s20}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= yplain=@tools/bin/ab_yplain/libpsk.so yk2=@tools/bin/ab_yk2/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
exit $c
