#!/bin/bash
# Round-5 session 26: what K2's grid sums cost (probe builds; their scalars are wrong, their timing is not):
# PSK_LAB_K2_NOSUM (no sums at all), PSK_LAB_K2_NOPUB (the two block sums, no slot store / ticket reduction).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s26}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= nosum=@tools/bin/ab_k2nosum/libpsk.so nopub=@tools/bin/ab_k2nopub/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f" % (k, v["it_s"], v["spmv_ms"]) for k, v in r.items()))
    else: print(d)
PY
exit $c
