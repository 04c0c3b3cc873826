#!/bin/bash
# Round-5 session 21: the PCG loop's Ap store policy by size (diag_ykeep, spmv.hip): default limit 96 MiB
# vs never (PSK_SPMV_YKEEP_MB=0, non-temporal) vs always, at N = 10M, 4096^2 and 16384^2; the layout tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s21}
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py -k "fd or pcg or layout" -x -q --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -2 $OUT/${TAG}_tests.log; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,4096,16384 --rounds 2 base= never=PSK_SPMV_YKEEP_MB=0 always=PSK_SPMV_YKEEP_MB=65536 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
exit $c
