#!/bin/bash
# Round-5 session 17: fused K3 + SpMV variants (PSK_PCG_FUSED_VARIANT 1: one slice per workgroup, 2: a 64-VGPR
# cap, 3: both) against the separate launches (PSK_PCG_FUSED=0), after the fused-path tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s17}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or maxiter or breakdown or gridsum or run_to_run" -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -5; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 f0=PSK_PCG_FUSED=1 f1=PSK_PCG_FUSED_VARIANT=1 f2=PSK_PCG_FUSED_VARIANT=2 f3=PSK_PCG_FUSED_VARIANT=3 sep=PSK_PCG_FUSED=0 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
exit $c
