#!/bin/bash
# Round-5 session 16: the fused K3 + SpMV launch of the PCG loop (spmv.hip pcg_fused_kernel): parity tests
# (fused vs separate launches bitwise, the PCG parity set, the layout set), then a same-box A/B, fused vs
# separate (PSK_PCG_FUSED=0), at N = 10M and 16384^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s16}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -5; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 fused=PSK_PCG_FUSED=1 sep=PSK_PCG_FUSED=0 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
exit $c
