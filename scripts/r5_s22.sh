#!/bin/bash
# Round-5 session 22: the PCG init fused into the first SpMV on the diagonal layout (spmv.hip
# pcg_init_diag_kernel; pcg_init_kernel over the SpMV's 256-row tiles elsewhere): the GPU suite, then
# same-box A/B against the previous build (a1a5d83e, tools/bin/ab_old) on 20-iteration regions and the
# fixed-cost fit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s22}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 3 new= old=@tools/bin/ab_old/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s %s spmv %.4f %s" % (k, v["it_s"], [round(x) for x in v["regions_it_s"]], v["spmv_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
[ $c -eq 0 ] || exit $c
timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed_new.json 2>&1; echo "fixed new $?"; tail -2 $OUT/${TAG}_fixed_new.json
PSK_LIBRARY=tools/bin/ab_old/libpsk.so timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed_old.json 2>&1; echo "fixed old $?"; tail -2 $OUT/${TAG}_fixed_old.json
