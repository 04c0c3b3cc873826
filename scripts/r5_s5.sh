#!/bin/bash
# Round-5 session 5: the one-round-trip diagonal SpMV (flag, presence bytes and gathers issued together,
# tickets drawn while they fly) — layout/parity tests, then A/B against the previous build and the
# persistent variant, and its per-workgroup timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s5}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -3 $OUT/${TAG}_tests.log; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 prev=@tools/bin/ab_prev/libpsk.so spmv=@tools/bin/ab_spmv/libpsk.so base= persist=PSK_SPMV_PERSIST=1 persist4=PSK_SPMV_PERSIST=1,PSK_SPMV_PERSIST_PER_CU=4 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
ok $c || exit $c
PSK_LIBRARY=tools/bin/ab_sprof/libpsk.so timeout -k 10 180 python -u tools/spmv_probe.py > $OUT/${TAG}_spmvprobe.jsonl 2> $OUT/${TAG}_spmvprobe.err
c=$?; echo "spmv probe exit $c"; cat $OUT/${TAG}_spmvprobe.jsonl
