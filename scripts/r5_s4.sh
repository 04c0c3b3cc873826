#!/bin/bash
# Round-5 session 4: forward-progress tests (occupiers), diagonal-layout slices per workgroup A/B
# (tools/ab_pcg.py, TPW 2 / 4 / 8) and the per-workgroup SpMV timeline of TPW 2 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s4}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -v --timeout 200 --timeout-method thread > $OUT/${TAG}_progress.log 2>&1
c=$?; echo "progress tests exit $c"; grep -E "PASS|FAIL" $OUT/${TAG}_progress.log | tail -6; ok $c || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= tpw4=@tools/bin/ab_dtpw4/libpsk.so tpw8=@tools/bin/ab_dtpw8/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
ok $c || exit $c
PSK_LIBRARY=tools/bin/ab_sprof/libpsk.so timeout -k 10 180 python -u tools/spmv_probe.py > $OUT/${TAG}_spmvprobe2.jsonl 2> $OUT/${TAG}_spmvprobe2.err
c=$?; echo "spmv probe tpw2 exit $c"; cat $OUT/${TAG}_spmvprobe2.jsonl; ok $c || exit $c
PSK_PROBE_TPW=4 PSK_LIBRARY=tools/bin/ab_sprof4/libpsk.so timeout -k 10 180 python -u tools/spmv_probe.py > $OUT/${TAG}_spmvprobe4.jsonl 2> $OUT/${TAG}_spmvprobe4.err
c=$?; echo "spmv probe tpw4 exit $c"; cat $OUT/${TAG}_spmvprobe4.jsonl
