#!/bin/bash
# Round-5 session 15: levels schedule with the fma chain cut at the step's widest row; prefetch depth 4 vs 8
# (PSK_LEVELS_D) on AMG level 1; AMG tests; the multirank tests with the mailbox self-check; PCG x-update
# deferral depth 2 / 3 / 4 / 8 (PSK_PCG_DEFER builds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s15}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -5; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --use-levels 1 > $OUT/${TAG}_level1.jsonl 2> $OUT/${TAG}_level1.err
c=$?; echo "level1 exit $c"; cat $OUT/${TAG}_level1.jsonl; ok $c || exit $c
PSK_LEVELS_D=8 timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --use-levels 1 > $OUT/${TAG}_level1_d8.jsonl 2> $OUT/${TAG}_level1_d8.err
c=$?; echo "level1 d8 exit $c"; cat $OUT/${TAG}_level1_d8.jsonl; ok $c || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= defer2=@tools/bin/ab_defer2/libpsk.so defer3=@tools/bin/ab_defer3/libpsk.so defer8=@tools/bin/ab_defer8/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
