#!/bin/bash
# Round-5 session 6: K0/K2/K3 with element pairs per lane (PSK_PCG_PL) and flush-specialised K3 —
# parity/layout tests, then A/B: previous builds, PL 1 / 2 (default) / 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s6}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -3 $OUT/${TAG}_tests.log; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 spmv=@tools/bin/ab_spmv/libpsk.so pl1=@tools/bin/ab_pl1/libpsk.so base= pl4=@tools/bin/ab_pl4/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
ok $c || exit $c
timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed.json 2> $OUT/${TAG}_fixed.err
c=$?; echo "fixed exit $c"; cat $OUT/${TAG}_fixed.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python -u tools/fixed_cost.py --iters 20,200 --reps 5 > $OUT/${TAG}_fixedprof.json 2> $OUT/${TAG}_fixedprof.err
c=$?; echo "profiled exit $c"; ok $c || exit $c
python tools/solve_gaps.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) --iters 20 > $OUT/${TAG}_gaps.json
head -30 $OUT/${TAG}_gaps.json
cp $(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_kernel_stats.csv
rm -rf $OUT/${TAG}_prof
