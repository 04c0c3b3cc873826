#!/bin/bash
# Round-5 session 1: the -m gpu suite on the ADVICE-r4 build, the per-solve fixed cost at N = 10M
# (tools/fixed_cost.py) and its GPU timeline (rocprofv3 kernel trace -> tools/solve_gaps.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s1}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; ok $c || exit $c
timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed.json 2> $OUT/${TAG}_fixed.err
c=$?; echo "fixed exit $c"; cat $OUT/${TAG}_fixed.json; ok $c || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/${TAG}_prof -o run --output-format csv -- \
    python -u tools/fixed_cost.py --iters 20,200 --reps 5 > $OUT/${TAG}_fixedprof.json 2> $OUT/${TAG}_fixedprof.err
c=$?; echo "profiled exit $c"; ok $c || exit $c
python tools/solve_gaps.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) --iters 20 > $OUT/${TAG}_gaps.json
cat $OUT/${TAG}_gaps.json | head -40
rm -rf $OUT/${TAG}_prof
