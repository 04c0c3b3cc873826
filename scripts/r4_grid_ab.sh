#!/bin/bash
# Grid schedule round 4b: deferred Markstein range check (conditional IEEE re-solve), published-line
# sentinel fill. GPU tests of the triangular solves first, then the same-box A/B against round 3's tree
# (tools/bin/r3tree) and the configs[4] hierarchy probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4g4}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_part.py tests/test_gpu_amg.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
R=$PWD
for r in 1 2; do
  for v in new r3; do
    d=$R; [ $v = r3 ] && d=$R/tools/bin/r3tree
    (cd $d && timeout -k 10 300 python -u tools/grid_probe.py --side 8192 --level3 0) > $OUT/${TAG}_${v}_$r.json 2>> $OUT/${TAG}.err
    c=$?; echo "$v round $r exit $c $(cat $OUT/${TAG}_${v}_$r.json)"; [ $c -eq 0 ] || exit $c
  done
done
PSK_NO_TORCH=1 timeout -k 10 400 python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; cat $OUT/${TAG}_amg.json; exit $c
