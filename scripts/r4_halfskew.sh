#!/bin/bash
# Half-integer grid skew (g(y) = (sigma2*y + phase) >> 1): the triangular-solve GPU tests, then configs[4]
# (PCG + AMG, -FD 8192^2) with the half skew off / on, alternating, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4hs}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_amg.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
for r in 1 2; do
  for hs in 0 1; do
    PSK_GRID_HALF_SKEW=$hs PSK_NO_TORCH=1 timeout -k 10 400 python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_hs${hs}_$r.json 2> $OUT/${TAG}_hs${hs}_$r.err
    c=$?; echo "half-skew $hs round $r exit $c $(cat $OUT/${TAG}_hs${hs}_$r.json)"; [ $c -eq 0 ] || exit $c
  done
done
