#!/bin/bash
# Same-box A/B of the grid triangular solve: round 3's tree (tools/bin/r3tree: commit 142536b's package
# and libpsk, built here) vs the in-tree build, FD 8192^2 Gauss-Seidel factor (two rounds) and the SA
# level-3 operator (one round).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4g3}
R=$PWD
for r in 1 2; do
  for v in new r3; do
    d=$R; [ $v = r3 ] && d=$R/tools/bin/r3tree
    for l3 in 0 1; do
      [ $l3 = 1 ] && [ $r = 2 ] && continue
      (cd $d && timeout -k 10 300 python -u tools/grid_probe.py --side 8192 --level3 $l3) > $OUT/${TAG}_${v}_${l3}_$r.json 2>> $OUT/${TAG}.err
      c=$?; echo "$v l3=$l3 round $r exit $c $(cat $OUT/${TAG}_${v}_${l3}_$r.json)"; [ $c -eq 0 ] || exit $c
    done
  done
done
