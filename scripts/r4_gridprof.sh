#!/bin/bash
# Grid schedule per-band timeline (a -DPSK_GRID_PROF build: s_memtime start / end, waits on the band above)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4gp}
for l3 in 0 1; do
  PSK_LIBRARY=$PWD/tools/bin/ab_gridprof/libpsk.so timeout -k 10 300 python -u tools/grid_probe.py --side 8192 --level3 $l3 > $OUT/${TAG}_$l3.json 2>> $OUT/${TAG}.err
  c=$?; echo "l3=$l3 exit $c"; [ $c -eq 0 ] || exit $c
done
