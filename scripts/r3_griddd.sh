#!/bin/bash
# grid-schedule prefetch depth with the record dictionary (PSK_GRID_DD): fine -FD 8192^2 and SA level 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in 1 2; do
for L in pysolvers_amd/_lib tools/bin/ab_dd8 tools/bin/ab_dd16 tools/bin/ab_dd24; do
  for L3 in 0 1; do
    echo -n "$L level3=$L3 "; PSK_LIBRARY=$L/libpsk.so timeout -k 10 300 python tools/grid_probe.py --side 8192 --level3 $L3 || exit $?
  done
done
done
