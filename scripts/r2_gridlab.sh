#!/bin/bash
# builds of libpsk with grid-schedule probes (run on the CPU side first: make with EXTRA flags into
# tools/bin/ab_<name>/) timed with tools/grid_probe.py, each step time-limited
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2g}
mkdir -p $OUT
for v in "$@"; do
  for a in ${PROBE_ARGS:-"--side 8192"}; do :; done
  PSK_LIBRARY=tools/bin/ab_$v/libpsk.so timeout -k 10 300 python tools/grid_probe.py ${PROBE_ARGS:---side 8192} > $OUT/${TAG}_$v.json 2> $OUT/${TAG}_$v.err \
    || { echo "probe $v failed"; tail -5 $OUT/${TAG}_$v.err; exit 1; }
  echo "== $v"; cat $OUT/${TAG}_$v.json
done
