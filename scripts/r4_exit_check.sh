#!/bin/bash
# Exit status of the bench under rocprofv3 --kernel-trace --stats with one extra key ($1: config4 | config2 |
# gmres | config1 | general), /proc/self/maps dumped at exit (PSK_DUMP_MAPS) to resolve a fault PC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
KEY=${1:-config4}; TAG=r4x_$KEY
ARGS="--config1 0 --config2 0 --config4 0 --gmres 0 --general 0"
ARGS=${ARGS/--$KEY 0/}
PSK_DUMP_MAPS=$OUT/${TAG}_maps.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_p -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 5 --cpu-iters 0 --scaling-side 0 $ARGS > $OUT/${TAG}.json 2> $OUT/${TAG}.err
c=$?; echo "$KEY exit $c"; grep -a "SIGSEGV\|    @ " $OUT/${TAG}.err | head -24
rm -rf $OUT/${TAG}_p
exit $c
