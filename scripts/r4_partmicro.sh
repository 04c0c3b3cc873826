#!/bin/bash
# partitioned triangular solve: per-phase stamps of an LDS hand-off chain (a -DPSK_PART_PROF build), and
# the same chains timed on the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4pm}
PSK_LIBRARY=$PWD/tools/bin/ab_partprof/libpsk.so PART_MICRO_CASES=chain1 timeout -k 10 300 python -u tools/part_micro.py > $OUT/${TAG}_prof.json 2> $OUT/${TAG}_prof.err
c=$?; echo "part_micro (probe build) exit $c"; cat $OUT/${TAG}_prof.json; [ $c -eq 0 ] || exit $c
timeout -k 10 300 python -u tools/part_micro.py > $OUT/${TAG}.json 2> $OUT/${TAG}.err
c=$?; echo "part_micro exit $c"; cat $OUT/${TAG}.json; exit $c
