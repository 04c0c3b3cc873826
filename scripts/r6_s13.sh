#!/bin/bash
# round 6: timing probe of the paired sweep chains with a check-free Markstein quotient (not a product path)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s13}
timeout -k 10 400 python -u tools/amg_pair_ab.py --rounds 1 > $OUT/${TAG}_base.json 2> $OUT/${TAG}_base.err
c=$?; cat $OUT/${TAG}_base.json; [ $c -eq 0 ] || exit $c
PSK_LIBRARY=tools/bin/ab_mkprobe/libpsk.so timeout -k 10 400 python -u tools/amg_pair_ab.py --rounds 1 --no-lab > $OUT/${TAG}_mk.json 2> $OUT/${TAG}_mk.err
c=$?; cat $OUT/${TAG}_mk.json; exit $c
