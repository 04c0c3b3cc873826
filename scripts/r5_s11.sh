#!/bin/bash
# Round-5 session 11: is a launch that must recycle workgroups dispatched beside occupiers (dispatch probe
# kernel, 147 KiB LDS like the grid schedule)? AMG level 1 (-FD 8192^2) under the partitioned schedule at
# 256 / 64 / 32 / 16 strips; the remaining GPU test file.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s11}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 120 python -u tools/progress_probe.py --dispatch 32,150528,300 --wgs 192,240,248 --seconds 3 > $OUT/${TAG}_dispatch.jsonl 2> $OUT/${TAG}_dispatch.err
c=$?; echo "dispatch exit $c"; cat $OUT/${TAG}_dispatch.jsonl; tail -2 $OUT/${TAG}_dispatch.err; ok $c || exit $c
timeout -k 10 120 python -u tools/progress_probe.py --dispatch 64,16384,300 --wgs 240,248 --seconds 3 >> $OUT/${TAG}_dispatch.jsonl 2>> $OUT/${TAG}_dispatch.err
c=$?; echo "dispatch2 exit $c"; tail -3 $OUT/${TAG}_dispatch.jsonl; ok $c || exit $c
timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --strips 256,64,32,16 > $OUT/${TAG}_level1.jsonl 2> $OUT/${TAG}_level1.err
c=$?; echo "level1 exit $c"; cat $OUT/${TAG}_level1.jsonl; tail -3 $OUT/${TAG}_level1.err; ok $c || exit $c
timeout -k 10 300 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -2 $OUT/${TAG}_tests.log
