#!/bin/bash
# Round-5 session 14: levels schedule with host-assigned LDS slots (AMG level 1), grid launch capped at one
# workgroup per CU + one-workgroup re-solve; AMG / progress / layout tests, PCG+AMG at -FD 8192^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s14}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_progress.py tests/test_gpu_part.py -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -5; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --use-levels 1 > $OUT/${TAG}_level1.jsonl 2> $OUT/${TAG}_level1.err
c=$?; echo "level1 exit $c"; cat $OUT/${TAG}_level1.jsonl; tail -3 $OUT/${TAG}_level1.err; ok $c || exit $c
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_amgprof -o run --output-format csv -- python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; tail -c 2500 $OUT/${TAG}_amg.json; ok $c || exit $c
cp $(find $OUT/${TAG}_amgprof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_amg_kernel_stats.csv
rm -rf $OUT/${TAG}_amgprof
