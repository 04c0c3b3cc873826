#!/bin/bash
# Round-5 session 12: the levels triangular-solve schedule (one workgroup, x in an LDS ring) on AMG level 1,
# the grid schedule drawing bands until they run out (progress beside 248 occupiers), AMG / progress tests,
# PCG+AMG at -FD 8192^2 with rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s12}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_progress.py -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -5; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 240 python -u tools/progress_probe.py --factor gs --m 2048 --sched grid --wgs 192,240,248 --seconds 5 > $OUT/${TAG}_probe.jsonl 2> $OUT/${TAG}_probe.err
c=$?; echo "probe exit $c"; cat $OUT/${TAG}_probe.jsonl; ok $c || exit $c
timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --use-levels 1 > $OUT/${TAG}_level1.jsonl 2> $OUT/${TAG}_level1.err
c=$?; echo "level1 exit $c"; cat $OUT/${TAG}_level1.jsonl; tail -3 $OUT/${TAG}_level1.err; ok $c || exit $c
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_amgprof -o run --output-format csv -- python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; tail -c 2000 $OUT/${TAG}_amg.json; ok $c || exit $c
cp $(find $OUT/${TAG}_amgprof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_amg_kernel_stats.csv
rm -rf $OUT/${TAG}_amgprof
