#!/bin/bash
# Round-5 session 10: the dense coarse GEMV without fences (probe at the coarse level's size), the full GPU
# suite with the DPP neighbour SpMV as default and the reworked grid progress test, PCG+AMG at -FD 8192^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s10}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 240 python -u tools/dense_probe.py --n 16642 --reps 20 > $OUT/${TAG}_dense.jsonl 2> $OUT/${TAG}_dense.err
c=$?; echo "dense exit $c"; cat $OUT/${TAG}_dense.jsonl; tail -3 $OUT/${TAG}_dense.err; ok $c || exit $c
timeout -k 10 240 python -u tools/dense_probe.py --n 16642 --reps 20 --refine 1 >> $OUT/${TAG}_dense.jsonl 2>> $OUT/${TAG}_dense.err
c=$?; echo "dense refine exit $c"; tail -1 $OUT/${TAG}_dense.jsonl; ok $c || exit $c
timeout -k 10 240 python -u tools/progress_probe.py --factor gs --m 2048 --sched grid --wgs 192,240 --seconds 5 > $OUT/${TAG}_probe.jsonl 2> $OUT/${TAG}_probe.err
c=$?; echo "probe exit $c"; cat $OUT/${TAG}_probe.jsonl; ok $c || exit $c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -4 $OUT/${TAG}_tests.log; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_amgprof -o run --output-format csv -- python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; tail -c 1500 $OUT/${TAG}_amg.json; ok $c || exit $c
cp $(find $OUT/${TAG}_amgprof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_amg_kernel_stats.csv
rm -rf $OUT/${TAG}_amgprof
