#!/bin/bash
# Round-5 session 13: where the grid schedule's bands run beside 240 / 248 occupiers (-DPSK_GRID_PROF lab build:
# per band XCD, workgroup, start / end), AMG level 1 on the levels schedule, PCG+AMG at -FD 8192^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s13}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
PSK_LIBRARY=tools/bin/ab_gridprof/libpsk.so timeout -k 10 200 python -u tools/progress_probe.py --factor gs --m 2048 --sched grid --wgs 240,248 --seconds 3 > $OUT/${TAG}_probe.jsonl 2> $OUT/${TAG}_probe.err
c=$?; echo "probe exit $c"; cut -c1-600 $OUT/${TAG}_probe.jsonl; tail -2 $OUT/${TAG}_probe.err; ok $c || exit $c
timeout -k 10 600 python -u tools/level_probe.py --side 8192 --levels 5 --level 1 --use-levels 1 > $OUT/${TAG}_level1.jsonl 2> $OUT/${TAG}_level1.err
c=$?; echo "level1 exit $c"; cat $OUT/${TAG}_level1.jsonl; tail -3 $OUT/${TAG}_level1.err; ok $c || exit $c
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_amgprof -o run --output-format csv -- python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; tail -c 2500 $OUT/${TAG}_amg.json; ok $c || exit $c
cp $(find $OUT/${TAG}_amgprof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_amg_kernel_stats.csv
rm -rf $OUT/${TAG}_amgprof
