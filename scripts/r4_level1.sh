#!/bin/bash
# configs[4] hierarchy: every level's Gauss-Seidel factor under each schedule with the partitioned layouts
# built (PSK_TRISOLVE_PART=1), then the partitioned LDS hand-off with and without the spin's s_sleep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
PSK_NO_TORCH=1 PSK_TRISOLVE_PART=1 timeout -k 10 600 python -u tools/level_sched_probe.py --side 8192 > $OUT/r4_levels_part.jsonl 2> $OUT/r4_levels_part.err
c=$?; echo "levels exit $c"; cat $OUT/r4_levels_part.jsonl; [ $c -eq 0 ] || exit $c
for v in base sl0; do
  if [ $v = sl0 ]; then export PSK_LIBRARY=$PWD/tools/bin/ab_partsl0/libpsk.so; else unset PSK_LIBRARY; fi
  PART_MICRO_CASES=chain1,chain64+1 timeout -k 10 300 python -u tools/part_micro.py > $OUT/r4_pm_$v.json 2>> $OUT/r4_pm.err
  c=$?; echo "$v exit $c"; cat $OUT/r4_pm_$v.json; [ $c -eq 0 ] || exit $c
done
