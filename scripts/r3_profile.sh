#!/bin/bash
# Round 3 evidence: rocprofv3 kernel trace + stats of the bench headline (+ 16384^2 scaling key),
# then the PMC traffic passes at 3163^2 and 16384^2 (scripts/gpu_pmc.sh) of the same libpsk build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum pysolvers_amd/_lib/libpsk.so | tee $OUT/r3_prof_lib.sha256
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r3_prof -o run --output-format csv -- python bench.py --steps 200 --repeats 3 \
   --cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 1 > $OUT/r3_prof_bench.json 2> $OUT/r3_prof_bench.err || exit $?
f=$(find $OUT/r3_prof -name "*kernel_trace.csv" | head -1); python tools/trace_stats.py $f > $OUT/r3_prof_trace_stats.csv
f2=$(find $OUT/r3_prof -name "*kernel_stats.csv" | head -1); cp $f2 $OUT/r3_prof_kernel_stats.csv
python -c "
import csv
for r in list(csv.reader(open('$OUT/r3_prof_trace_stats.csv')))[:14]: print(r[0][:60], r[1:5])"
TAG=r3 SIDES="3163 16384" PMC_ARGS="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0" bash scripts/gpu_pmc.sh || exit $?
