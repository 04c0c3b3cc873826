#!/bin/bash
# rocprofv3 kernel trace + stats of the configs[2] (ILU) and configs[4] (AMG) bench keys of the in-tree build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/r3ai_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 2 \
   --cpu-iters 0 --general 0 --config1 0 --gmres 0 --scaling-side 0 > $OUT/r3ai_prof.json 2> $OUT/r3ai_prof.err; echo "profiled run exit $?"
python tools/trace_stats.py $(find $OUT/r3ai_prof -name "*kernel_trace.csv" | head -1) > $OUT/r3ai_trace_stats.csv
rm -rf $OUT/r3ai_prof
