#!/bin/bash
# Round 3 final evidence for the committed build: the driver's bench command, a rocprofv3 kernel trace +
# stats of the same headline, and the PMC traffic passes (scripts/gpu_pmc.sh), all of one libpsk.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum pysolvers_amd/_lib/libpsk.so | tee $OUT/r3f_lib.sha256
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r3f_smoke.log 2>&1 || { tail -5 $OUT/r3f_smoke.log; exit 1; }
tail -2 $OUT/r3f_smoke.log
echo "== bench (defaults)"; timeout -k 10 900 python bench.py > $OUT/r3f_bench.json 2> $OUT/r3f_bench.err || { tail -5 $OUT/r3f_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r3f_bench.json'));print('value %.1f'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'), d['roofline'].get('traffic_note'))"
echo "== rocprofv3 kernel trace + stats of the headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r3f_prof -o run --output-format csv -- python bench.py --cpu-iters 0 --general 0 \
   --config1 0 --config2 0 --config4 0 --gmres 1 > $OUT/r3f_prof_bench.json 2> $OUT/r3f_prof_bench.err || exit $?
python tools/trace_stats.py $(find $OUT/r3f_prof -name "*kernel_trace.csv" | head -1) > $OUT/r3f_trace_stats.csv
cp $(find $OUT/r3f_prof -name "*kernel_stats.csv" | head -1) $OUT/r3f_kernel_stats.csv
TAG=r3f SIDES="3163 16384" PMC_ARGS="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0" bash scripts/gpu_pmc.sh || exit $?
