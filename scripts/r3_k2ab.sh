#!/bin/bash
# K2 with the LDS-combined tile gridsum vs the previous build (block_sum + gridsum_publish)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread 2>&1 | tail -1
for i in 1 2; do for L in pysolvers_amd/_lib/libpsk.so tools/bin/ab_prev/libpsk.so; do
  PSK_LIBRARY=$L timeout -k 10 300 python bench.py --steps 200 --repeats 5 --cpu-iters 0 --general 0 --scaling-side 16384 --config1 0 --config2 0 --config4 0 --gmres 0 > $OUT/r3k2_$i.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('$OUT/r3k2_$i.json'));print('$L it/s %.1f'%d['value'],'loop %.4f'%d['roofline']['avg_launch_ms'],'noev %.1f'%d['regions_without_kernel_events']['median_it_s'],'16384 %.1f'%d['strong_scaling_16384']['pcg_it_per_s'])"
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3k2_prof -o run --output-format csv -- python bench.py --steps 200 --repeats 2 --cpu-iters 0 --general 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 > /dev/null 2>&1 || exit $?
python tools/trace_stats.py $(find $OUT/r3k2_prof -name "*kernel_trace.csv" | head -1) | head -5 | cut -c1-60,200-
