#!/bin/bash
# whole-line gridsum slots with epoch arrays: timing vs the previous build, then the GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for R in 1 2; do
for L in tools/bin/ab_intree2/libpsk.so pysolvers_amd/_lib/libpsk.so; do
  for MODE in 0 1; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
  done
done
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 0 --scaling-side 0 > gpurun_out/r3l_bench.json 2> gpurun_out/r3l_bench.err || { tail -5 gpurun_out/r3l_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3l_bench.json'));print('bench it/s %.1f'%d['value'], 'spmv %.4f'%d['roofline']['avg_launch_ms'], 'noev', d.get('regions_without_kernel_events',{}).get('median_it_s'))"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r3l_tests.log; exit $rc
