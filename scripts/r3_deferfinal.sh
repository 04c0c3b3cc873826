#!/bin/bash
# the SpMV grid sum's final stage deferred to K2: A/B against the in-launch final stage (same library,
# PSK_PCG_DEFER_FINAL=0), then the GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for R in 1 2 3; do
for DF in 1 0; do
  PSK_PCG_DEFER_FINAL=$DF timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 0 --scaling-side 0 > gpurun_out/r3df_b.json 2> gpurun_out/r3df_b.err || { tail -5 gpurun_out/r3df_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3df_b.json'));print('defer_final=$DF', 'it/s %.1f'%d['value'], 'spmv %.4f'%d['roofline']['avg_launch_ms'], 'noev %.1f'%d.get('regions_without_kernel_events',{}).get('median_it_s'))"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3df_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3df_tests.log; exit $rc
