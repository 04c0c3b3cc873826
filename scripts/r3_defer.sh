#!/bin/bash
# x-update deferral depth: GPU suite with the in-tree build (kPcgDefer = 4), then bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3d_tests.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
for L in tools/bin/ab_intree2 tools/bin/ab_defer2 pysolvers_amd/_lib tools/bin/ab_defer8; do
  PSK_LIBRARY=$L/libpsk.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 0 --scaling-side 0 > gpurun_out/r3d_b.json 2> gpurun_out/r3d_b.err || { tail -5 gpurun_out/r3d_b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3d_b.json'));print('$L', 'it/s %.1f'%d['value'], 'spmv %.4f'%d['roofline']['avg_launch_ms'], 'noev %.1f'%d.get('regions_without_kernel_events',{}).get('median_it_s'))"
done
done
