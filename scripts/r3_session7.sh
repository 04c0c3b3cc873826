#!/bin/bash
# Round 3 session 7: parity suites touched this round (gridsum per tile, one-shot MGS, exit reasons,
# DefaultDirect), the epilogue lab, and the bench headline + GMRES Arnoldi key.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_newton.py tests/test_gpu_configs.py \
  -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3s7_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3s7_pytest.log; grep -E "^FAILED|Error" $OUT/r3s7_pytest.log | head -5; [ $rc -le 1 ] || exit $rc
for MODE in 0 1; do for M in 3163 16384; do
  PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py $M 100 || exit $?
done; done
timeout -k 10 400 python bench.py --steps 200 --repeats 5 --cpu-iters 0 --general 0 --scaling-side 16384 --config1 0 --config2 0 --config4 0 --gmres 1 > $OUT/r3s7_bench.json 2> $OUT/r3s7_bench.err || exit $?
python -c "
import json;d=json.load(open('$OUT/r3s7_bench.json'))
print('it/s %.1f'%d['value'],'loop %.4f'%d['roofline']['avg_launch_ms'],'batch %.4f'%d['spmv_plain_batch50']['avg_launch_ms'],'noev %.1f'%d['regions_without_kernel_events']['median_it_s'], 's16384 %.1f %.4f'%(d['strong_scaling_16384']['pcg_it_per_s'],d['strong_scaling_16384']['spmv_avg_launch_ms']))
print(json.dumps(d['gmres30_jacobi_4096']))"
bash scripts/r3_gridprobe.sh
