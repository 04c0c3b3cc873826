#!/bin/bash
# Round 3 session 4: the GPU suite on the current build, then the N = 10M headline A/B
# (dot-mode batch vs plain, in-loop) against the round-2 build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
if [ "${TESTS:-1}" = 1 ]; then
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/r3s4_pytest.log 2>&1
rc=$?; tail -4 $OUT/r3s4_pytest.log; [ $rc -le 1 ] || exit $rc
fi
for v in new r2; do
  L=pysolvers_amd/_lib/libpsk.so; [ $v = r2 ] && L=tools/bin/ab_r2/libpsk.so
  for MODE in 0 1; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 300 python bench.py --steps 200 --repeats 5 --cpu-iters 0 --general 0 \
      --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 > $OUT/r3s4_${v}_mode$MODE.json 2> $OUT/r3s4_${v}_mode$MODE.err || exit $?
    python -c "import json;d=json.load(open('$OUT/r3s4_${v}_mode$MODE.json'));print('$v mode $MODE it/s %.1f'%d['value'],'loop %.4f'%d['roofline']['avg_launch_ms'],'batch %.4f'%d['spmv_plain_batch50']['avg_launch_ms'],'noev %.1f'%d['regions_without_kernel_events']['median_it_s'])"
  done
done
