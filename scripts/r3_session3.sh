#!/bin/bash
# Round 3 session 3: configs[3] tests at size, the multirank suite (halo overlap cases included),
# N=2 host-transport rehearsals of bench.py at FD 4096^2 with the halo overlap off and on (the
# round-2 failure: an expired gridsum wait), and the dot-mode SpMV batch vs plain at N = 10M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs3.py tests/test_gpu_multirank.py -x -v -p no:cacheprovider \
  --timeout 600 --timeout-method thread > $OUT/r3s3_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/r3s3_pytest.log | tail -15; [ $rc -le 1 ] || exit $rc
for OV in 0 1; do
  echo "== rehearsal N=2 4096^2 overlap=$OV"
  PSK_HALO_OVERLAP=$OV PSK_BENCH_TRANSPORT=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 2953$OV bench.py --gpus 2 --side 4096 --steps 50 --warmup 5 --repeats 3 \
    --scaling-side 0 --cpu-iters 0 > $OUT/r3s3_rehearsal_ov$OV.json 2> $OUT/r3s3_rehearsal_ov$OV.err
  rc=$?; grep -h PskError $OUT/r3s3_rehearsal_ov$OV.err | head -3
  python -c "import json;d=json.load(open('$OUT/r3s3_rehearsal_ov$OV.json'));print('it/s',d['value'],d['repeats']['it_s'])" || true
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "== dot-mode batch vs plain, N=10M"
for MODE in 0 1; do
  PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 300 python bench.py --steps 100 --repeats 3 --cpu-iters 0 --general 0 --scaling-side 0 \
    --config1 0 --config2 0 --config4 0 --gmres 0 > $OUT/r3s3_mode$MODE.json 2> $OUT/r3s3_mode$MODE.err || exit $?
  python -c "import json;d=json.load(open('$OUT/r3s3_mode$MODE.json'));print('mode $MODE it/s %.1f'%d['value'],'loop %.4f'%d['roofline']['avg_launch_ms'],'batch %.4f'%d['spmv_plain_batch50']['avg_launch_ms'],'noev %.1f'%d['regions_without_kernel_events']['median_it_s'])"
done
