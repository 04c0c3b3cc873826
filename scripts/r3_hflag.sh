#!/bin/bash
# Round 3: PCG convergence polling through a host-mapped done stamp (no per-chunk D2H blit):
# PCG parity / multirank / shard tests, then the N=10M headline with the new scheme and the old
# (PSK_PCG_FLAG_COPY=1), alternated on the same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_shards.py tests/test_gpu_newton.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3hf_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3hf_pytest.log; grep -E "^FAILED|Error" $OUT/r3hf_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
A="--cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 0 --scaling-side 0"
for v in 0 1 0 1; do
  PSK_PCG_FLAG_COPY=$v timeout -k 10 300 python bench.py $A > $OUT/r3hf_bench_$v.json 2> $OUT/r3hf_bench_$v.err || exit $?
  python -c "import json;d=json.load(open('$OUT/r3hf_bench_$v.json'));print('copy=$v', round(d['value'],1), 'noev', round(d['regions_without_kernel_events']['median_it_s'],1), 'spmv', round(d['roofline']['avg_launch_ms']*1000,2))"
done
