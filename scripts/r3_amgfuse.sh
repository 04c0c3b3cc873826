#!/bin/bash
# Round 3: AMG smoother x += U^-1 r fused into the trisolve's last gather, x = copy(b) fused into the
# ||b||^2 pass: AMG GPU tests, then configs[4] with the fusion on / off (PSK_AMG_FUSE), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_configs.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3af_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3af_pytest.log; grep -E "^FAILED|Error" $OUT/r3af_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
A="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --general 0 --config1 0 --config2 0 --gmres 0 --scaling-side 0"
for v in 1 0 1 0; do
  PSK_AMG_FUSE=$v timeout -k 10 400 python bench.py $A > $OUT/r3af_bench_$v.json 2> $OUT/r3af_bench_$v.err || { tail -3 $OUT/r3af_bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r3af_bench_$v.json'));c=d['configs4_pcg_amg_8192'];print('fuse=$v', round(c['pcg_it_per_s'],3), 'apply', round(c['amg_apply_ms'],2), 'fineGS', round(c['fine_gs_sweep']['ms'],3))"
done
