#!/bin/bash
# Round 3 session 9: grid record dictionary (tests + the FD 8192^2 sweep / AMG bench), then the
# profiling evidence of the build (scripts/r3_profile.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3s9_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3s9_pytest.log; grep -E "^FAILED|Error" $OUT/r3s9_pytest.log | head -5; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/grid_probe.py --side 8192 > $OUT/r3s9_grid.json 2>&1 || exit $?
cat $OUT/r3s9_grid.json | cut -c1-300
PSK_TRISOLVE_GRID_DICT=0 timeout -k 10 300 python tools/grid_probe.py --side 8192 > $OUT/r3s9_grid_nodict.json 2>&1 || exit $?
cat $OUT/r3s9_grid_nodict.json | cut -c1-300
timeout -k 10 600 python bench.py --steps 200 --repeats 5 --cpu-iters 0 --general 0 --scaling-side 0 --config1 0 --config2 0 --config4 1 --gmres 0 > $OUT/r3s9_bench.json 2> $OUT/r3s9_bench.err || exit $?
python -c "import json;d=json.load(open('$OUT/r3s9_bench.json'));print(json.dumps(d['configs4_pcg_amg_8192']))"
bash scripts/r3_gslab2.sh
