#!/bin/bash
# Round 3: the grid kernel's NB path (DPP neighbour, no LDS ring round trip): grid tests, the FD 8192^2
# Gauss-Seidel sweep with NB on / off, and the configs[4] PCG+AMG bench key
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py -x -q -p no:cacheprovider -k "grid or gs or amg" --timeout 300 --timeout-method thread > $OUT/r3nb_pytest.log 2>&1
rc=$?; tail -3 $OUT/r3nb_pytest.log; grep -E "^FAILED|Error" $OUT/r3nb_pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/grid_probe.py --side 8192 > $OUT/r3nb_grid.json 2>&1 || exit $?
cut -c1-400 $OUT/r3nb_grid.json
PSK_TRISOLVE_GRID_NB=0 timeout -k 10 300 python tools/grid_probe.py --side 8192 > $OUT/r3nb_grid_off.json 2>&1 || exit $?
cut -c1-400 $OUT/r3nb_grid_off.json
timeout -k 10 600 python bench.py --steps 200 --repeats 5 --cpu-iters 0 --general 0 --scaling-side 0 --config1 0 --config2 0 --config4 1 --gmres 0 > $OUT/r3nb_bench.json 2> $OUT/r3nb_bench.err || exit $?
python -c "import json;d=json.load(open('$OUT/r3nb_bench.json'));print(json.dumps(d['configs4_pcg_amg_8192']))"
