#!/bin/bash
# Round-5 session 19: the configs[3] / configs[4] full-size tests (true vs reported residual added).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s19}
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_configs3.py -x -v --timeout 600 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; grep -E "PASSED|FAILED|passed|failed|Error" $OUT/${TAG}_tests.log | tail -12; exit $c
