#!/bin/bash
# round 6 (session 2): the dense-A parity fixtures (tests/golden/make_dense.py) on the device
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s20}
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dense or zero_rhs" > $OUT/${TAG}_pytest.log 2>&1
c=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/${TAG}_pytest.log | tail -12; exit $c
