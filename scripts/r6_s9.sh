#!/bin/bash
# Round-6 session 9: the pair-row fused PCG init — layout / parity / smoke tests, then the short-solve timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s9}
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py tests/test_gpu_smoke.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
bash scripts/r6_s8.sh ${TAG}tl
