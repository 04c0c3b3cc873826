#!/bin/bash
# After the plain-launch change: the triangular-solve GPU tests, the exit probe (sync-free schedule) and the
# whole bench under rocprofv3 (exit status recorded)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_part.py tests/test_gpu_amg.py tests/test_gpu_configs.py > $OUT/r4xf_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -2 $OUT/r4xf_pytest.log; [ $c -eq 0 ] || exit $c
bash scripts/r4_exit_probe.sh && bash scripts/r4_exit_check.sh config4 && bash scripts/r4_exit_check.sh config2
