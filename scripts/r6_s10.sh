#!/bin/bash
# round 6: paired Gauss-Seidel sweeps — bitwise vs serialized, the AMG suites, and the 8192^2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s10}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_gs_pair.py > $OUT/${TAG}_pair.log 2>&1
c=$?; tail -15 $OUT/${TAG}_pair.log; [ $c -eq 0 ] || exit $c
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_amg.py tests/test_gpu_configs.py tests/test_gpu_progress.py tests/test_gpu_layout.py -k "amg or AMG or configs4" > $OUT/${TAG}_amg.log 2>&1
c=$?; tail -5 $OUT/${TAG}_amg.log; [ $c -eq 0 ] || exit $c
timeout -k 10 600 python -u tools/amg_pair_ab.py > $OUT/${TAG}_ab.json 2> $OUT/${TAG}_ab.err
c=$?; cat $OUT/${TAG}_ab.json; exit $c
