#!/bin/bash
# round 6 (session 2): the GPU tests that load libpsk_lab.so, on the final tree (the lab library gained
# psk_lab_spmv_rotate; libpsk.so unchanged, e9bd5bbd), then the smoke entry point
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s25}
sha256sum pysolvers_amd/_lib/libpsk.so pysolvers_amd/_lib/libpsk_lab.so > $OUT/${TAG}_lib.sha256
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_progress.py tests/test_gpu_gs_pair.py tests/test_gpu_configs.py tests/test_gpu_smoke.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; tail -3 $OUT/${TAG}_pytest.log; exit $c
