#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in pysolvers_amd/_lib/libpsk.so tools/bin/ab_pad4/libpsk.so tools/bin/ab_pad32/libpsk.so tools/bin/ab_nostore/libpsk.so; do
  for MODE in 0 1; do for M in 3163 16384; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py $M 100 || exit $?
  done; done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread 2>&1 | tail -2
