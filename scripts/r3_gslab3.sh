#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in pysolvers_amd/_lib/libpsk.so tools/bin/ab_xchg/libpsk.so tools/bin/ab_nostore/libpsk.so; do
  for MODE in 0 1; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
  done
done
PSK_LIBRARY=tools/bin/ab_xchg/libpsk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "gridsum or golden or fd4096" -p no:cacheprovider --timeout 300 --timeout-method thread 2>&1 | tail -2
