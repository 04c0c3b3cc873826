#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in tools/bin/ab_nostore/libpsk.so tools/bin/ab_onestore/libpsk.so tools/bin/ab_plainstore/libpsk.so tools/bin/ab_noticket/libpsk.so; do
  for MODE in 0 1; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
  done
done
