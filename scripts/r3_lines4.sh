#!/bin/bash
# hybrid gridsum (tile slot lines + packed group sums): dot-mode SpMV back to back at N = 10M and 16384^2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in 1 2; do
for L in tools/bin/ab_intree2 pysolvers_amd/_lib tools/bin/ab_h_nofinal tools/bin/ab_h_noticket; do
    PSK_LIBRARY=$L/libpsk.so PSK_SPMV_TIMED_MODE=1 timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
done
done
for L in tools/bin/ab_intree2 pysolvers_amd/_lib; do
    PSK_LIBRARY=$L/libpsk.so PSK_SPMV_TIMED_MODE=1 timeout -k 10 120 python tools/spmv_batch.py 16384 20 || exit $?
done
