#!/bin/bash
# whole-line gridsum slots: which part costs (probe builds, dot-mode SpMV back to back at N = 10M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PSK_LIBRARY=pysolvers_amd/_lib/libpsk.so PSK_SPMV_TIMED_MODE=0 timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
for R in 1 2; do
for L in tools/bin/ab_intree2 pysolvers_amd/_lib tools/bin/ab_l_noarm tools/bin/ab_l_noticket tools/bin/ab_l_noarm_noticket tools/bin/ab_l_line8 tools/bin/ab_noticket; do
    PSK_LIBRARY=$L/libpsk.so PSK_SPMV_TIMED_MODE=1 timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
done
done
