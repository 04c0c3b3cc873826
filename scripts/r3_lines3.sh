#!/bin/bash
# whole-line gridsum slots: group size (probe builds, dot-mode SpMV back to back at N = 10M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in 1 2; do
for L in tools/bin/ab_intree2 pysolvers_amd/_lib tools/bin/ab_l_gl1 tools/bin/ab_l_gl2 tools/bin/ab_l_gl3 tools/bin/ab_l_noticket; do
    PSK_LIBRARY=$L/libpsk.so PSK_SPMV_TIMED_MODE=1 timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
done
done
