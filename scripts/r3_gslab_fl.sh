#!/bin/bash
# full-line slot probe: every tile's slot on its own 128-B line, written whole (PSK_LAB_GS_FULLLINE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in 1 2; do
for L in tools/bin/ab_intree2/libpsk.so tools/bin/ab_fullline/libpsk.so tools/bin/ab_noticket/libpsk.so tools/bin/ab_fl_noticket/libpsk.so; do
  for MODE in 0 1; do
    PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py 3163 200 || exit $?
  done
done
done
