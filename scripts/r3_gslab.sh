#!/bin/bash
# dot-epilogue lab: plain vs dot-mode back-to-back SpMV for the in-tree build and the gridsum probes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in pysolvers_amd/_lib/libpsk.so tools/bin/ab_noticket/libpsk.so tools/bin/ab_nopublish/libpsk.so tools/bin/ab_r2/libpsk.so; do
  for MODE in 0 1; do
    for M in 3163 16384; do
      PSK_LIBRARY=$L PSK_SPMV_TIMED_MODE=$MODE timeout -k 10 120 python tools/spmv_batch.py $M 100 || exit $?
    done
  done
done
