#!/bin/bash
# grid-schedule Gauss-Seidel: unconditional buffer rhs loads / x stores (in-tree) vs branches (ab_head);
# then the GPU suite (grid vs band bit-identity tests included)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for R in 1 2; do
for L in tools/bin/ab_head pysolvers_amd/_lib; do
  for L3 in 0 1; do
    echo -n "$L level3=$L3 "; PSK_LIBRARY=$L/libpsk.so timeout -k 10 300 python tools/grid_probe.py --side 8192 --level3 $L3 || exit $?
  done
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3m_tests.log; exit $rc
