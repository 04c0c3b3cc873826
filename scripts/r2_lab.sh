#!/bin/bash
# tools/bin/pcg_lab (library SpMV modes in and out of a PCG-like context) against the in-tree libpsk
# and the experiment builds under tools/bin/ab_<name>/ given as arguments
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2lab}
mkdir -p $OUT
for v in new "$@"; do
  if [ "$v" = new ]; then L=pysolvers_amd/_lib; else L=tools/bin/ab_$v; fi
  echo "== $v"
  LD_LIBRARY_PATH=$L timeout -k 10 120 tools/bin/pcg_lab ${LAB_SIDES:-3163 16384} > $OUT/${TAG}_$v.txt 2>&1 || { echo "lab $v failed"; tail -5 $OUT/${TAG}_$v.txt; exit 1; }
  grep -E "plain batch|dot batch|dot\+flag after k3like  " $OUT/${TAG}_$v.txt
done
