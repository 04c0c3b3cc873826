#!/bin/bash
# Round-4 lab: slices per workgroup of the compact SpMV (PSK_SPMV_TPW) and the y store policy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r4c}
timeout -k 10 1000 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 tpw1= tpw2=PSK_SPMV_TPW=2 tpw3=PSK_SPMV_TPW=3 tpw4=PSK_SPMV_TPW=4 tpw2ydef=@tools/bin/ab_ydef/libpsk.so,PSK_SPMV_TPW=2 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
echo "ab exit $?"
