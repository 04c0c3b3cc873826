#!/bin/bash
# round 6 (session 2): is the in-loop SpMV's "loop context" the Infinity Cache? back-to-back SpMV launches cycling
# through 1/2/4/8 (x, y) pairs at N = 10M and 16384^2 (tools/mall_probe.py, psk_lab_spmv_rotate)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s24}
timeout -k 10 300 python -u tools/mall_probe.py 3163 120 > $OUT/${TAG}_3163.txt 2> $OUT/${TAG}.err || exit 1
cat $OUT/${TAG}_3163.txt | grep -v "^{"
timeout -k 10 300 python -u tools/mall_probe.py 8192 40 > $OUT/${TAG}_8192.txt 2>> $OUT/${TAG}.err || exit 1
cat $OUT/${TAG}_8192.txt | grep -v "^{"
