#!/bin/bash
# round 6 (session 2): K3 (and K2) tiles on the SpMV's XCD bands, so each XCD writes the p rows it gathers in the next
# SpMV (tools/mall_probe.py: a launch reading an x the previous kernel wrote is ~5 us slower at N = 10M), bit-checked
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s28}
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 2 \
  cur=@tools/bin/ab_cur/libpsk.so k3b=@tools/bin/ab_k3b/libpsk.so k23b=@tools/bin/ab_k23b/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl
timeout -k 10 300 python -u tools/ab_pcg.py --sides 3163 --steps 200 --rounds 1 \
  cur=@tools/bin/ab_cur/libpsk.so k3b=@tools/bin/ab_k3b/libpsk.so k23b=@tools/bin/ab_k23b/libpsk.so > $OUT/${TAG}_s200.jsonl 2>> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s200.jsonl
