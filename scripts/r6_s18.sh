#!/bin/bash
# round 6 (session 2): K2 variants — stream loads issued before the done-flag wait (k2e), both grid-sum block reductions
# in one barrier pair (k2s, block_sum2: same bits), both (k2es) — against the in-tree build (pro), bit-checked
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s18}
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 3 \
  pro=@tools/bin/ab_pro/libpsk.so k2e=@tools/bin/ab_k2e/libpsk.so k2s=@tools/bin/ab_k2s/libpsk.so \
  k2es=@tools/bin/ab_k2es/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl
timeout -k 10 400 python -u tools/ab_pcg.py --sides 3163 --steps 200 --rounds 2 \
  pro=@tools/bin/ab_pro/libpsk.so k2e=@tools/bin/ab_k2e/libpsk.so k2s=@tools/bin/ab_k2s/libpsk.so \
  k2es=@tools/bin/ab_k2es/libpsk.so > $OUT/${TAG}_s200.jsonl 2>> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s200.jsonl
