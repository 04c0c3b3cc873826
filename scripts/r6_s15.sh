#!/bin/bash
# round 6 (session 2): K2/K3 scalar prologue (done flag, p.Ap, udr[k], tau*||b|| loaded together) against HEAD,
# alternating, bit-checked (resid_bits / x_sha), at the driver's 20-iteration regions and at 200
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s15}
timeout -k 10 480 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 3 \
  head=@tools/bin/ab_head/libpsk.so pro=@tools/bin/ab_pro/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
timeout -k 10 300 python -u tools/ab_pcg.py --sides 3163 --steps 200 --rounds 2 \
  head=@tools/bin/ab_head/libpsk.so pro=@tools/bin/ab_pro/libpsk.so > $OUT/${TAG}_s200.jsonl 2>> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl; python tools/ab_summary.py $OUT/${TAG}_s200.jsonl
