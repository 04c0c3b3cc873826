#!/bin/bash
# round 6 (session 2): the deferred gridsum final stage (SpMV p.Ap collected by K2, K2's [r.r, u.r] by K3) —
# PCG parity + layout tests on the in-tree build, then an A/B against HEAD and the prologue-only build, bit-checked
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s16}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_smoke.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; tail -3 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 3 \
  head=@tools/bin/ab_head/libpsk.so pro=@tools/bin/ab_pro/libpsk.so def=@tools/bin/ab_def/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl
timeout -k 10 300 python -u tools/ab_pcg.py --sides 3163 --steps 200 --rounds 2 \
  pro=@tools/bin/ab_pro/libpsk.so def=@tools/bin/ab_def/libpsk.so > $OUT/${TAG}_s200.jsonl 2>> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s200.jsonl
