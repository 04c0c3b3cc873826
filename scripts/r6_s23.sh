#!/bin/bash
# round 6 (session 2): K2 wave totals by DPP + one LDS combine (K2 sums change
# bits) — PCG parity on that build (PSK_LIBRARY), then an A/B against the current build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s23}
PSK_LIBRARY=tools/bin/ab_dpp/libpsk.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_layout.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; tail -2 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 3 \
  cur=@tools/bin/ab_cur/libpsk.so dpp=@tools/bin/ab_dpp/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl
timeout -k 10 300 python -u tools/ab_pcg.py --sides 3163 --steps 200 --rounds 2 \
  cur=@tools/bin/ab_cur/libpsk.so dpp=@tools/bin/ab_dpp/libpsk.so > $OUT/${TAG}_s200.jsonl 2>> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s200.jsonl
