#!/bin/bash
# round 6 (session 2): the round-end driver's sequence on the final tree — pytest -m gpu, then the bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s26}
sha256sum pysolvers_amd/_lib/libpsk.so pysolvers_amd/_lib/libpsk_lab.so > $OUT/${TAG}_lib.sha256
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; tail -2 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
c=$?; echo "bench exit $c"; cut -c1-300 $OUT/${TAG}_bench.json; exit $c
