#!/bin/bash
# Round-6 session 7: the whole GPU suite on the cleaned-up build (lab knobs compile-time, CSR chunked tile map,
# K2 / pair-SpMV variants removed), then the driver's bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s7}
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
c=$?; echo "bench exit $c"; tail -3 $OUT/${TAG}_bench.err
exit $c
