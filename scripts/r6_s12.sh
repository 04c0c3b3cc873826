#!/bin/bash
# round 6: paired Gauss-Seidel sweeps (streamed) — bitwise tests, per-band profile, 8192^2 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s12}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_pair.py > $OUT/${TAG}_pair.log 2>&1
c=$?; tail -4 $OUT/${TAG}_pair.log; [ $c -eq 0 ] || exit $c
PSK_LIBRARY=tools/bin/ab_gpprof/libpsk.so timeout -k 10 300 python -u tools/gp_prof.py --m 2048 > $OUT/${TAG}_prof2048.json 2>&1
c=$?; cat $OUT/${TAG}_prof2048.json; [ $c -eq 0 ] || exit $c
timeout -k 10 600 python -u tools/amg_pair_ab.py --rounds 2 > $OUT/${TAG}_ab.json 2> $OUT/${TAG}_ab.err
c=$?; cat $OUT/${TAG}_ab.json; exit $c
