#!/bin/bash
# Round-6 session 1: the pair-row diagonal SpMV (spmv_diagp_kernel) — layout/shard/parity GPU tests, then a
# same-box A/B: H = 2 (default), H = 1, the one-row kernel (PSK_DIAG_PAIR=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_shards.py tests/test_gpu_smoke.py -x -v --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -5 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 h2= h1=PSK_DIAG_PAIR=1 one=PSK_DIAG_PAIR=0 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl
exit $c
