#!/bin/bash
# Round-6 session 2: K2 with one tile per wave (in-tree) vs round 6a (tools/bin/ab_r6a: the pair SpMV, K2 one tile
# per workgroup); pair-SpMV epilogue probes (lab builds: no epilogue / no group reduction / ticket first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layout.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -5 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 k2w= r6a=@tools/bin/ab_r6a/libpsk.so noepi=@tools/bin/ab_noepi/libpsk.so nored=@tools/bin/ab_nored/libpsk.so tfirst=@tools/bin/ab_tfirst/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl
exit $c
