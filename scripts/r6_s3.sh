#!/bin/bash
# Round-6 session 3: pair-SpMV quad tickets (one per workgroup; lab build tools/bin/ab_quad) vs one per slice (in-tree),
# with the no-epilogue / no-reduction probes; the AMG tests (coarse auto = dense + 1 refinement step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s3}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= quad=@tools/bin/ab_quad/libpsk.so noepi=@tools/bin/ab_noepi/libpsk.so nored=@tools/bin/ab_nored/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl; [ $c -le 1 ] || exit $c
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_parity.py tests/test_gpu_progress.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -5 $OUT/${TAG}_pytest.log
exit $c
