#!/bin/bash
# Round-6 session 5: pair-SpMV quad tickets (tools/bin/ab_quad) vs one ticket per slice (in-tree), with the
# no-epilogue / no-reduction probes (lab builds, wrong p.Ap: timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s5}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 3 base= quad=@tools/bin/ab_quad/libpsk.so noepi=@tools/bin/ab_noepi/libpsk.so nored=@tools/bin/ab_nored/libpsk.so k2wave=@tools/bin/ab_k2wave/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl
exit $c
