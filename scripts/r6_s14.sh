#!/bin/bash
# round 6: batched band publications in the paired sweep launch — bitwise tests, then the 8192^2 apply A/B against
# the committed build (tools/bin/ab_head, scripts/build_worktree.sh), alternating, pairing on in both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s14}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gs_pair.py > $OUT/${TAG}_pair.log 2>&1
c=$?; tail -2 $OUT/${TAG}_pair.log; [ $c -eq 0 ] || exit $c
for r in 1 2; do
  timeout -k 10 300 python -u tools/amg_pair_ab.py --rounds 1 --no-lab > $OUT/${TAG}_new_$r.json 2>> $OUT/${TAG}.err || exit 1
  PSK_LIBRARY=tools/bin/ab_head/libpsk.so timeout -k 10 300 python -u tools/amg_pair_ab.py --rounds 1 --no-lab > $OUT/${TAG}_head_$r.json 2>> $OUT/${TAG}.err || exit 1
  echo "round $r"; cat $OUT/${TAG}_new_$r.json $OUT/${TAG}_head_$r.json | python -c "import sys,json; [print(json.loads(l)['on']['apply_ms_median'], json.loads(l)['on']['pcg_it_s_median']) for l in sys.stdin]"
done
