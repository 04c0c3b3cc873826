#!/bin/bash
# triangular-solve schedules: the AMG/trisolve GPU tests, then configs[4] per-level timings under
# every schedule; each GPU step time-limited, stop at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2t}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_amg.py -x -v --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_amg.log 2>&1 \
  || { echo "pytest failed"; tail -40 $OUT/${TAG}_pytest_amg.log; exit 1; }
tail -3 $OUT/${TAG}_pytest_amg.log
timeout -k 10 400 python tools/bench_amg.py --side ${SIDE:-8192} --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err \
  || { echo "bench_amg failed"; tail -20 $OUT/${TAG}_amg.err; exit 1; }
cat $OUT/${TAG}_amg.json
echo "== done"
