#!/bin/bash
# Evidence for the shipped build, each GPU step time-limited, stop at the first failure.
# STAGES (space separated, in order): pmc trace bench tests smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2}
mkdir -p $OUT
export TMPDIR=/tmp
for st in ${STAGES:-pmc trace bench}; do
  case $st in
    pmc)
      TAG=$TAG bash scripts/gpu_pmc.sh || exit 1 ;;
    trace)
      echo "== trace"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- \
          python bench.py --cpu-iters 0 --config2 0 --config4 0 > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof_bench.err \
          || { echo "trace failed"; tail -5 $OUT/${TAG}_prof_bench.err; exit 1; } ;;
    bench)
      echo "== bench"
      timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
          || { echo "bench failed"; tail -20 $OUT/${TAG}_bench.err; exit 1; } ;;
    tests)
      echo "== tests"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gpu.log 2>&1 \
          || { echo "pytest failed"; tail -30 $OUT/${TAG}_pytest_gpu.log; exit 1; }
      tail -2 $OUT/${TAG}_pytest_gpu.log ;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 \
          || { echo "smoke failed"; tail -20 $OUT/${TAG}_smoke.log; exit 1; } ;;
  esac
done
echo "== evidence done"
