#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout stops the script (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r1}

stop_if_crashed() {  # $1 = exit code of the previous GPU step
    case "$1" in
        0|1) return 0 ;;             # ok / test failures: the GPU is fine
        *) echo "GPU step exited $1: stopping"; exit "$1" ;;
    esac
}

echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; tail -3 $OUT/smoke_$TAG.log; stop_if_crashed $rc

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu_$TAG.log; stop_if_crashed $rc
fi

echo "== bench"; timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; cat $OUT/bench_$TAG.json; tail -5 $OUT/bench_$TAG.err; stop_if_crashed $rc

if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
      python bench.py ${PROF_ARGS:---cpu-iters 0 --spmv10m 0 --config1 0} > $OUT/prof_bench_$TAG.json 2> $OUT/prof_$TAG.err
  rc=$?; tail -3 $OUT/prof_$TAG.err; stop_if_crashed $rc
  find $OUT/prof_$TAG -name '*kernel_stats.csv' -exec head -20 {} \;
fi
echo "== done"
