#!/bin/bash
# round-end evidence: every GPU test, smoke(), the bench line, its rocprofv3 kernel trace, and the
# configs[2] / configs[4] benches; each GPU step time-limited, stop at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r1h_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/r1h_pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r1h_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > $OUT/r1h_bench_final.json 2> $OUT/r1h_bench_final.err || { echo "bench failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r1h_prof -o run --output-format csv -- python bench.py --cpu-iters 0 > $OUT/r1h_prof_bench.json 2> $OUT/r1h_prof_bench.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 python tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/r1h_amg8192.json 2> $OUT/r1h_amg8192.err || { echo "amg failed"; exit 1; }
timeout -k 10 300 python tools/bench_gmres.py --side 2896 --restart 30 --steps 60 > $OUT/r1h_gmres_ilut_2896.json 2> $OUT/r1h_gmres.err || { echo "gmres failed"; exit 1; }
echo "== done"
