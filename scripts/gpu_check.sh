#!/bin/bash
# Round-4 GPU check: the -m gpu suite, the driver-style bench (--steps 20 --warmup 5) and the
# rocprofv3 trace of the configs[2]/[4] keys with the process maps dumped at exit (exit-fault hunt).
# Each GPU step has its own time limit; a step that ends by signal/timeout stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r4}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }   # 0 pass, 1 test/bench failure; anything else: stop
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; ok $c || exit $c
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
c=$?; echo "bench exit $c"; ok $c || exit $c
PSK_DUMP_MAPS=$OUT/${TAG}_maps.txt timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 2 --cpu-iters 0 --general 0 --config1 0 --gmres 0 --scaling-side 0 \
    > $OUT/${TAG}_prof.json 2> $OUT/${TAG}_prof.err
echo "profiled exit $?"
python tools/trace_stats.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) > $OUT/${TAG}_trace_stats.csv
rm -rf $OUT/${TAG}_prof
