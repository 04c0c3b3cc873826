#!/bin/bash
# round 6 (session 2): deferred gridsum final stage, v2 (wave-0 collection, exact loads) — PCG parity/layout tests on the
# in-tree build, A/B against the prologue-only build (bit-checked), and per-kernel times of both under rocprofv3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s17}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_layout.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; tail -2 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
timeout -k 10 400 python -u tools/ab_pcg.py --sides 3163,16384 --steps 20 --rounds 2 \
  pro=@tools/bin/ab_pro/libpsk.so def2=@tools/bin/ab_def2/libpsk.so > $OUT/${TAG}_s20.jsonl 2> $OUT/${TAG}.err || exit 1
python tools/ab_summary.py $OUT/${TAG}_s20.jsonl
for v in pro def2; do
  PSK_LIBRARY=tools/bin/ab_$v/libpsk.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof_$v -o run -- python3 tools/ab_pcg.py --child --sides 3163 --steps 200 > $OUT/${TAG}_prof_$v.log 2>&1 || exit 1
done
for v in pro def2; do
  f=$(find $OUT/${TAG}_prof_$v -name '*kernel_trace.csv' -print -quit)
  python tools/trace_stats.py "$f" > $OUT/${TAG}_stats_$v.csv
  python -c "import csv,sys; [print('%-60s %6s %10s %10s' % (r['Name'][:60], r['Calls'], r['AverageNs'], r['MedianNs'])) for r in list(csv.DictReader(open(sys.argv[1])))[:8]]" $OUT/${TAG}_stats_$v.csv
done
