#!/bin/bash
# Round-5 session 2: the new diagonal layout and the forward-progress schedules first (their own tests),
# then the whole -m gpu suite, the per-solve fixed cost, and the driver-style bench with the diagonal
# layout on / off (PSK_SPMV_DIAG=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s2}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -v --timeout 200 --timeout-method thread -k "diag or auto or fd_large" > $OUT/${TAG}_diag.log 2>&1
c=$?; echo "diag tests exit $c"; tail -3 $OUT/${TAG}_diag.log; ok $c || exit $c
timeout -k 10 300 python -u -m pytest tests/test_gpu_progress.py -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_progress.log 2>&1
c=$?; echo "progress tests exit $c"; tail -3 $OUT/${TAG}_progress.log; ok $c || exit $c
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; ok $c || exit $c
timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed.json 2> $OUT/${TAG}_fixed.err
c=$?; echo "fixed exit $c"; cat $OUT/${TAG}_fixed.json; ok $c || exit $c
for v in 1 0 1 0; do
  PSK_SPMV_DIAG=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-iters 0 --general 0 --config1 0 --gmres 0 --config2 0 --config4 0 > $OUT/${TAG}_bench_diag$v.json 2> $OUT/${TAG}_bench_diag$v.err
  c=$?; echo "bench diag=$v exit $c"; ok $c || exit $c
  python -c "import json,sys; d=json.load(open('$OUT/${TAG}_bench_diag$v.json')); r=d['roofline']; print('diag=$v', round(d['value'],1), r['avg_launch_ms'], round(r['frac'],3), d['roofline']['layout'], d.get('strong_scaling_16384',{}).get('pcg_it_per_s'), d['fixed_overhead']['fixed_overhead_ms'], d['spmv_plain_batch50']['avg_launch_ms'])"
done
