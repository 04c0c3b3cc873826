#!/bin/bash
# Round 3, first GPU session: the ticket gridsum (placement-independent) under the GPU suite, then a
# same-box A/B of bench.py against the round-2 build (tools/bin/ab_r2/libpsk.so) at 16384^2 and 3163^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3_pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/r3_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for v in new r2; do
    if [ $v = new ]; then L=pysolvers_amd/_lib/libpsk.so; else L=tools/bin/ab_r2/libpsk.so; fi
    for s in 16384 3163; do
      echo "== $v side $s round $i"
      PSK_LIBRARY=$L timeout -k 10 300 python bench.py --side $s --steps 100 --repeats 5 --cpu-iters 0 --general 0 \
        --spmv10m 0 --config1 0 --config2 0 --config4 0 > $OUT/r3_ab_${v}_${s}_$i.json 2> $OUT/r3_ab_${v}_${s}_$i.err || exit $?
      python -c "import json;d=json.load(open('$OUT/r3_ab_${v}_${s}_$i.json'));print(d['value'],d['roofline']['avg_launch_ms'],d['spmv_plain_batch20']['avg_launch_ms'])"
    done
  done
done
