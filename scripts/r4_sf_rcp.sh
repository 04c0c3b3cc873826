#!/bin/bash
# sync-free quotient from a per-row reciprocal (Markstein) vs the IEEE division (tools/bin/ab_prev: the
# previous commit's build): configs[2]'s ILU apply and its result checksum, two rounds; then the
# triangular-solve GPU tests; then the level probe and the partitioned hand-off spin A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export PSK_LIBRARY=$PWD/tools/bin/ab_prev/libpsk.so; else unset PSK_LIBRARY; fi
    PSK_NO_TORCH=1 timeout -k 10 300 python -u tools/sf_probe.py 2896 > $OUT/r4rcp_${v}_$r.json 2>> $OUT/r4rcp.err
    c=$?; echo "$v $r exit $c $(cat $OUT/r4rcp_${v}_$r.json | cut -c1-160)"; [ $c -eq 0 ] || exit $c
  done
done
unset PSK_LIBRARY
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_part.py tests/test_gpu_amg.py tests/test_gpu_parity.py tests/test_gpu_newton.py > $OUT/r4rcp_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -2 $OUT/r4rcp_pytest.log; [ $c -eq 0 ] || exit $c
bash scripts/r4_level1.sh
