#!/bin/bash
# Same-box A/B of bench.py's headline (PCG+Jacobi, in-loop SpMV) between the in-tree libpsk,
# the same with PSK_SPMV_XCD_BANDS=0, and the round-2 build (tools/bin/ab_r2/libpsk.so).
# SIDES (default "3163 16384"), ROUNDS (2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in new nobands r2; do
    L=pysolvers_amd/_lib/libpsk.so; B=1
    [ $v = r2 ] && L=tools/bin/ab_r2/libpsk.so
    [ $v = nobands ] && B=0
    for s in ${SIDES:-3163 16384}; do
      PSK_SPMV_XCD_BANDS=$B PSK_LIBRARY=$L timeout -k 10 300 python bench.py --side $s --steps 100 --repeats 5 --cpu-iters 0 --general 0 \
        --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 > $OUT/r3ab_${v}_${s}_$i.json 2> $OUT/r3ab_${v}_${s}_$i.err || exit $?
      python -c "import json;d=json.load(open('$OUT/r3ab_${v}_${s}_$i.json'));print('$v',$s,'it/s %.1f'%d['value'],'spmv_loop %.4f'%d['roofline']['avg_launch_ms'],'plain %.4f'%d['spmv_plain_batch50']['avg_launch_ms'],'csr %.4f'%d['spmv_csr_layout_batch50']['avg_launch_ms'])"
    done
  done
done
if [ "${PROF:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/r3ab_prof -o run --output-format csv -- python bench.py --side 3163 --steps 100 --repeats 2 \
     --cpu-iters 0 --general 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 > /dev/null 2> $OUT/r3ab_prof.err || exit $?
  python tools/trace_stats.py $(ls $OUT/r3ab_prof/*/run_kernel_trace.csv $OUT/r3ab_prof/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/r3ab_prof_stats.csv; cut -c1-150 $OUT/r3ab_prof_stats.csv | head -12
fi
