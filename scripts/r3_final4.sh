#!/bin/bash
# Round 3 final evidence (fourth pass: the compact SpMV stream, PSK_SPMV_COMPACT): GPU suite, the
# headline with the compact stream off / on, then PMC passes, the default bench and the headline trace: the driver's bench command, rocprofv3 kernel trace + stats of the headline and of the
# configs[2] / configs[4] runs (ILU and AMG kernels), and the PMC traffic passes, all of one libpsk.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum pysolvers_amd/_lib/libpsk.so | tee $OUT/r3h4_lib.sha256
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r3h4_smoke.log 2>&1 || { tail -5 $OUT/r3h4_smoke.log; exit 1; }
tail -2 $OUT/r3h4_smoke.log
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3h4_pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/r3h4_pytest_gpu.log; grep -E "^FAILED" $OUT/r3h4_pytest_gpu.log | head -5; [ $rc -eq 0 ] || exit 1
echo "== headline A/B: compact stream off / on"
A="--cpu-iters 0 --general 0 --config1 0 --config2 0 --config4 0 --gmres 0 --scaling-side 0"
for v in 0 1 0 1; do
  PSK_SPMV_COMPACT=$v timeout -k 10 300 python bench.py $A > $OUT/r3h4_ab_$v.json 2> $OUT/r3h4_ab_$v.err || { tail -3 $OUT/r3h4_ab_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r3h4_ab_$v.json'));print('compact=$v', round(d['value'],1), 'noev', round(d['regions_without_kernel_events']['median_it_s'],1), 'spmv_ms', round(d['roofline']['avg_launch_ms'],4), 'alg_B', d['roofline']['algorithmic_bytes_per_launch'])"
done
echo "== PMC passes"
TAG=r3h4 SIDES="3163 16384" PMC_ARGS="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0" bash scripts/gpu_pmc.sh || exit $?
PA="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0"
for S in 3163 16384; do   # the traffic profiles of this build, where bench.py looks for them
  python tools/pmc_summary.py $OUT/pmc_r3h4_${S}_FETCH_SIZE $OUT/pmc_r3h4_${S}_WRITE_SIZE $OUT/pmc_r3h4_calib_FETCH_SIZE \
      $OUT/pmc_r3h4_calib_WRITE_SIZE $S "$PA" $OUT/pmc_r3h4_lib.sha256 > profiles/r3_pmc_traffic_$S.json || exit $?
  cp profiles/r3_pmc_traffic_$S.json $OUT/r3h4_pmc_traffic_$S.json
done
rm -rf $OUT/pmc_r3h4_*_FETCH_SIZE $OUT/pmc_r3h4_*_WRITE_SIZE
echo "== bench (defaults)"; timeout -k 10 900 python bench.py > $OUT/r3h4_bench.json 2> $OUT/r3h4_bench.err || { tail -5 $OUT/r3h4_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r3h4_bench.json'));print('value %.1f'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'), d['roofline'].get('traffic_note'))"
echo "== rocprofv3 kernel trace + stats of the headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r3h4_prof -o run --output-format csv -- python bench.py --cpu-iters 0 --general 0 \
   --config1 0 --config2 0 --config4 0 --gmres 1 > $OUT/r3h4_prof_bench.json 2> $OUT/r3h4_prof_bench.err || exit $?
python tools/trace_stats.py $(find $OUT/r3h4_prof -name "*kernel_trace.csv" | head -1) > $OUT/r3h4_trace_stats.csv
cp $(find $OUT/r3h4_prof -name "*kernel_stats.csv" | head -1) $OUT/r3h4_kernel_stats.csv
rm -rf $OUT/r3h4_prof
