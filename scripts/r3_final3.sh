#!/bin/bash
# Round 3 final evidence for the committed build (third pass: host-mapped PCG done word, AMG
# smoother fusion, MatrixMarket size-line check; the GPU test suite first): the driver's bench command, rocprofv3 kernel trace + stats of the headline and of the
# configs[2] / configs[4] runs (ILU and AMG kernels), and the PMC traffic passes, all of one libpsk.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
sha256sum pysolvers_amd/_lib/libpsk.so | tee $OUT/r3f_lib.sha256
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r3f_smoke.log 2>&1 || { tail -5 $OUT/r3f_smoke.log; exit 1; }
tail -2 $OUT/r3f_smoke.log
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/r3f_pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/r3f_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
echo "== PMC passes"
TAG=r3f SIDES="3163 16384" PMC_ARGS="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0" bash scripts/gpu_pmc.sh || exit $?
PA="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --scaling-side 0 --config1 0 --config2 0 --config4 0 --gmres 0 --general 0"
for S in 3163 16384; do   # the traffic profiles of this build, where bench.py looks for them
  python tools/pmc_summary.py $OUT/pmc_r3f_${S}_FETCH_SIZE $OUT/pmc_r3f_${S}_WRITE_SIZE $OUT/pmc_r3f_calib_FETCH_SIZE \
      $OUT/pmc_r3f_calib_WRITE_SIZE $S "$PA" $OUT/pmc_r3f_lib.sha256 > profiles/r3_pmc_traffic_$S.json || exit $?
  cp profiles/r3_pmc_traffic_$S.json $OUT/r3f_pmc_traffic_$S.json
done
rm -rf $OUT/pmc_r3f_*_FETCH_SIZE $OUT/pmc_r3f_*_WRITE_SIZE
echo "== bench (defaults)"; timeout -k 10 900 python bench.py > $OUT/r3f_bench.json 2> $OUT/r3f_bench.err || { tail -5 $OUT/r3f_bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r3f_bench.json'));print('value %.1f'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'), d['roofline'].get('traffic_note'))"
echo "== rocprofv3 kernel trace + stats of the headline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r3f_prof -o run --output-format csv -- python bench.py --cpu-iters 0 --general 0 \
   --config1 0 --config2 0 --config4 0 --gmres 1 > $OUT/r3f_prof_bench.json 2> $OUT/r3f_prof_bench.err || exit $?
python tools/trace_stats.py $(find $OUT/r3f_prof -name "*kernel_trace.csv" | head -1) > $OUT/r3f_trace_stats.csv
cp $(find $OUT/r3f_prof -name "*kernel_stats.csv" | head -1) $OUT/r3f_kernel_stats.csv
rm -rf $OUT/r3f_prof
echo "== rocprofv3 kernel trace + stats of configs[2] (ILU) and configs[4] (AMG)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/r3f_prof2 -o run --output-format csv -- python bench.py --steps 20 --warmup 2 \
   --cpu-iters 0 --general 0 --config1 0 --gmres 0 --scaling-side 0 > $OUT/r3f_prof_amg_ilu.json 2> $OUT/r3f_prof_amg_ilu.err; echo "profiled run exit $?"
python tools/trace_stats.py $(find $OUT/r3f_prof2 -name "*kernel_trace.csv" | head -1) > $OUT/r3f_amg_ilu_trace_stats.csv
rm -rf $OUT/r3f_prof2
