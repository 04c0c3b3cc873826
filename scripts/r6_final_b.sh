#!/bin/bash
# Round 6 final evidence, part B: rocprofv3 kernel trace + stats of the default bench (every key; exit
# code recorded: the configs[2]/[4] keys faulted in exit() under the profiler before round 4), then the
# PMC traffic passes of the headline sides (FETCH_SIZE / WRITE_SIZE, one counter per pass) + calibration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6fb}
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 5 --cpu-iters 0 > $OUT/${TAG}_prof.json 2> $OUT/${TAG}_prof.err
c=$?; echo "profiled bench exit $c"
python tools/trace_stats.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) > $OUT/${TAG}_trace_stats.csv
# the headline regions' own SpMV launches (the bench line's roofline.avg_launch_ms samples every 8th of them)
python tools/region_trace.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) > $OUT/${TAG}_headline_regions.json
cp $(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_kernel_stats.csv
rm -rf $OUT/${TAG}_prof
[ $c -eq 0 ] || exit $c
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
TAG=$TAG PMC_ARGS="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --config1 0 --config2 0 --config4 0 --general 0 --gmres 0 --scaling-side 0" \
    bash scripts/gpu_pmc.sh
c=$?; echo "pmc exit $c"; [ $c -eq 0 ] || exit $c
for S in 3163 16384; do
  python tools/pmc_summary.py $OUT/pmc_${TAG}_${S}_FETCH_SIZE $OUT/pmc_${TAG}_${S}_WRITE_SIZE $OUT/pmc_${TAG}_calib_FETCH_SIZE \
      $OUT/pmc_${TAG}_calib_WRITE_SIZE $S "--steps 20 --warmup 2 --repeats 1" $OUT/pmc_${TAG}_lib.sha256 > $OUT/${TAG}_pmc_traffic_$S.json
done
for d in $OUT/pmc_${TAG}_*; do [ -d "$d" ] && rm -rf "$d"; done
echo done
