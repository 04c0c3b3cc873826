#!/bin/bash
# Round 6 final evidence, part A: the GPU suite, then the driver-style bench line twice: on the system
# ROCm runtime (bench.py's N = 1 default, PSK_NO_TORCH=1) and on torch's bundled runtime (PSK_NO_TORCH=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6fa}
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/${TAG}_lib.sha256
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err
c=$?; echo "bench exit $c"; [ $c -le 1 ] || exit $c
PSK_NO_TORCH=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --config2 0 --config4 0 --gmres 0 --config1 0 --cpu-iters 0 > $OUT/${TAG}_bench_torchrt.json 2> $OUT/${TAG}_bench_torchrt.err
echo "bench torch-runtime exit $?"
# the headline regions' SpMV launches under rocprofv3 (the bench line's roofline samples every 8th of them)
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- \
    python -u bench.py --steps 20 --warmup 5 --cpu-iters 0 --config1 0 --config2 0 --config4 0 --gmres 0 > $OUT/${TAG}_prof.json 2> $OUT/${TAG}_prof.err
c=$?; echo "profiled headline exit $c"
python tools/region_trace.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) > $OUT/${TAG}_headline_regions.json
python tools/trace_stats.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) > $OUT/${TAG}_trace_stats.csv
rm -rf $OUT/${TAG}_prof
cat $OUT/${TAG}_headline_regions.json
