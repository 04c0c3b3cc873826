#!/bin/bash
# Round-6 session 8: where a short psk_pcg call's fixed cost goes — HIP API + kernel trace of 0 / 1 / 20-iteration
# solves at N = 10M with host marks (tools/solve_timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s8}
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace -d $OUT/${TAG}_tl -o run --output-format csv -- \
    python tools/solve_timeline.py --out $OUT/${TAG}_marks.json > $OUT/${TAG}_tl.log 2>&1
c=$?; echo "timeline exit $c"; [ $c -eq 0 ] || { tail -20 $OUT/${TAG}_tl.log; exit $c; }
python tools/solve_timeline.py --analyze $(find $OUT/${TAG}_tl -name "*hip_api_trace.csv" | head -1) \
    $(find $OUT/${TAG}_tl -name "*kernel_trace.csv" | head -1) $OUT/${TAG}_marks.json > $OUT/${TAG}_timeline.jsonl
c=$?; cat $OUT/${TAG}_timeline.jsonl | cut -c1-900; rm -rf $OUT/${TAG}_tl
exit $c
