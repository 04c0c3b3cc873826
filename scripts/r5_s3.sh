#!/bin/bash
# Round-5 session 3: the forward-progress probe (tools/progress_probe.py) beside occupiers, plain and
# under a rocprofv3 kernel trace; the lap3d diagonal-layout test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s3}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 120 python -u tools/progress_probe.py --seconds 6 > $OUT/${TAG}_probe.jsonl 2> $OUT/${TAG}_probe.err
c=$?; echo "probe exit $c"; cat $OUT/${TAG}_probe.jsonl; tail -3 $OUT/${TAG}_probe.err; ok $c || exit $c
PSK_SYNCFREE_PER_CU=3 timeout -k 10 120 python -u tools/progress_probe.py --seconds 6 > $OUT/${TAG}_probe3.jsonl 2> $OUT/${TAG}_probe3.err
c=$?; echo "probe per_cu=3 exit $c"; cat $OUT/${TAG}_probe3.jsonl; ok $c || exit $c
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/${TAG}_prof -o run --output-format csv -- python -u tools/progress_probe.py --seconds 6 > $OUT/${TAG}_probep.jsonl 2> $OUT/${TAG}_probep.err
c=$?; echo "profiled probe exit $c"; ok $c || exit $c
f=$(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python - "$f" > $OUT/${TAG}_probe_trace.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%12.1f %10.1f %8s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Grid_Size_X", ""), r["Kernel_Name"][:90]))
PY
tail -40 $OUT/${TAG}_probe_trace.txt
rm -rf $OUT/${TAG}_prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_layout.py -x -v --timeout 200 --timeout-method thread -k "diag_layout" > $OUT/${TAG}_diag.log 2>&1
c=$?; echo "diag tests exit $c"; tail -3 $OUT/${TAG}_diag.log
PSK_LIBRARY=tools/bin/ab_sprof/libpsk.so timeout -k 10 180 python -u tools/spmv_probe.py > $OUT/${TAG}_spmvprobe.jsonl 2> $OUT/${TAG}_spmvprobe.err
c=$?; echo "spmv probe exit $c"; cat $OUT/${TAG}_spmvprobe.jsonl; tail -3 $OUT/${TAG}_spmvprobe.err
