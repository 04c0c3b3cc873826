#!/bin/bash
# grid-schedule Gauss-Seidel sweep, FD 8192^2: per-step phase breakdown (s_memtime probe build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
PSK_LIBRARY=tools/bin/ab_gridprof/libpsk.so timeout -k 10 300 python tools/grid_probe.py --side 8192 > $OUT/r3_gridprobe.json 2> $OUT/r3_gridprobe.err || exit $?
python -c "import json;d=json.load(open('$OUT/r3_gridprobe.json'));print({k:d[k] for k in d if k!='probe'})"
