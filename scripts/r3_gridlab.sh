#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in pysolvers_amd/_lib/libpsk.so tools/bin/ab_noxstore/libpsk.so tools/bin/ab_norhs/libpsk.so tools/bin/ab_noboth/libpsk.so; do
  PSK_LIBRARY=$L timeout -k 10 300 python tools/grid_probe.py --side 8192 2>/dev/null | python -c "import sys,json;d=json.loads(sys.stdin.read());print('$L', d['grid_ms'])" || exit $?
done
