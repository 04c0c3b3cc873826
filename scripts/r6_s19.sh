#!/bin/bash
# round 6 (session 2): the PMC calibration passes of scripts/gpu_pmc.sh alone (r6s2fb's side passes ran; tools/bin/pmc_calib
# was missing from that tree)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s2fb}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${TAG}_calib_$C -o calib --output-format csv -- \
      tools/bin/pmc_calib > /dev/null 2> $OUT/pmc_${TAG}_calib_$C.err
  rc=$?; [ $rc -ne 0 ] && { echo "calib $C exit $rc"; exit $rc; }
done
echo "== calib done"
