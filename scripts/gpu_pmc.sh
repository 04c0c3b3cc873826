#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only; no sys/runtime trace with --pmc):
# FETCH_SIZE and WRITE_SIZE of the bench's kernels, plus the calibration streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r1}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${PMC_ARGS:---steps 20 --warmup 2 --cpu-iters 0 --spmv10m 0 --config1 0}
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${TAG}_$C -o run --output-format csv -- \
      python bench.py $ARGS > $OUT/pmc_${TAG}_$C.json 2> $OUT/pmc_${TAG}_$C.err
  rc=$?; [ $rc -ne 0 ] && { echo "pmc $C exit $rc"; tail -5 $OUT/pmc_${TAG}_$C.err; exit $rc; }
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${TAG}_calib_$C -o calib --output-format csv -- \
      tools/bin/pmc_calib > /dev/null 2> $OUT/pmc_${TAG}_calib_$C.err
  rc=$?; [ $rc -ne 0 ] && { echo "calib $C exit $rc"; exit $rc; }
done
echo "== done"
