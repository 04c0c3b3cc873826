#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only; no sys/runtime trace with --pmc):
# FETCH_SIZE and WRITE_SIZE of the bench's kernels at each side in SIDES, plus the calibration
# streams; the sha256 of the libpsk.so the passes ran with goes beside them (bench.py only uses a
# traffic profile of the same build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2}
mkdir -p $OUT
export TMPDIR=/tmp
sha256sum pysolvers_amd/_lib/libpsk.so > $OUT/pmc_${TAG}_lib.sha256
ARGS=${PMC_ARGS:---steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --spmv10m 0 --config1 0 --config2 0 --config4 0 --general 0}
for S in ${SIDES:-16384 3163}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc side $S $C"
    timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${TAG}_${S}_$C -o run --output-format csv -- \
        python bench.py --side $S $ARGS > $OUT/pmc_${TAG}_${S}_$C.json 2> $OUT/pmc_${TAG}_${S}_$C.err
    rc=$?; [ $rc -ne 0 ] && { echo "pmc $S $C exit $rc"; tail -5 $OUT/pmc_${TAG}_${S}_$C.err; exit $rc; }
  done
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_${TAG}_calib_$C -o calib --output-format csv -- \
      tools/bin/pmc_calib > /dev/null 2> $OUT/pmc_${TAG}_calib_$C.err
  rc=$?; [ $rc -ne 0 ] && { echo "calib $C exit $rc"; exit $rc; }
done
echo "== pmc done"
