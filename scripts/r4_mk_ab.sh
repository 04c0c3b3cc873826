#!/bin/bash
# Grid-schedule Markstein guard A/B: the in-tree build (exponent-bit range test beside the correction
# chain, wave-uniform fallback branch) vs tools/bin/ab_mkold (per-lane branch on |r| compares ahead
# of the chain), FD 8192^2 Gauss-Seidel factor and the SA level-3 operator, two rounds; then the
# triangular-solve / AMG / ILU GPU tests of the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4mk}
for r in 1; do
  for v in new old; do
    if [ $v = old ]; then export PSK_LIBRARY=$PWD/tools/bin/ab_mkold/libpsk.so; else unset PSK_LIBRARY; fi
    for l3 in 0 1; do
      timeout -k 10 300 python -u tools/grid_probe.py --side 8192 --level3 $l3 > $OUT/${TAG}_${v}_${l3}_$r.json 2>> $OUT/${TAG}.err
      c=$?; echo "$v l3=$l3 round $r exit $c $(cat $OUT/${TAG}_${v}_${l3}_$r.json)"; [ $c -eq 0 ] || exit $c
    done
  done
done
unset PSK_LIBRARY
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_part.py tests/test_gpu_amg.py > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -eq 0 ] || exit $c
# where a PCG+AMG iteration's time goes: kernel + copy trace of tools/bench_amg.py, window = its last PCG solve
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/${TAG}_amgprof -o run --output-format csv -- \
    python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg trace exit $c"; cat $OUT/${TAG}_amg.json
K=$(find $OUT/${TAG}_amgprof -name "*kernel_trace.csv" | head -1); C=$(find $OUT/${TAG}_amgprof -name "*memory_copy_trace.csv" | head -1)
python tools/window_trace.py $K pcg_gen_init $C > $OUT/${TAG}_amg_window.txt; head -40 $OUT/${TAG}_amg_window.txt
python tools/trace_stats.py $K > $OUT/${TAG}_amg_trace_stats.csv
rm -rf $OUT/${TAG}_amgprof
[ $c -eq 0 ] || exit $c
# sync-free geometry: workgroups per CU for configs[2]'s ILU apply (default = occupancy - 1)
for pc in default 2 4; do
  if [ $pc = default ]; then unset PSK_SYNCFREE_PER_CU; else export PSK_SYNCFREE_PER_CU=$pc; fi
  timeout -k 10 300 python -u tools/sf_probe.py 2896 >> $OUT/${TAG}_sf.jsonl 2>> $OUT/${TAG}_sf.err
  c=$?; echo "sf per_cu=$pc exit $c"; tail -1 $OUT/${TAG}_sf.jsonl; [ $c -eq 0 ] || exit $c
done
# partitioned kernel: per-phase stamps of an LDS hand-off chain (a -DPSK_PART_PROF build)
PSK_LIBRARY=$PWD/tools/bin/ab_partprof/libpsk.so PART_MICRO_CASES=chain1 timeout -k 10 300 python -u tools/part_micro.py > $OUT/${TAG}_partmicro.json 2> $OUT/${TAG}_partmicro.err
c=$?; echo "part_micro exit $c"; cat $OUT/${TAG}_partmicro.json; exit $c
