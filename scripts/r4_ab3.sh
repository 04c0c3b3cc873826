#!/bin/bash
# Round-4: GPU suite on the TPW=2 default, then A/B of the general (double-valued) path and the
# dot-mode back-to-back SpMV (PSK_SPMV_TIMED_MODE=1: plain_ms then times the kSpmvDot launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r4d}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -3 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 1 gen1=PSK_SPMV_LAYOUT=sliced,PSK_JACOBI_UNIFORM=0,PSK_SPMV_TPW=1 gen2=PSK_SPMV_LAYOUT=sliced,PSK_JACOBI_UNIFORM=0 dot1=PSK_SPMV_TIMED_MODE=1,PSK_SPMV_TPW=1 dot2=PSK_SPMV_TIMED_MODE=1 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
echo "ab exit $?"
timeout -k 10 700 python -u tools/ab_pcg.py --sides 3163 --rounds 2 band0= band1=PSK_K23_BANDS=1 band2=PSK_K23_BANDS=2 wt1=@tools/bin/ab_wt1/libpsk.so wt2=@tools/bin/ab_wt2/libpsk.so wt3=@tools/bin/ab_wt3/libpsk.so wt7=@tools/bin/ab_wt7/libpsk.so k2dpp=@tools/bin/ab_k2dpp/libpsk.so > $OUT/${TAG}_ab2.jsonl 2> $OUT/${TAG}_ab2.err
echo "ab exit $?"
# exit-fault probe: which path faults at exit under rocprofv3 (no GPU step runs after a fault)
for k in none pcg ilu amg; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_xp_$k -o run --output-format csv -- python tools/exit_probe.py $k > $OUT/${TAG}_xp_$k.out 2> $OUT/${TAG}_xp_$k.err
  c=$?; echo "exit probe $k: $c"; rm -rf $OUT/${TAG}_xp_$k
  [ $c -eq 0 ] || [ $c -eq 139 ] || exit $c
done
