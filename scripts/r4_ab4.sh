#!/bin/bash
# Round-4: the strip triangular-solve schedule (tests, ILU apply A/B), then the PCG A/Bs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r4e}
timeout -k 10 500 python -u -m pytest tests/test_gpu_strip.py -x -v --timeout 300 --timeout-method thread > $OUT/${TAG}_strip_tests.log 2>&1
c=$?; echo "strip tests exit $c"; tail -5 $OUT/${TAG}_strip_tests.log; [ $c -le 1 ] || exit $c
PSK_TRISOLVE_VERBOSE=1 timeout -k 10 400 python -u tools/ab_ilu.py 1024 2896 > $OUT/${TAG}_ab_ilu.jsonl 2> $OUT/${TAG}_ab_ilu.err
c=$?; echo "ab_ilu exit $c"; cat $OUT/${TAG}_ab_ilu.jsonl; grep "psk trisolve" $OUT/${TAG}_ab_ilu.err | tail -4; [ $c -le 1 ] || exit $c
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 1 gen1=PSK_SPMV_LAYOUT=sliced,PSK_JACOBI_UNIFORM=0,PSK_SPMV_TPW=1 gen2=PSK_SPMV_LAYOUT=sliced,PSK_JACOBI_UNIFORM=0 dot1=PSK_SPMV_TIMED_MODE=1,PSK_SPMV_TPW=1 dot2=PSK_SPMV_TIMED_MODE=1 > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; [ $c -le 1 ] || exit $c
timeout -k 10 700 python -u tools/ab_pcg.py --sides 3163 --rounds 2 band0= band1=PSK_K23_BANDS=1 band2=PSK_K23_BANDS=2 wt1=@tools/bin/ab_wt1/libpsk.so wt2=@tools/bin/ab_wt2/libpsk.so wt3=@tools/bin/ab_wt3/libpsk.so wt7=@tools/bin/ab_wt7/libpsk.so k2dpp=@tools/bin/ab_k2dpp/libpsk.so > $OUT/${TAG}_ab2.jsonl 2> $OUT/${TAG}_ab2.err
echo "ab2 exit $?"
