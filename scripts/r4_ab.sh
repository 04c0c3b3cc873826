#!/bin/bash
# Round-4 lab: A/B of SpMV/PCG variants (tools/ab_pcg.py) + parity of the TPW=2 kernel + the
# rocprofv3 exit-fault control (torch alone under the profiler).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r4b}
PSK_SPMV_TPW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_tpw2_tests.log 2>&1
c=$?; echo "tpw2 tests exit $c"; tail -2 $OUT/${TAG}_tpw2_tests.log; [ $c -le 1 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= tpw2=PSK_SPMV_TPW=2 k3pnt=@tools/bin/ab_k3pnt/libpsk.so ydef=@tools/bin/ab_ydef/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; [ $c -le 1 ] || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_tprof -o run --output-format csv -- python -c "import torch; t = torch.ones(1 << 20, device='cuda'); print(float(t.sum()))" > $OUT/${TAG}_torch_prof.out 2> $OUT/${TAG}_torch_prof.err
echo "torch-only profiled exit $?"
rm -rf $OUT/${TAG}_tprof
