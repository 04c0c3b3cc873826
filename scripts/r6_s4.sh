#!/bin/bash
# Round-6 session 4: quad-ticket A/B (as s3), the changed GPU tests (AMG auto coarse, parity, progress through
# libpsk_lab.so, abi), then the driver's N = 2 command rehearsed on one GPU (host transport; the line's new
# "comm" breakdown) — never a measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s4}
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= quad=@tools/bin/ab_quad/libpsk.so noepi=@tools/bin/ab_noepi/libpsk.so nored=@tools/bin/ab_nored/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl; [ $c -le 1 ] || exit $c
timeout -k 10 700 python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_parity.py tests/test_gpu_progress.py tests/test_abi.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1
c=$?; echo "pytest exit $c"; tail -5 $OUT/${TAG}_pytest.log; [ $c -le 1 ] || exit $c
PSK_BENCH_TRANSPORT=host timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/${TAG}_rehearsal_n2.json 2> $OUT/${TAG}_rehearsal_n2.err
c=$?; echo "rehearsal exit $c"; tail -4 $OUT/${TAG}_rehearsal_n2.err
exit $c
