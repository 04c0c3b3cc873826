#!/bin/bash
# round 6 (session 2): the driver's N = 4 command rehearsed with four ranks on ONE GPU (host shared-memory halo,
# mailbox dots; the ranks share the CUs, so the numbers are NOT measurements): the N > 1 line end to end at P = 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r6s21}
PSK_BENCH_TRANSPORT=host timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/${TAG}_rehearsal_n4_torchrun.json 2> $OUT/${TAG}_rehearsal_n4_torchrun.err
rc=$?; tail -4 $OUT/${TAG}_rehearsal_n4_torchrun.err; cut -c1-600 $OUT/${TAG}_rehearsal_n4_torchrun.json; exit $rc
