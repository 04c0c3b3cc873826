#!/bin/bash
# Round 3: the driver's N=2 bench command rehearsed with both ranks on ONE GPU (PSK_BENCH_TRANSPORT=host:
# host shared-memory collectives; two processes share the CUs, so the numbers are NOT measurements),
# default workload (N=10M headline + the 16384^2 strong-scaling key), halo overlap on (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
PSK_BENCH_TRANSPORT=host timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 > $OUT/r3_rehearsal_n2.json 2> $OUT/r3_rehearsal_n2.err
rc=$?; tail -3 $OUT/r3_rehearsal_n2.err; cut -c1-600 $OUT/r3_rehearsal_n2.json; exit $rc
