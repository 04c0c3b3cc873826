#!/bin/bash
# The driver's N=2 bench command rehearsed with both ranks on ONE GPU (PSK_BENCH_TRANSPORT=host:
# host shared-memory collectives; two processes share the CUs, so the numbers are NOT measurements),
# in both launch forms: torchrun, and `python bench.py --gpus 2` (bench.py spawns the ranks itself).
# Default workload (N=10M headline + the 16384^2 strong-scaling key), halo overlap on (default).
#   bash scripts/rehearsal_n2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${1:-r4}
PSK_BENCH_TRANSPORT=host timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/${TAG}_rehearsal_n2_torchrun.json 2> $OUT/${TAG}_rehearsal_n2_torchrun.err
rc=$?; tail -3 $OUT/${TAG}_rehearsal_n2_torchrun.err; cut -c1-400 $OUT/${TAG}_rehearsal_n2_torchrun.json; [ $rc -eq 0 ] || exit $rc
PSK_BENCH_TRANSPORT=host timeout -k 10 900 python bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/${TAG}_rehearsal_n2_spawn.json 2> $OUT/${TAG}_rehearsal_n2_spawn.err
rc=$?; tail -3 $OUT/${TAG}_rehearsal_n2_spawn.err; cut -c1-400 $OUT/${TAG}_rehearsal_n2_spawn.json; exit $rc
