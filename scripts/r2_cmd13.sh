set -o pipefail
export PSK_BENCH_TRANSPORT=host
for SIDE in 1024 2048; do
NP=2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port 295$((SIDE/64)) bench.py --gpus $NP --side $SIDE --steps 20 --warmup 3 --repeats 2 --cpu-iters 0 > gpurun_out/r2_rehearsal_s$SIDE.json 2> gpurun_out/r2_rehearsal_s$SIDE.err || { echo "side=$SIDE failed"; grep -h "PskError" gpurun_out/r2_rehearsal_s$SIDE.err | head -2; continue; }
python -c "import json; d=json.load(open('gpurun_out/r2_rehearsal_s$SIDE.json')); print('side=$SIDE', d['value'], d['n_gpus'])"
done
