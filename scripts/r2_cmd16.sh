set -o pipefail
for NP in 2 4; do
PSK_BENCH_TRANSPORT=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 --master-port 2954$NP bench.py --gpus $NP --side 4096 --steps 20 --warmup 3 --repeats 2 --cpu-iters 0 > gpurun_out/r2_rehearsal_final_n$NP.json 2> gpurun_out/r2_rehearsal_final_n$NP.err || { grep -h PskError gpurun_out/r2_rehearsal_final_n$NP.err | head -3; tail -5 gpurun_out/r2_rehearsal_final_n$NP.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2_rehearsal_final_n$NP.json')); print('N=$NP side 4096', d['value'], d['n_gpus'], d['config'].get('parallelism'))"
done
