set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2m_pytest.log 2>&1 || { tail -30 gpurun_out/r2m_pytest.log; exit 1; }
tail -2 gpurun_out/r2m_pytest.log
PSK_BENCH_TRANSPORT=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --side 4096 --steps 20 --warmup 3 --repeats 2 --cpu-iters 0 > gpurun_out/r2_rehearsal_default.json 2> gpurun_out/r2_rehearsal_default.err || { grep -h PskError gpurun_out/r2_rehearsal_default.err | head -3; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r2_rehearsal_default.json')); print('default N=2 side 4096', d['value'])"
