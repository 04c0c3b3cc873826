set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_part.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r2p_pytest.log 2>&1 || { tail -40 gpurun_out/r2p_pytest.log; exit 1; }
tail -8 gpurun_out/r2p_pytest.log
timeout -k 10 600 python -u tools/ilu_probe.py 1024 2048 > gpurun_out/r2p_probe.log 2>&1 || { tail -20 gpurun_out/r2p_probe.log; exit 1; }
cat gpurun_out/r2p_probe.log
