set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_newton.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2n_pytest.log 2>&1 || { grep -E "code|Error|FAIL|assert" gpurun_out/r2n_pytest.log | head -20; exit 1; }
tail -2 gpurun_out/r2n_pytest.log
