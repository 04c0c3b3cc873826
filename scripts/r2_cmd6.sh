set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2g9_pytest.log 2>&1 || { grep -E "code|Error|FAIL|assert" gpurun_out/r2g9_pytest.log | head; exit 1; }
tail -2 gpurun_out/r2g9_pytest.log
TAG=r2g9 bash scripts/r2_trisolve.sh
