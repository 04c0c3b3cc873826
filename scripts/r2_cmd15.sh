set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2x_pytest.log 2>&1 || { tail -30 gpurun_out/r2x_pytest.log; exit 1; }
tail -2 gpurun_out/r2x_pytest.log
timeout -k 10 600 python bench.py --cpu-iters 0 --config2 0 --config4 0 --spmv10m 0 --general 0 > gpurun_out/r2x_bench.json 2> gpurun_out/r2x_bench.err || { tail -20 gpurun_out/r2x_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r2x_bench.json')); print(d['value'], d['roofline']['avg_launch_ms'], d['repeats']['it_s'], d['configs1_pcg_jacobi_4096']['pcg_it_per_s'])"
