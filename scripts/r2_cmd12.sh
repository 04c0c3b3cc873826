set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_amg.py -x -q -k "grid or gauss" --timeout 240 --timeout-method thread > gpurun_out/r2h_pytest.log 2>&1 || { tail -30 gpurun_out/r2h_pytest.log; exit 1; }
tail -2 gpurun_out/r2h_pytest.log
timeout -k 10 400 python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 --cycles 2 > gpurun_out/r2h_amg.log 2>&1 || { tail -20 gpurun_out/r2h_amg.log; exit 1; }
grep '^{' gpurun_out/r2h_amg.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('amg', d['amg_apply_ms'], d['pcg_it_per_s'], d['fine_gs_sweep_ms_grid'], [ (l['level'], l.get('schedule'), round(l.get('op_ms', l.get('coarse_solve_ms',0)),2)) for l in d['per_level']])"
