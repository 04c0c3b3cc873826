set -o pipefail
export PSK_TRISOLVE_VERBOSE=1
timeout -k 10 400 python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 --cycles 2 > gpurun_out/r2p_amg.log 2>&1 || { tail -20 gpurun_out/r2p_amg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2p_amg.log | cut -c1-600
timeout -k 10 500 python -u tools/bench_gmres.py --side 2896 --restart 30 --steps 60 > gpurun_out/r2p_gmres.log 2>&1 || { tail -20 gpurun_out/r2p_gmres.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2p_gmres.log | cut -c1-600
