set -o pipefail
timeout -k 10 300 python -u tools/part_micro.py > gpurun_out/r2p_micro.log 2>&1 || { tail -20 gpurun_out/r2p_micro.log; exit 1; }
cat gpurun_out/r2p_micro.log
PSK_LIBRARY=tools/bin/ab_pprof/libpsk.so timeout -k 10 300 python -u tools/part_micro.py > gpurun_out/r2p_micro_prof.log 2>&1 || { tail -20 gpurun_out/r2p_micro_prof.log; exit 1; }
