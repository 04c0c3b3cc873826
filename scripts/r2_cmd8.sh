set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_part.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r2p_pytest.log 2>&1 || { tail -30 gpurun_out/r2p_pytest.log; exit 1; }
tail -2 gpurun_out/r2p_pytest.log
for lib in pysolvers_amd/_lib/libpsk.so tools/bin/ab_sleep0/libpsk.so; do
echo "== $lib"
PART_MICRO_CASES=chain1,chain64 PSK_LIBRARY=$lib timeout -k 10 300 python -u tools/part_micro.py > gpurun_out/r2p_micro.log 2>&1 || { tail -20 gpurun_out/r2p_micro.log; exit 1; }
cat gpurun_out/r2p_micro.log
PSK_LIBRARY=$lib timeout -k 10 600 python -u tools/ilu_probe.py 1024 2048 > gpurun_out/r2p_probe.log 2>&1 || { tail -20 gpurun_out/r2p_probe.log; exit 1; }
grep '^{' gpurun_out/r2p_probe.log | cut -c1-400
done
