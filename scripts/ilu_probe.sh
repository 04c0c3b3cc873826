set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_amg.py tests/test_gpu_newton.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_ilu.log 2>&1
rc=$?; tail -3 gpurun_out/t_ilu.log; [ $rc -gt 1 ] && exit $rc
for pc in 2 default; do
  if [ $pc = default ]; then unset PSK_SYNCFREE_PER_CU; else export PSK_SYNCFREE_PER_CU=$pc; fi
  timeout -k 10 200 python tools/bench_gmres.py --side 2048 --steps 30 > gpurun_out/gm_$pc.json 2>gpurun_out/gm_$pc.err || exit $?
  echo "per_cu=$pc"; cat gpurun_out/gm_$pc.json
done
