#!/bin/bash
# branch-free sync-free / LDS triangular-solve kernels: GPU suite, then configs[2] (ILU) and configs[4]
# (AMG) against the previous kernels (ab_head)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3sf_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3sf_tests.log; [ $rc -eq 0 ] || exit $rc
for L in pysolvers_amd/_lib tools/bin/ab_head; do
  PSK_LIBRARY=$L/libpsk.so timeout -k 10 400 python bench.py --steps 20 --warmup 2 --cpu-iters 0 --general 0 --config1 0 --gmres 0 --scaling-side 0 > gpurun_out/r3sf_b.json 2> gpurun_out/r3sf_b.err || { tail -5 gpurun_out/r3sf_b.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/r3sf_b.json'));c2=d['configs2_gmres30_ilut'];c4=d['configs4_pcg_amg_8192']
print('$L', 'ilu_apply %.2f ms'%c2['ilu_apply']['ms'], 'steps/s %.2f'%c2['steps_per_s'], '| amg_apply %.1f ms'%c4['amg_apply_ms'], 'pcg+amg it/s %.3f'%c4['pcg_it_per_s'], 'fineGS %.3f'%c4['fine_gs_sweep']['ms'], 'coarse %.2f'%c4['coarse_solve_ms'])"
done
