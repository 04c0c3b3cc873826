#!/bin/bash
# partitioned trisolve with a branch-free fast path: configs[4] (AMG level 2) and configs[2]'s ILU with
# the partitioned schedule forced (PSK_TRISOLVE_PART=1), against the previous kernel (ab_head)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in pysolvers_amd/_lib tools/bin/ab_head; do
  PSK_LIBRARY=$L/libpsk.so timeout -k 10 400 python bench.py --steps 20 --warmup 2 --cpu-iters 0 --general 0 --config1 0 --config2 0 --gmres 0 --scaling-side 0 > gpurun_out/r3pb_b.json 2> gpurun_out/r3pb_b.err || { tail -5 gpurun_out/r3pb_b.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/r3pb_b.json'));c4=d['configs4_pcg_amg_8192']
print('$L', 'amg_apply %.1f ms'%c4['amg_apply_ms'], 'pcg+amg it/s %.3f'%c4['pcg_it_per_s'], 'fineGS %.3f'%c4['fine_gs_sweep']['ms'], 'coarse %.2f'%c4['coarse_solve_ms'])"
  PSK_TRISOLVE_PART=1 PSK_LIBRARY=$L/libpsk.so timeout -k 10 400 python bench.py --steps 20 --warmup 2 --cpu-iters 0 --general 0 --config1 0 --config4 0 --gmres 0 --scaling-side 0 > gpurun_out/r3pb_c.json 2> gpurun_out/r3pb_c.err || { tail -5 gpurun_out/r3pb_c.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/r3pb_c.json'));c2=d['configs2_gmres30_ilut']
print('$L PART=1', 'ilu_apply %.2f ms'%c2['ilu_apply']['ms'], 'schedules', c2['schedules'])"
done
