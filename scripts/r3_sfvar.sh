#!/bin/bash
# sync-free kernel variants on configs[2]'s ILU apply (GMRES(30)+RightILUT, FD 2896^2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in tools/bin/ab_head pysolvers_amd/_lib tools/bin/ab_sf_l0; do
  PSK_LIBRARY=$L/libpsk.so timeout -k 10 400 python bench.py --steps 20 --warmup 2 --cpu-iters 0 --general 0 --config1 0 --config4 0 --gmres 0 --scaling-side 0 > gpurun_out/r3sv_b.json 2> gpurun_out/r3sv_b.err || { tail -5 gpurun_out/r3sv_b.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/r3sv_b.json'));c2=d['configs2_gmres30_ilut']
print('$L', 'ilu_apply %.2f ms'%c2['ilu_apply']['ms'], 'steps/s %.2f'%c2['steps_per_s'])"
done
