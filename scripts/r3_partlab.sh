#!/bin/bash
# Round 3 lab: partitioned trisolve publish order (LDS slot before the global store) and spin sleep 0,
# forced on configs[2]'s ILUT factors (PSK_TRISOLVE_PART=1); variants under tools/bin/ab_*, alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
A="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --general 0 --config1 0 --config4 0 --gmres 0 --scaling-side 0"
for v in base lf ps0 base lf ps0; do
  PSK_TRISOLVE_PART=1 PSK_LIBRARY=tools/bin/ab_$v/libpsk.so timeout -k 10 300 python bench.py $A > $OUT/r3pl_$v.json 2> $OUT/r3pl_$v.err || { tail -3 $OUT/r3pl_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r3pl_$v.json'));c=d['configs2_gmres30_ilut'];print('$v', c['schedules'], round(c['ilu_apply']['ms'],3), round(c['steps_per_s'],2), c['status'], repr(c['rec_resid_ratio']))"
done
