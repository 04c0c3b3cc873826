#!/bin/bash
# Round 3: sync-free triangular solve with the poll sleep of wait_pub (PSK_WAIT_SLEEP x 64 clocks) —
# configs[2] GMRES(30)+ILUT 2896^2 ILU apply with libpsk variants (tools/bin/ab_pd*), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
A="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --general 0 --config1 0 --config4 0 --gmres 0 --scaling-side 0"
for v in sl4 sl16 sl48 sl4 sl16 sl48; do
  PSK_LIBRARY=tools/bin/ab_$v/libpsk.so timeout -k 10 300 python bench.py $A > $OUT/r3sl_$v.json 2> $OUT/r3sl_$v.err || { tail -3 $OUT/r3sl_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/r3sl_$v.json'));c=d['configs2_gmres30_ilut'];print('$v', c['schedules'], round(c['ilu_apply']['ms'],3), round(c['steps_per_s'],2), c['status'], repr(c['rec_resid_ratio']))"
done
