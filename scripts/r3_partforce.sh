#!/bin/bash
# Round 3: the partitioned triangular-solve schedule forced (PSK_TRISOLVE_PART=1) on the configs[4]
# SA levels and on the configs[2] ILUT factors (FD 2896^2), against the default choice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
PSK_TRISOLVE_PART=1 timeout -k 10 400 python tools/level_sched_probe.py --side 8192 > $OUT/r3pf_levels.json 2> $OUT/r3pf_levels.err || { tail -3 $OUT/r3pf_levels.err; exit 1; }
cut -c1-420 $OUT/r3pf_levels.json
A="--steps 20 --warmup 2 --repeats 1 --cpu-iters 0 --general 0 --config1 0 --config4 0 --gmres 0 --scaling-side 0"
PSK_TRISOLVE_PART=1 timeout -k 10 500 python bench.py $A > $OUT/r3pf_ilu.json 2> $OUT/r3pf_ilu.err || { tail -3 $OUT/r3pf_ilu.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/r3pf_ilu.json'));c=d['configs2_gmres30_ilut'];print('ILU forced part', c['schedules'], c['ilu_apply']['ms'], c['steps_per_s'], c.get('status'), c.get('rec_resid_ratio'))"
