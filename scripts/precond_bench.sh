#!/bin/bash
# configs[2] and configs[4] measurements (GMRES+ILUT, PCG+AMG), each step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r1}
timeout -k 10 400 python tools/bench_gmres.py --side ${GM_SIDE:-2896} --steps 60 > gpurun_out/gmres_ilut_$TAG.json 2> gpurun_out/gmres_ilut_$TAG.err
rc=$?; cat gpurun_out/gmres_ilut_$TAG.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/gmres_ilut_$TAG.err; exit $rc; }
timeout -k 10 500 python tools/bench_amg.py --side ${AMG_SIDE:-8192} --levels 5 --iters 6 > gpurun_out/pcg_amg_$TAG.json 2> gpurun_out/pcg_amg_$TAG.err
rc=$?; cat gpurun_out/pcg_amg_$TAG.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/pcg_amg_$TAG.err; exit $rc; }
echo "== done"
