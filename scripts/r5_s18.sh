#!/bin/bash
# Round-5 session 18: per-region wall times of the headline solve in several orders (tools/region_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s18}
timeout -k 10 300 python -u tools/region_probe.py > $OUT/${TAG}_regions.jsonl 2> $OUT/${TAG}_regions.err
c=$?; echo "probe exit $c"; cat $OUT/${TAG}_regions.jsonl; exit $c
