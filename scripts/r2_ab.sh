#!/bin/bash
# same-box A/B of libpsk builds after the GPU test suite: bench.py with the in-tree lib ("new") and
# the libraries under tools/bin/ab_<name>/ given as arguments; every GPU step time-limited, stop at
# the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${TAG:-r2a}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/${TAG}_pytest.log; exit 1; }
  tail -2 $OUT/${TAG}_pytest.log
fi
for i in 1 2; do
  for v in new "$@"; do
    if [ "$v" = new ]; then L=pysolvers_amd/_lib/libpsk.so; else L="tools/bin/ab_$v/libpsk.so"; fi
    PSK_LIBRARY=$L timeout -k 10 300 python bench.py --cpu-iters 0 ${BENCH_ARGS:---steps 60} > $OUT/${TAG}_ab_${v}_$i.json 2> $OUT/${TAG}_ab_${v}_$i.err \
      || { echo "bench $v failed"; tail -5 $OUT/${TAG}_ab_${v}_$i.err; exit 1; }
    python - "$OUT/${TAG}_ab_${v}_$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; t = d.get("spmv_N10M", {}); c = d.get("configs1_pcg_jacobi_4096", {})
print("%-6s it/s %.1f  spmv %.3f ms frac %.3f  plain %.3f ms | N10M %.4f ms (b2b %.4f) | 4096 %.0f it/s" % (
    sys.argv[2], d["value"], r["avg_launch_ms"], r["frac"], d.get("spmv_plain_batch20", {}).get("avg_launch_ms", 0),
    t.get("avg_launch_ms", 0), t.get("batch50", {}).get("avg_launch_ms", 0), c.get("pcg_it_per_s", 0)))
PY
  done
done
echo "== done"
