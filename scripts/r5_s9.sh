#!/bin/bash
# Round-5 session 9: grid-schedule progress probe (occupier XCD placement), the GPU files after
# test_gpu_progress, DPP A/B, fixed cost + timeline, PCG+AMG with the dense coarse solve (rocprof stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r5s9}
ok() { local c=$1; [ $c -eq 0 ] || [ $c -eq 1 ]; }
timeout -k 10 240 python -u tools/progress_probe.py --factor gs --m 1024 --sched grid --wgs 128,192,224,240,248 --seconds 3 > $OUT/${TAG}_probe.jsonl 2> $OUT/${TAG}_probe.err
c=$?; echo "probe exit $c"; cat $OUT/${TAG}_probe.jsonl; ok $c || exit $c
timeout -k 10 400 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1
c=$?; echo "tests exit $c"; tail -3 $OUT/${TAG}_tests.log; ok $c || exit $c
[ $c -eq 0 ] || exit 1
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 base= dpp=@tools/bin/ab_dpp/libpsk.so dpptpw4=@tools/bin/ab_dpptpw4/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python - $OUT/${TAG}_ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["result"]
    if isinstance(r, dict):
        print(d["round"], d["variant"], " | ".join("%s: %.1f it/s spmv %.4f plain %.4f %s" % (k, v["it_s"], v["spmv_ms"], v["plain_ms"], v["resid_bits"][-6:] + "/" + v["x_sha"][:6]) for k, v in r.items()))
    else: print(d)
PY
ok $c || exit $c
timeout -k 10 600 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 2 csr=PSK_SPMV_LAYOUT=csr csrband=PSK_SPMV_LAYOUT=csr,PSK_SPMV_CSR_BANDS=1 >> $OUT/${TAG}_ab.jsonl 2>> $OUT/${TAG}_ab.err
c=$?; echo "ab csr exit $c"; tail -4 $OUT/${TAG}_ab.jsonl | cut -c1-400; ok $c || exit $c
timeout -k 10 300 python -u tools/fixed_cost.py > $OUT/${TAG}_fixed.json 2> $OUT/${TAG}_fixed.err
c=$?; echo "fixed exit $c"; cat $OUT/${TAG}_fixed.json; ok $c || exit $c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run --output-format csv -- python -u tools/fixed_cost.py --iters 20,200 --reps 5 > $OUT/${TAG}_fixedprof.json 2> $OUT/${TAG}_fixedprof.err
c=$?; echo "profiled exit $c"; ok $c || exit $c
python tools/solve_gaps.py $(find $OUT/${TAG}_prof -name "*kernel_trace.csv" | head -1) --iters 20 > $OUT/${TAG}_gaps.json
head -40 $OUT/${TAG}_gaps.json
cp $(find $OUT/${TAG}_prof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_kernel_stats.csv
rm -rf $OUT/${TAG}_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_amgprof -o run --output-format csv -- python -u tools/bench_amg.py --side 8192 --levels 5 --iters 6 > $OUT/${TAG}_amg.json 2> $OUT/${TAG}_amg.err
c=$?; echo "amg exit $c"; tail -c 3000 $OUT/${TAG}_amg.json; ok $c || exit $c
cp $(find $OUT/${TAG}_amgprof -name "*kernel_stats.csv" | head -1) $OUT/${TAG}_amg_kernel_stats.csv
rm -rf $OUT/${TAG}_amgprof
