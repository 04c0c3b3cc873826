#!/bin/bash
# Round-6 session 6: K2 grid sums — block_sum butterflies + barriers (in-tree) vs DPP wave totals combined in LDS
# (tools/bin/ab_k2dpp) vs one tile per wave with DPP totals (tools/bin/ab_k2wave); the pair SpMV with grid-implied
# presence masks (tools/bin/ab_gridm), whose layout/shard tests run first on that build; the CSR layout's tile maps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${1:-r6s6}
PSK_LIBRARY=$PWD/tools/bin/ab_gridm/libpsk.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py tests/test_gpu_shards.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gridm.log 2>&1
c=$?; echo "pytest (gridm build) exit $c"; tail -3 $OUT/${TAG}_pytest_gridm.log; [ $c -le 1 ] || exit $c
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163,16384 --rounds 3 base= k2dpp=@tools/bin/ab_k2dpp/libpsk.so k2wave=@tools/bin/ab_k2wave/libpsk.so gridm=@tools/bin/ab_gridm/libpsk.so > $OUT/${TAG}_ab.jsonl 2> $OUT/${TAG}_ab.err
c=$?; echo "ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_ab.jsonl; [ $c -le 1 ] || exit $c
# the CSR layout in the loop (the north star's kernel): block order vs XCD bands vs chunked XCD maps
timeout -k 10 900 python -u tools/ab_pcg.py --sides 3163 --rounds 2 csr=PSK_SPMV_LAYOUT=csr csrband=PSK_SPMV_LAYOUT=csr,PSK_SPMV_CSR_BANDS=1 c512=PSK_SPMV_LAYOUT=csr,PSK_SPMV_CSR_CHUNK=512 c128=PSK_SPMV_LAYOUT=csr,PSK_SPMV_CSR_CHUNK=128 > $OUT/${TAG}_csr_ab.jsonl 2> $OUT/${TAG}_csr_ab.err
c=$?; echo "csr ab exit $c"; python tools/ab_summary.py $OUT/${TAG}_csr_ab.jsonl
exit $c
