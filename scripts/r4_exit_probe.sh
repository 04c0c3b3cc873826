#!/bin/bash
# which libpsk launch leaves exit() faulting under rocprofv3: a plain launch (LDS schedule), then a
# cooperative one (sync-free schedule); stops at the first fault
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for k in none lds coop; do
  PSK_NO_TORCH=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/xp_$k -o run --output-format csv -- python -u tools/exit_probe.py $k > $OUT/xp_$k.log 2>&1
  c=$?; echo "$k exit $c"; rm -rf $OUT/xp_$k; [ $c -eq 0 ] || exit $c
done
