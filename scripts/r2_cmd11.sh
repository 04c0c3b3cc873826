set -o pipefail
for lib in pysolvers_amd/_lib/libpsk.so tools/bin/ab_sl1/libpsk.so tools/bin/ab_sl0/libpsk.so; do  # default sleep 2, sl1 = 1, sl0 = 4
echo "== $lib"
PART_MICRO_CASES=chain1,chain64 PSK_LIBRARY=$lib timeout -k 10 300 python -u tools/part_micro.py > gpurun_out/r2s_micro.log 2>&1 || { tail -20 gpurun_out/r2s_micro.log; exit 1; }
cut -c1-220 gpurun_out/r2s_micro.log | grep '^{'
PSK_LIBRARY=$lib timeout -k 10 600 python -u tools/ilu_probe.py 2048 > gpurun_out/r2s_probe.log 2>&1 || { tail -20 gpurun_out/r2s_probe.log; exit 1; }
grep '^{' gpurun_out/r2s_probe.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['m'], 'part', d['part_ms'], 'syncfree', d['syncfree_ms'])"
done
