# same-box A/B of libpsk builds: bench.py with the in-tree lib and with tools/bin/ab_old/libpsk.so
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for v in new ab_old; do
    if [ "$v" = new ]; then L=pysolvers_amd/_lib/libpsk.so; else L="tools/bin/$v/libpsk.so"; fi
    PSK_LIBRARY=$L timeout -k 10 300 python bench.py --cpu-iters 0 --config1 0 --steps 60 > gpurun_out/ab_${v}_$i.json 2>/dev/null
  done
done
