# coarse-solve A/B of the LDS triangular-solve ring depth (PSK_LDS_DEPTH) on the AMG 8192^2 hierarchy
set -e
mkdir -p gpurun_out
for d in 1 2 3; do
  PSK_LDS_DEPTH=$d timeout -k 10 300 python tools/bench_amg.py --side 8192 --levels 5 --iters 6 > gpurun_out/lds_depth_$d.json 2> gpurun_out/lds_depth_$d.err
done
