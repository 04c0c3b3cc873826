# rocprofv3 kernel traces of bench.py with the in-tree libpsk and with tools/bin/ab_old (A/B, same box)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abp_new -o run --output-format csv -- python bench.py --steps 20 --cpu-iters 0 --spmv10m 0 --config1 0 > gpurun_out/abp_new.json 2>/dev/null
PSK_LIBRARY=tools/bin/ab_old/libpsk.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abp_old -o run --output-format csv -- python bench.py --steps 20 --cpu-iters 0 --spmv10m 0 --config1 0 > gpurun_out/abp_old.json 2>/dev/null
