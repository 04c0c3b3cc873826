#!/bin/bash
# build_wt.sh WORKTREE OUTDIR: libpsk from another checkout (same flags as the Makefile)
set -e
src=$1/pysolvers_amd/csrc; out=$2
mkdir -p $out /tmp/bwt_$(basename $out)
pids=()
for f in runtime spmv pcg gmres dist shmcomm ilu amg dense mmio; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None -w -c $src/$f.hip -o /tmp/bwt_$(basename $out)/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o $out/libpsk.so /tmp/bwt_$(basename $out)/*.o -L/opt/rocm/lib -lrccl -lamdhip64 -ldl
