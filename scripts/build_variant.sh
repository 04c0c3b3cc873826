#!/bin/bash
# build_variant.sh NAME [extra hipcc flags...]: an experiment build of libpsk into tools/bin/ab_NAME/
# (objects in /tmp, the in-tree build untouched); CPU side only.
set -e
name=$1; shift
cd "$(dirname "$0")/../pysolvers_amd/csrc"
mkdir -p ../../tools/bin/ab_$name /tmp/bv_$name
pids=()
for f in runtime spmv pcg gmres dist shmcomm ilu amg dense mmio; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None -w "$@" -c $f.hip -o /tmp/bv_$name/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o ../../tools/bin/ab_$name/libpsk.so /tmp/bv_$name/*.o \
  -L/opt/rocm/lib -lrccl -lamdhip64 -ldl
