#!/bin/bash
# AddressSanitizer + UBSan run of libpsk's host-only C++ (MatrixMarket reader, SA aggregation,
# sharding plan) on the CPU — no GPU: every libpsk source rebuilt with the sanitizers on its HOST
# side only (-Xarch_host; device code as shipped) into tools/bin/asan/, driven by tools/asan_host.cpp.
# Output: profiles/r3_asan_host.txt
set -e -o pipefail
cd "$(dirname "$0")/.."
B=tools/bin/asan; mkdir -p $B /tmp/asan_obj
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
pids=()
for f in runtime spmv pcg gmres dist shmcomm ilu amg mmio; do
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -w $SAN \
      -c pysolvers_amd/csrc/$f.hip -o /tmp/asan_obj/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -fPIC --offload-arch=gfx950 -shared -fsanitize=address,undefined -shared-libasan \
    -o $B/libpsk.so /tmp/asan_obj/*.o -L/opt/rocm/lib -lrccl -lamdhip64
/opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -fsanitize=address,undefined -shared-libasan -fno-omit-frame-pointer \
    -Iinclude tools/asan_host.cpp -o $B/asan_host -L$B -lpsk -Wl,-rpath,$PWD/$B -Wl,-rpath,$(dirname $(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)) -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib
{
  echo "# $(date -u +%F) scripts/asan_host.sh: libpsk host code under -fsanitize=address,undefined (clang $(/opt/rocm/llvm/bin/clang++ --version | head -1 | sed 's/.*version //'))"
  echo "# sources sha256: $(cat pysolvers_amd/csrc/*.hip pysolvers_amd/csrc/*.hpp | sha256sum | cut -c1-16)"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:verify_asan_link_order=0 UBSAN_OPTIONS=print_stacktrace=1 LSAN_OPTIONS=suppressions=$PWD/tools/lsan_hip.supp \
      $B/asan_host tests/golden/mtx 2>&1
  echo "# exit $?"
} | tee profiles/r3_asan_host.txt
