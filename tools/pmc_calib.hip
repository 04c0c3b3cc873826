// pmc_calib.hip — known-byte streams for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950.
// MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of 16-B/lane streams; other widths
// are uncalibrated. This runs one read kernel per access width the SpMV uses (4 B and 8 B per lane,
// default and non-temporal policy) plus 16 B, and one 8-B/lane write stream, each over 1 GiB.
//   hipcc -O3 --offload-arch=gfx950 -o pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d out -o calib --output-format csv -- ./pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T, bool NT>
__global__ __launch_bounds__(256) void rd(int64_t n, const T* __restrict__ a, T* __restrict__ out) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * per;
    const int64_t b1 = b0 + per < n ? b0 + per : n;
    T acc{};
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) {
        T v = NT ? __builtin_nontemporal_load(a + i) : a[i];
        acc += v;
    }
    if (acc == (T)123457) out[0] = acc;
}

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void rd16(int64_t n, const dv2* __restrict__ a, double* __restrict__ out) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * per;
    const int64_t b1 = b0 + per < n ? b0 + per : n;
    double acc = 0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) { dv2 v = __builtin_nontemporal_load(a + i); acc += v.x + v.y; }
    if (acc == 123457.0) out[0] = acc;
}

__global__ __launch_bounds__(256) void wr8(int64_t n, double* __restrict__ a) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * per;
    const int64_t b1 = b0 + per < n ? b0 + per : n;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) __builtin_nontemporal_store(1.0, a + i);
}

int main() {
    const int64_t bytes = 1ll << 30;
    char* buf; double* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes);
    for (int rep = 0; rep < 2; ++rep) {
        rd<int, false><<<1024, 256>>>(bytes / 4, (const int*)buf, (int*)out);
        rd<int, true><<<1024, 256>>>(bytes / 4, (const int*)buf, (int*)out);
        rd<double, false><<<1024, 256>>>(bytes / 8, (const double*)buf, out);
        rd<double, true><<<1024, 256>>>(bytes / 8, (const double*)buf, out);
        rd16<<<1024, 256>>>(bytes / 16, (const dv2*)buf, out);
        wr8<<<1024, 256>>>(bytes / 8, (double*)buf);
    }
    hipDeviceSynchronize();
    printf("pmc_calib: %lld bytes per kernel\n", (long long)bytes);
    return 0;
}
