// pcg_lab.hip — where does the SpMV lose time inside the PCG loop? (development tool, not shipped)
// Links libpsk.so and calls its internal launch_spmv in the modes the solvers use, back to back and
// interleaved with a K3-like streaming kernel that rewrites x (as K3 rewrites p), timing each case
// with HIP events on libpsk's stream.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -o tools/bin/pcg_lab tools/pcg_lab.hip \
//         -Lpysolvers_amd/_lib -lpsk -Wl,-rpath,$PWD/pysolvers_amd/_lib
//   tools/bin/pcg_lab 3163 16384
#include "../pysolvers_amd/csrc/psk_internal.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);             \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)
#define PK(x)                                                                           \
    do {                                                                                \
        int r_ = (x);                                                                   \
        if (r_ != 0) {                                                                  \
            std::printf("psk error %d (%s) at %d\n", r_, psk_last_error(), __LINE__);   \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

// K3-shaped stream: reads a, b, writes a (32 B/element traffic with 2 loads + 1 store of 16 B);
// NT = the store non-temporal
template <bool NT>
__global__ __launch_bounds__(256) void k3like(int64_t n, double *__restrict__ a, const double *__restrict__ b) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i + 1 < n) {
        psk::dv2 va = psk::ld2(a + i), vb = psk::ld2nt(b + i);
        va.x = va.x * 0.5 + vb.x * 0.25;
        va.y = va.y * 0.5 + vb.y * 0.25;
        if (NT) psk::st2nt(a + i, va);
        else psk::st2(a + i, va);
    }
}

__global__ void fill(int64_t n, double *x, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 31)) * 0xBF58476D1CE4E5B9ull;
        x[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    }
}

int main(int argc, char **argv) {
    PK(psk_set_device(0));
    psk::Context *c;
    PK(psk::ctx(&c));
    hipStream_t s = c->stream;
    for (int ai = 1; ai < argc; ++ai) {
        const int64_t m = atoll(argv[ai]), n = m * m, nnz = 5 * n - 4 * m;
        const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
        psk_csr *A = nullptr;
        PK(psk_csr_create_fd2d(-1.0, 1.0, m, &A));
        double *x, *y, *z, *part;
        int32_t *done;
        CK(hipMalloc(&x, n * 8));
        CK(hipMalloc(&y, n * 8));
        CK(hipMalloc(&z, n * 8));
        CK(hipMalloc(&part, 4096 * 8));
        CK(hipMalloc(&done, 4));
        CK(hipMemset(done, 0, 4));
        const unsigned nb = (unsigned)((n + 255) / 256);
        hipLaunchKernelGGL(fill, dim3(nb), dim3(256), 0, s, n, x, 1ull);
        hipLaunchKernelGGL(fill, dim3(nb), dim3(256), 0, s, n, z, 2ull);
        CK(hipStreamSynchronize(s));
        const int reps = m >= 8192 ? 10 : 50;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<hipEvent_t> ta(reps), tb(reps);
        for (int i = 0; i < reps; ++i) {
            CK(hipEventCreate(&ta[i]));
            CK(hipEventCreate(&tb[i]));
        }
        struct Case {
            const char *name;
            int mode;
            bool dot, flag, per_launch, interleave;
            int k3 = 0;   // interleaved kernel: 0 k3like on x, 1 k3like-nt on x, 2 k3like on z (not gathered)
        };
        const Case cases[] = {
            {"plain batch", psk::kSpmvPlain, false, false, false, false},
            {"dot batch", psk::kSpmvDot, true, false, false, false},
            {"dot+flag batch", psk::kSpmvDot, true, true, false, false},
            {"plain per-launch ev", psk::kSpmvPlain, false, false, true, false},
            {"dot+flag per-launch ev", psk::kSpmvDot, true, true, true, false},
            {"plain after k3like", psk::kSpmvPlain, false, false, true, true},
            {"dot+flag after k3like", psk::kSpmvDot, true, true, true, true},
            {"dot+flag after k3like-nt", psk::kSpmvDot, true, true, true, true, 1},
            {"dot+flag after k3like(z)", psk::kSpmvDot, true, true, true, true, 2},
            {"plain after k3like-nt", psk::kSpmvPlain, false, false, true, true, 1},
        };
        for (int round = 0; round < 3; ++round)
            for (const Case &cs : cases) {
                auto launch = [&]() {
                    PK(psk::launch_spmv(A, cs.mode, x, y, nullptr, nullptr, cs.dot ? part : nullptr,
                                        cs.flag ? done : nullptr, s));
                };
                launch();   // warm
                double ms = 0.0;
                if (!cs.per_launch) {
                    CK(hipEventRecord(e0, s));
                    for (int r = 0; r < reps; ++r) launch();
                    CK(hipEventRecord(e1, s));
                    CK(hipEventSynchronize(e1));
                    float f;
                    CK(hipEventElapsedTime(&f, e0, e1));
                    ms = f / reps;
                } else {
                    for (int r = 0; r < reps; ++r) {
                        const dim3 g3((unsigned)((n / 2 + 255) / 256));
                        if (cs.interleave && cs.k3 == 0) hipLaunchKernelGGL(k3like<false>, g3, dim3(256), 0, s, n, x, z);
                        if (cs.interleave && cs.k3 == 1) hipLaunchKernelGGL(k3like<true>, g3, dim3(256), 0, s, n, x, z);
                        if (cs.interleave && cs.k3 == 2) hipLaunchKernelGGL(k3like<false>, g3, dim3(256), 0, s, n, z, y);
                        CK(hipEventRecord(ta[r], s));
                        launch();
                        CK(hipEventRecord(tb[r], s));
                    }
                    CK(hipStreamSynchronize(s));
                    for (int r = 0; r < reps; ++r) {
                        float f;
                        CK(hipEventElapsedTime(&f, ta[r], tb[r]));
                        ms += f;
                    }
                    ms /= reps;
                }
                PK(psk::gridsum_check(c));
                if (round == 2)
                    std::printf("m=%-6lld %-26s %9.1f us  %6.0f GB/s  %5.1f%% of 8 TB/s\n", (long long)m, cs.name,
                                ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12 * 100);
            }
        for (int i = 0; i < reps; ++i) {
            CK(hipEventDestroy(ta[i]));
            CK(hipEventDestroy(tb[i]));
        }
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
        CK(hipFree(x));
        CK(hipFree(y));
        CK(hipFree(z));
        CK(hipFree(part));
        CK(hipFree(done));
        PK(psk_csr_destroy(A));
    }
    return 0;
}
