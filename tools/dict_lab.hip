// dict_lab.hip — what bounds the sliced SpMV once the values are dictionary indices?
// FD 16384^2 (5-point, stored order diag, -m, +m, -1, +1), 256-row slices of width 5, 16-bit column
// deltas two per word. Variants (plain y = A x, non-temporal stores):
//   VAL   : double values in slot pairs (the product's "sliced" stream)
//   DGLB  : one-byte value indices, value = dict[idx] loaded from global memory (first dict cut)
//   DSEL  : one-byte value indices, value selected from the dictionary held in scalar registers
// each with SPW = 1, 2, 4 slices per 256-lane workgroup (the slices' loads issued together).
// Every variant must equal a plain CSR kernel bit for bit.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/dict_lab.hip -o tools/bin/dict_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);                       \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

constexpr int BS = 256, W = 5, NP = 3, NQ = 2;   // slice width, column words, index words
typedef double dv2 __attribute__((ext_vector_type(2)));

__global__ void fd2d(int64_t m, int *rp, int *ci, double *va, double dv, double ov) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = m * m;
    if (i >= n) return;
    const int64_t ix = i % m, iy = i / m;
    // entries before row i: whole grid lines (5m - 2 each, m fewer in line 0), then this line's rows
    int64_t e = iy * (5 * m - 2) - (iy > 0 ? m : 0) + ix * (5 - (iy == 0) - (iy == m - 1)) - (ix > 0 ? 1 : 0);
    rp[i] = (int)e;
    ci[e] = (int)i, va[e++] = dv;
    if (iy > 0) ci[e] = (int)(i - m), va[e++] = ov;
    if (iy < m - 1) ci[e] = (int)(i + m), va[e++] = ov;
    if (ix > 0) ci[e] = (int)(i - 1), va[e++] = ov;
    if (ix < m - 1) ci[e] = (int)(i + 1), va[e++] = ov;
    if (i == n - 1) rp[n] = (int)e;
}

__global__ void fillx(int64_t n, double *x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = 0.5 + 1e-3 * (double)(i % 9973) - 1e-7 * (double)(i % 101);
}

__global__ void csr_ref(int64_t n, const int *rp, const int *ci, const double *va, const double *x, double *y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int e = rp[i]; e < rp[i + 1]; ++e) s = s + va[e] * x[ci[e]];
    y[i] = s;
}

// slice t: column words at t*NP*BS + p*BS + l, index words at t*NQ*BS + q*BS + l, values at
// t*W*BS + (pairs 0,1: 2p*BS + 2l + k; slot 4: 4*BS + l)
__global__ void fill(int64_t n, const int *rp, const int *ci, const double *va, const double *dict, int *pw,
                     int *vw, double *vals) {
    const int64_t t = blockIdx.x, row = t * BS + threadIdx.x;
    const int l = threadIdx.x;
    const int a = row < n ? rp[row] : 0, len = row < n ? rp[row + 1] - a : 0;
    for (int p = 0; p < NP; ++p) {
        uint32_t w = 0;
        for (int k = 0; k < 2; ++k) {
            const int j = 2 * p + k;
            const int16_t d = j < len ? (int16_t)(ci[a + j] - row) : (int16_t)-32768;
            w |= (uint32_t)(uint16_t)d << (16 * k);
        }
        pw[t * NP * BS + p * BS + l] = (int)w;
    }
    for (int q = 0; q < NQ; ++q) {
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k) {
            const int j = 4 * q + k;
            uint32_t idx = 0;
            if (j < len && va[a + j] != dict[0]) idx = 1;
            w |= idx << (8 * k);
        }
        vw[t * NQ * BS + q * BS + l] = (int)w;
    }
    for (int j = 0; j < W; ++j) {
        const double v = j < len ? va[a + j] : 0.0;
        const int64_t pos = j < 4 ? t * W * BS + (j & ~1) * BS + 2 * l + (j & 1) : t * W * BS + 4 * BS + l;
        vals[pos] = v;
    }
}

enum { VAL = 0, DGLB = 1, DSEL = 2 };

__device__ __forceinline__ int32_t dec(int32_t row, uint32_t w, int k) {
    const int16_t d = (int16_t)(k ? (w >> 16) : (w & 0xffff));
    return d == (int16_t)-32768 ? -1 : row + (int32_t)d;
}

template <int MODE, int SPW>
__global__ __launch_bounds__(BS) void spmv(int64_t n, const int *__restrict__ pw, const int *__restrict__ vw,
                                            const double *__restrict__ vals, const double *__restrict__ dict,
                                            const double *__restrict__ x, double *__restrict__ y) {
    const int l = threadIdx.x;
    uint32_t cw[SPW][NP], iw[SPW][NQ];
    double vv[SPW][W], xv[SPW][W];
    double d0 = 0.0, d1 = 0.0;
    if (MODE == DSEL) {
        d0 = dict[0];
        d1 = dict[1];
    }
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        const int64_t t = (int64_t)blockIdx.x * SPW + s;
#pragma unroll
        for (int p = 0; p < NP; ++p) cw[s][p] = (uint32_t)__builtin_nontemporal_load(pw + t * NP * BS + p * BS + l);
        if (MODE == VAL) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(vals + t * W * BS + 2 * p * BS) + l);
                vv[s][2 * p] = v.x;
                vv[s][2 * p + 1] = v.y;
            }
            vv[s][4] = __builtin_nontemporal_load(vals + t * W * BS + 4 * BS + l);
        } else {
#pragma unroll
            for (int q = 0; q < NQ; ++q) iw[s][q] = (uint32_t)__builtin_nontemporal_load(vw + t * NQ * BS + q * BS + l);
        }
    }
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        const int32_t row = (int32_t)(((int64_t)blockIdx.x * SPW + s) * BS + l);
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int32_t c = dec(row, cw[s][j >> 1], j & 1);
            xv[s][j] = c >= 0 ? x[c] : 0.0;
        }
    }
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        const int64_t row = ((int64_t)blockIdx.x * SPW + s) * BS + l;
        double sum = 0.0;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const int32_t c = dec((int32_t)row, cw[s][j >> 1], j & 1);
            if (c < 0) continue;
            double v;
            if (MODE == VAL) v = vv[s][j];
            else {
                const uint32_t idx = (iw[s][j >> 2] >> (8 * (j & 3))) & 0xff;
                v = MODE == DGLB ? dict[idx] : (idx ? d1 : d0);
            }
            sum = sum + v * xv[s][j];
        }
        if (row < n) __builtin_nontemporal_store(sum, y + row);
    }
}

int main(int argc, char **argv) {
    const int64_t m = argc > 1 ? std::atoll(argv[1]) : 16384, n = m * m, nnz = 5 * n - 4 * m;
    const int64_t nt = (n + BS - 1) / BS;
    const double h = 2.0 / (double)(m + 1), dv = -4.0 / h / h, ov = 1.0 / h / h;
    int *rp, *ci, *pw, *vw;
    double *va, *x, *y, *yref, *vals, *dict;
    CK(hipMalloc(&rp, (n + 1) * 4));
    CK(hipMalloc(&ci, nnz * 4));
    CK(hipMalloc(&va, nnz * 8));
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMalloc(&yref, n * 8));
    CK(hipMalloc(&pw, nt * NP * BS * 4));
    CK(hipMalloc(&vw, nt * NQ * BS * 4));
    CK(hipMalloc(&vals, nt * W * BS * 8));
    CK(hipMalloc(&dict, 16));
    const double hd[2] = {dv, ov};
    CK(hipMemcpy(dict, hd, 16, hipMemcpyHostToDevice));
    const unsigned g = (unsigned)((n + 255) / 256);
    fd2d<<<g, 256>>>(m, rp, ci, va, dv, ov);
    fillx<<<g, 256>>>(n, x);
    csr_ref<<<g, 256>>>(n, rp, ci, va, x, yref);
    fill<<<(unsigned)nt, BS>>>(n, rp, ci, va, dict, pw, vw, vals);
    CK(hipDeviceSynchronize());
    CK(hipFree(ci));
    CK(hipFree(va));
    std::vector<double> href(n), hy(n);
    CK(hipMemcpy(href.data(), yref, n * 8, hipMemcpyDeviceToHost));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
        const char *name;
        void (*k)(int64_t, const int *, const int *, const double *, const double *, const double *, double *);
        int mode, spw;
    } vs[] = {{"VAL/1", spmv<VAL, 1>, VAL, 1},    {"VAL/2", spmv<VAL, 2>, VAL, 2},
              {"DGLB/1", spmv<DGLB, 1>, DGLB, 1}, {"DGLB/2", spmv<DGLB, 2>, DGLB, 2},
              {"DSEL/1", spmv<DSEL, 1>, DSEL, 1}, {"DSEL/2", spmv<DSEL, 2>, DSEL, 2},
              {"DSEL/4", spmv<DSEL, 4>, DSEL, 4}};
    for (auto &v : vs) {
        if (nt % v.spw) continue;
        const unsigned gg = (unsigned)(nt / v.spw);
        std::vector<float> ts;
        for (int r = 0; r < 25; ++r) {
            CK(hipEventRecord(e0));
            v.k<<<gg, BS>>>(n, pw, vw, vals, dict, x, y);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 5) ts.push_back(ms);
        }
        CK(hipMemcpy(hy.data(), y, n * 8, hipMemcpyDeviceToHost));
        const bool ok = std::memcmp(hy.data(), href.data(), n * 8) == 0;
        std::sort(ts.begin(), ts.end());
        const double bytes = v.mode == VAL ? (double)nt * BS * (W * 8 + NP * 4) + 16.0 * n
                                           : (double)nt * BS * (NQ * 4 + NP * 4) + 16.0 * n;
        std::printf("m=%lld %-7s best %7.1f us med %7.1f us  stream+x+y %6.2f GB -> %6.0f GB/s (%5.1f%%)  %s\n",
                    (long long)m, v.name, ts[0] * 1e3, ts[ts.size() / 2] * 1e3, bytes / 1e9,
                    bytes / (ts[ts.size() / 2] * 1e-3) / 1e9, bytes / (ts[ts.size() / 2] * 1e-3) / 1e9 / 80.0,
                    ok ? "bitwise" : "MISMATCH");
    }
    return 0;
}
