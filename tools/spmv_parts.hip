// spmv_parts.hip — where the one-shot CSR SpMV loses time against a pure stream (development tool).
// Variants of the shipped one-shot kernel (256-row tile per workgroup, 1280-entry LDS chunk) with
// parts removed, timed back to back at FDLaplacian2D(m):
//   full     : the shipped schedule (stream -> gather -> LDS -> ordered row sums -> nt store)
//   nogather : x[c] replaced by 1.0 (no gather; LDS and row sums kept)
//   nolds    : gather kept, products summed in registers per lane (no LDS, no barrier)
//   stream   : colidx/vals streamed and folded in registers, y stored (no gather, no LDS)
//   rowptr   : rowptr-only pass (per-row start/end loads + store)
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/bin/spmv_parts tools/spmv_parts.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__);                    \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int BS = 256, CH = 1280, KU = CH / BS, TR = 256;

template <int V>
__global__ __launch_bounds__(BS) void spmv_v(int64_t n, const int *__restrict__ rp, const int *__restrict__ ci,
                                             const double *__restrict__ va, const double *__restrict__ x,
                                             double *__restrict__ y) {
    __shared__ double prod[CH + BS];
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * TR, r1 = r0 + TR < n ? r0 + TR : n;
    const int last = rp[n] - 1;
    const int e0 = rp[r0], e1 = rp[r1];
    const int64_t row = r0 + tid;
    const bool has = row < r1;
    const int64_t rowc = has ? row : r0;
    if (V == 4) {
        const int rs = rp[rowc], re = rp[rowc + 1];
        if (has) __builtin_nontemporal_store((double)(re - rs), y + row);
        return;
    }
    int cc[KU];
    double vv[KU];
    const int c1 = e1 - e0 > CH ? e0 + CH : e1;
    const int base = e0 < last ? e0 : last;
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        const int e = e0 + k * BS + tid;
        const int ee = e < c1 ? e : base;
        cc[k] = __builtin_nontemporal_load(ci + ee);
        vv[k] = __builtin_nontemporal_load(va + ee);
    }
    const int rs = rp[rowc], re = rp[rowc + 1];
    double sum = 0.0;
    if (V == 3) {
#pragma unroll
        for (int k = 0; k < KU; ++k) sum += vv[k] + (double)cc[k];
        if (has) __builtin_nontemporal_store(sum + (double)(re - rs), y + row);
        return;
    }
    double pv[KU];
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        // V == 5: the gather stays inside the tile's own 256-row x window (dependent on colidx, but
        // every load an L1/L2 hit) — separates the dependent round trip from where x comes from
        const int64_t gi = V == 5 ? r0 + ((cc[k] & 255) < (r1 - r0) ? (cc[k] & 255) : 0) : (int64_t)cc[k];
        pv[k] = vv[k] * (V == 1 ? 1.0 : x[gi]);
    }
    if (V == 2) {
#pragma unroll
        for (int k = 0; k < KU; ++k) sum += pv[k];
        if (has) __builtin_nontemporal_store(sum + (double)(re - rs), y + row);
        return;
    }
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        const int e = e0 + k * BS + tid;
        prod[(e < c1 ? k * BS : CH) + tid] = pv[k];
    }
    __syncthreads();
    const int a = rs > e0 ? rs : e0, b = re < c1 ? re : c1;
    if (has)
        for (int e = a; e < b; ++e) sum = sum + prod[e - e0];
    if (has) __builtin_nontemporal_store(sum, y + row);
}

__global__ void fd2d(int64_t m, int *rp, int *ci, double *va, double dv, double ov) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = m * m;
    if (k > n) return;
    auto rpf = [m](int64_t k) -> int64_t {
        int64_t mk = k < m ? k : m, top = k - m * (m - 1);
        if (top < 0) top = 0;
        return 5 * k - mk - top - (k + m - 1) / m - k / m;
    };
    int64_t p = rpf(k);
    rp[k] = (int)p;
    if (k == n) return;
    const int64_t ix = k % m, iy = k / m;
    ci[p] = (int)k; va[p++] = dv;
    if (iy > 0) { ci[p] = (int)(k - m); va[p++] = ov; }
    if (iy < m - 1) { ci[p] = (int)(k + m); va[p++] = ov; }
    if (ix > 0) { ci[p] = (int)(k - 1); va[p++] = ov; }
    if (ix < m - 1) { ci[p] = (int)(k + 1); va[p++] = ov; }
}

__global__ void fillx(int64_t n, double *x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = 1.0 + (double)(i % 7) * 0.125;
}


// SELL-256 (sliced ELL, one 256-row slice per workgroup, slot-major inside a slice): entry j of
// row 256t+l at off[t] + j*256 + l; row lengths as uint8. Each lane sums its own row over slots
// 0..len-1 in stored order (bit-identical to csr_matvec), no LDS.
template <int W>
__global__ __launch_bounds__(BS) void spmv_sell(int64_t n, const int64_t *__restrict__ off,
                                                const unsigned char *__restrict__ len, const int *__restrict__ sc,
                                                const double *__restrict__ sv, const double *__restrict__ x,
                                                double *__restrict__ y) {
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x, row = t * TR + tid;
    const bool has = row < n;
    const int64_t o = off[t];
    const int w = (int)((off[t + 1] - o) / TR);
    const int L = has ? len[row] : 0;
    double sum = 0.0;
    if (w <= W) {
        int cc[W];
        double vv[W];
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < L) {
                cc[j] = __builtin_nontemporal_load(sc + o + (int64_t)j * TR + tid);
                vv[j] = __builtin_nontemporal_load(sv + o + (int64_t)j * TR + tid);
            }
        double xv[W];
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < L) xv[j] = x[cc[j]];
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < L) sum = sum + vv[j] * xv[j];
    } else {
        for (int j = 0; j < L; ++j)
            sum = sum + __builtin_nontemporal_load(sv + o + (int64_t)j * TR + tid) *
                            x[__builtin_nontemporal_load(sc + o + (int64_t)j * TR + tid)];
    }
    if (has) __builtin_nontemporal_store(sum, y + row);
}

__global__ void sell_fill(int64_t n, const int *rp, const int *ci, const double *va, const int64_t *off,
                          unsigned char *len, int *sc, double *sv) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n) return;
    const int64_t t = row / TR, l = row % TR, o = off[t];
    const int w = (int)((off[t + 1] - o) / TR);
    const int a = rp[row], b = rp[row + 1];
    len[row] = (unsigned char)(b - a);
    for (int j = 0; j < w; ++j) {
        const bool in = j < b - a;
        sc[o + (int64_t)j * TR + l] = in ? ci[a + j] : (int)row;
        sv[o + (int64_t)j * TR + l] = in ? va[a + j] : 0.0;
    }
}

typedef void (*Kern)(int64_t, const int *, const int *, const double *, const double *, double *);

int main(int argc, char **argv) {
    std::vector<int64_t> ms;
    for (int i = 1; i < argc; ++i) ms.push_back(atoll(argv[i]));
    if (ms.empty()) ms = {3163, 16384};
    for (int64_t m : ms) {
        const int64_t n = m * m, nnz = 5 * n - 4 * m;
        int *rp, *ci;
        double *va, *x, *y;
        CK(hipMalloc(&rp, (n + 1) * 4));
        CK(hipMalloc(&ci, nnz * 4));
        CK(hipMalloc(&va, nnz * 8));
        CK(hipMalloc(&x, n * 8));
        CK(hipMalloc(&y, n * 8));
        const double h = 2.0 / (double)(m + 1);
        fd2d<<<(unsigned)((n + 256) / 256), 256>>>(m, rp, ci, va, -4.0 / h / h, 1.0 / h / h);
        fillx<<<(unsigned)((n + 255) / 256), 256>>>(n, x);
        CK(hipDeviceSynchronize());
        struct V {
            const char *name;
            Kern k;
            double bytes;
        };
        const double full = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
        std::vector<V> vs = {{"full", spmv_v<0>, full},
                             {"nogather", spmv_v<1>, full - 8.0 * n},
                             {"nolds", spmv_v<2>, full},
                             {"stream", spmv_v<3>, full - 8.0 * n},
                             {"rowptr", spmv_v<4>, 4.0 * (n + 1) + 8.0 * n},
                             {"owngather", spmv_v<5>, full}};
        const unsigned grid = (unsigned)((n + TR - 1) / TR);
        // working-set probe: the same kernels over the first n/16 rows of the big matrix
        {
            const int64_t ns = n / 16;
            const unsigned gs = (unsigned)((ns + TR - 1) / TR);
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            for (int v = 0; v < 2; ++v) {
                Kern k = v == 0 ? spmv_v<0> : spmv_v<3>;
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    k<<<gs, BS>>>(ns, rp, ci, va, x, y);
                    CK(hipEventRecord(a));
                    for (int l = 0; l < 20; ++l) k<<<gs, BS>>>(ns, rp, ci, va, x, y);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float f;
                    CK(hipEventElapsedTime(&f, a, b));
                    best = std::min(best, f / 20);
                }
                const double nzs = 5.0 * ns, by = 12.0 * nzs + 4.0 * ns + (v == 0 ? 16.0 : 8.0) * ns;
                std::printf("m=%-6lld %-10s first n/16 rows: %8.1f us  %6.0f GB/s  %5.1f%%\n", (long long)m,
                            v == 0 ? "full" : "stream", best * 1e3, by / (best * 1e-3) / 1e9,
                            by / (best * 1e-3) / 8e12 * 100);
            }
        }
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<std::vector<float>> t(vs.size());
        const int R = 5, L = m >= 8192 ? 10 : 40;
        for (int r = 0; r < R; ++r)
            for (size_t i = 0; i < vs.size(); ++i) {
                vs[i].k<<<grid, BS>>>(n, rp, ci, va, x, y);
                CK(hipEventRecord(e0));
                for (int l = 0; l < L; ++l) vs[i].k<<<grid, BS>>>(n, rp, ci, va, x, y);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms_;
                CK(hipEventElapsedTime(&ms_, e0, e1));
                t[i].push_back(ms_ / L);
            }
        for (size_t i = 0; i < vs.size(); ++i) {
            std::sort(t[i].begin(), t[i].end());
            const double s = t[i][0] * 1e-3;
            std::printf("m=%-6lld %-10s %9.1f us  moved %6.2f GB  %6.0f GB/s  %5.1f%% of 8 TB/s\n", (long long)m,
                        vs[i].name, s * 1e6, vs[i].bytes / 1e9, vs[i].bytes / s / 1e9, vs[i].bytes / s / 8e12 * 100);
        }
        {   // SELL-256 of the same matrix (FD: width 5 in every slice)
            const int64_t nt = (n + TR - 1) / TR;
            std::vector<int> hrp(n + 1);
            CK(hipMemcpy(hrp.data(), rp, (n + 1) * 4, hipMemcpyDeviceToHost));
            std::vector<int64_t> hoff(nt + 1);
            hoff[0] = 0;
            for (int64_t tt = 0; tt < nt; ++tt) {
                int w = 0;
                for (int64_t r = tt * TR; r < std::min(n, tt * TR + TR); ++r) w = std::max(w, hrp[r + 1] - hrp[r]);
                hoff[tt + 1] = hoff[tt] + (int64_t)w * TR;
            }
            int64_t *doff;
            unsigned char *dlen;
            int *dsc;
            double *dsv, *y2;
            CK(hipMalloc(&doff, (nt + 1) * 8));
            CK(hipMalloc(&dlen, n));
            CK(hipMalloc(&dsc, hoff[nt] * 4));
            CK(hipMalloc(&dsv, hoff[nt] * 8));
            CK(hipMalloc(&y2, n * 8));
            CK(hipMemcpy(doff, hoff.data(), (nt + 1) * 8, hipMemcpyHostToDevice));
            sell_fill<<<(unsigned)((n + 255) / 256), 256>>>(n, rp, ci, va, doff, dlen, dsc, dsv);
            spmv_v<0><<<grid, BS>>>(n, rp, ci, va, x, y);
            spmv_sell<8><<<(unsigned)nt, BS>>>(n, doff, dlen, dsc, dsv, x, y2);
            CK(hipDeviceSynchronize());
            std::vector<double> h1(n), h2(n);
            CK(hipMemcpy(h1.data(), y, n * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), y2, n * 8, hipMemcpyDeviceToHost));
            const bool same = std::equal(h1.begin(), h1.end(), h2.begin(), [](double a, double b) {
                return std::memcmp(&a, &b, 8) == 0;
            });
            float best = 1e30f, bestc = 1e30f;
            for (int r = 0; r < 5; ++r) {
                for (int v = 0; v < 2; ++v) {
                    CK(hipEventRecord(e0));
                    for (int l = 0; l < L; ++l) {
                        if (v == 0) spmv_sell<8><<<(unsigned)nt, BS>>>(n, doff, dlen, dsc, dsv, x, y2);
                        else spmv_v<0><<<grid, BS>>>(n, rp, ci, va, x, y);
                    }
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float f;
                    CK(hipEventElapsedTime(&f, e0, e1));
                    if (v == 0) best = std::min(best, f / L); else bestc = std::min(bestc, f / L);
                }
            }
            const double moved = 12.0 * hoff[nt] + 1.0 * n + 8.0 * (nt + 1) + 16.0 * n;
            std::printf("m=%-6lld sell256    %9.1f us  csr-alg %6.0f GB/s (%5.1f%%)  moved %6.2f GB -> %6.0f GB/s  "
                        "bitwise=%s   [csr full interleaved %9.1f us]\n",
                        (long long)m, best * 1e3, full / (best * 1e-3) / 1e9, full / (best * 1e-3) / 8e12 * 100,
                        moved / 1e9, moved / (best * 1e-3) / 1e9, same ? "yes" : "NO", bestc * 1e3);
            CK(hipFree(doff));
            CK(hipFree(dlen));
            CK(hipFree(dsc));
            CK(hipFree(dsv));
            CK(hipFree(y2));
        }
        CK(hipFree(rp));
        CK(hipFree(ci));
        CK(hipFree(va));
        CK(hipFree(x));
        CK(hipFree(y));
    }
    return 0;
}
