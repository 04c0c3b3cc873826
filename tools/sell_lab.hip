// sell_lab.hip — sliced-ELL (SELL) layouts for the bit-exact SpMV against the shipped CSR kernel
// (development tool). All variants sum each row sequentially in stored order (sum = sum + v*x,
// products rounded: -ffp-contract=off), so every y is bit-identical to scipy csr_matvec; checked.
//   csr      : the shipped one-shot CSR kernel (256-row tile, LDS-staged products)
//   sell     : SELL-256, slot-major inside a slice, per-row length array (uint8), loads predicated
//   sellneg  : SELL-256, padding slots hold column -1 (no length array): loads predicated on the
//              slice width (uniform), gather + add predicated on c >= 0
//   sell2    : SELL-512, two rows per lane (rows l and l+256 of a 512-row slice)
//   csrdot / selldot / sell2dot : the same with the PCG epilogue (y store, x[row]*y block partial)
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/bin/sell_lab tools/sell_lab.hip
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

__device__ __forceinline__ double blk_sum(double v, double *sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    return sh[0] + sh[1] + sh[2] + sh[3];
}

template <bool DOT>
__global__ __launch_bounds__(BS) void spmv_csr(int64_t n, const int *__restrict__ rp, const int *__restrict__ ci,
                                               const double *__restrict__ va, const double *__restrict__ x,
                                               double *__restrict__ y, double *__restrict__ part) {
    __shared__ double prod[CH + BS];
    __shared__ double sh[4];
    const int tid = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * TR, r1 = r0 + TR < n ? r0 + TR : n;
    const int last = rp[n] - 1;
    const int e0 = rp[r0], e1 = rp[r1];
    const int64_t row = r0 + tid;
    const bool has = row < r1;
    const int64_t rowc = has ? row : r0;
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
    const double eq = DOT ? x[rowc] : 0.0;
    double pv[KU];
#pragma unroll
    for (int k = 0; k < KU; ++k) pv[k] = vv[k] * x[cc[k]];
#pragma unroll
    for (int k = 0; k < KU; ++k) {
        const int e = e0 + k * BS + tid;
        prod[(e < c1 ? k * BS : CH) + tid] = pv[k];
    }
    __syncthreads();
    double sum = 0.0;
    const int a = rs > e0 ? rs : e0, b = re < c1 ? re : c1;
    if (has)
        for (int e = a; e < b; ++e) sum = sum + prod[e - e0];
    if (has) __builtin_nontemporal_store(sum, y + row);
    if (DOT) {
        const double s = blk_sum(has ? eq * sum : 0.0, sh);
        if (tid == 0) part[blockIdx.x] = s;
    }
}

// SELL-256 with a uint8 length per row
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

// SELL-(R*256) with column -1 padding; R rows per lane (rows l, l+256, ... of an R*256-row slice);
// slot j of row (l + 256 q) at off[t] + j*R*256 + q*256 + l
template <int W, int R, bool DOT>
__global__ __launch_bounds__(BS) void spmv_sneg(int64_t n, const int64_t *__restrict__ off, const int *__restrict__ sc,
                                                const double *__restrict__ sv, const double *__restrict__ x,
                                                double *__restrict__ y, double *__restrict__ part) {
    __shared__ double sh[4];
    constexpr int S = R * TR;
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x;
    const int64_t o = off[t];
    const int w = (int)((off[t + 1] - o) / S);
    double sum[R];
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < R; ++q) sum[q] = 0.0;
    if (w <= W) {
        int cc[R][W];
        double vv[R][W];
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < w)
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    cc[q][j] = __builtin_nontemporal_load(sc + o + (int64_t)j * S + q * TR + tid);
                    vv[q][j] = __builtin_nontemporal_load(sv + o + (int64_t)j * S + q * TR + tid);
                }
        double xv[R][W];
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < w)
#pragma unroll
                for (int q = 0; q < R; ++q) xv[q][j] = cc[q][j] >= 0 ? x[cc[q][j]] : 0.0;
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < w)
#pragma unroll
                for (int q = 0; q < R; ++q)
                    if (cc[q][j] >= 0) sum[q] = sum[q] + vv[q][j] * xv[q][j];
    } else {
#pragma unroll
        for (int q = 0; q < R; ++q)
            for (int j = 0; j < w; ++j) {
                const int c = __builtin_nontemporal_load(sc + o + (int64_t)j * S + q * TR + tid);
                if (c >= 0) sum[q] = sum[q] + __builtin_nontemporal_load(sv + o + (int64_t)j * S + q * TR + tid) * x[c];
            }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
        const int64_t row = t * S + q * TR + tid;
        if (row < n) {
            __builtin_nontemporal_store(sum[q], y + row);
            if (DOT) acc += x[row] * sum[q];
        }
    }
    if (DOT) {
        const double s = blk_sum(acc, sh);
        if (tid == 0) part[blockIdx.x] = s;
    }
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
    if (i < n) x[i] = 1.0 + (double)(i % 7) * 0.125 - (double)(i % 3) * 0.3;
}

// S-row slices, slot-major; len != nullptr: uint8 lengths and padding col = row; else col = -1.
// One thread per (slice, lane), so the last slice's lanes past n are padded too.
__global__ void sell_fill(int64_t n, int S, const int *rp, const int *ci, const double *va, const int64_t *off,
                          unsigned char *len, int *sc, double *sv) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t t = g / S, l = g % S;
    const int64_t nt = (n + S - 1) / S;
    if (t >= nt) return;
    const int64_t o = off[t], row = g;
    const int w = (int)((off[t + 1] - o) / S);
    const int a = row < n ? rp[row] : 0, L = row < n ? rp[row + 1] - a : 0;
    if (len && row < n) len[row] = (unsigned char)L;
    for (int j = 0; j < w; ++j) {
        const bool in = j < L;
        sc[o + (int64_t)j * S + l] = in ? ci[a + j] : (len ? (int)(row < n ? row : 0) : -1);
        sv[o + (int64_t)j * S + l] = in ? va[a + j] : 0.0;
    }
}

struct Sell {
    int S;
    int64_t nt, slots;
    int64_t *off;
    unsigned char *len;
    int *sc;
    double *sv;
};

static Sell make_sell(int64_t n, int S, bool withlen, const std::vector<int> &hrp, const int *rp, const int *ci,
                      const double *va) {
    Sell s{};
    s.S = S;
    s.nt = (n + S - 1) / S;
    std::vector<int64_t> hoff(s.nt + 1);
    hoff[0] = 0;
    for (int64_t tt = 0; tt < s.nt; ++tt) {
        int w = 0;
        for (int64_t r = tt * S; r < std::min(n, tt * S + S); ++r) w = std::max(w, hrp[r + 1] - hrp[r]);
        hoff[tt + 1] = hoff[tt] + (int64_t)w * S;
    }
    s.slots = hoff[s.nt];
    CK(hipMalloc(&s.off, (s.nt + 1) * 8));
    s.len = nullptr;
    if (withlen) CK(hipMalloc(&s.len, n));
    CK(hipMalloc(&s.sc, s.slots * 4));
    CK(hipMalloc(&s.sv, s.slots * 8));
    CK(hipMemcpy(s.off, hoff.data(), (s.nt + 1) * 8, hipMemcpyHostToDevice));
    sell_fill<<<(unsigned)((s.nt * S + 255) / 256), 256>>>(n, S, rp, ci, va, s.off, s.len, s.sc, s.sv);
    CK(hipDeviceSynchronize());
    return s;
}

static void free_sell(Sell &s) {
    CK(hipFree(s.off));
    if (s.len) CK(hipFree(s.len));
    CK(hipFree(s.sc));
    CK(hipFree(s.sv));
}

int main(int argc, char **argv) {
    std::vector<int64_t> ms;
    for (int i = 1; i < argc; ++i) ms.push_back(atoll(argv[i]));
    if (ms.empty()) ms = {3163, 4096, 16384};
    for (int64_t m : ms) {
        const int64_t n = m * m, nnz = 5 * n - 4 * m;
        int *rp, *ci;
        double *va, *x, *y, *yr, *part;
        CK(hipMalloc(&rp, (n + 1) * 4));
        CK(hipMalloc(&ci, nnz * 4));
        CK(hipMalloc(&va, nnz * 8));
        CK(hipMalloc(&x, n * 8));
        CK(hipMalloc(&y, n * 8));
        CK(hipMalloc(&yr, n * 8));
        CK(hipMalloc(&part, ((n + 255) / 256 + 1) * 8));
        const double h = 2.0 / (double)(m + 1);
        fd2d<<<(unsigned)((n + 256) / 256), 256>>>(m, rp, ci, va, -4.0 / h / h, 1.0 / h / h);
        fillx<<<(unsigned)((n + 255) / 256), 256>>>(n, x);
        CK(hipDeviceSynchronize());
        std::vector<int> hrp(n + 1);
        CK(hipMemcpy(hrp.data(), rp, (n + 1) * 4, hipMemcpyDeviceToHost));
        Sell s1 = make_sell(n, 256, true, hrp, rp, ci, va);
        Sell s2 = make_sell(n, 256, false, hrp, rp, ci, va);
        Sell s3 = make_sell(n, 512, false, hrp, rp, ci, va);
        const unsigned g256 = (unsigned)((n + 255) / 256), g512 = (unsigned)((n + 511) / 512);
        spmv_csr<false><<<g256, BS>>>(n, rp, ci, va, x, yr, part);   // reference result
        CK(hipDeviceSynchronize());
        std::vector<double> href(n), hy(n);
        CK(hipMemcpy(href.data(), yr, n * 8, hipMemcpyDeviceToHost));
        struct V {
            const char *name;
            int id;
        };
        std::vector<V> vs = {{"csr", 0},    {"sell", 1},    {"sellneg", 2}, {"sell2", 3},
                             {"csrdot", 4}, {"selldot", 5}, {"sell2dot", 6}};
        auto launch = [&](int id) {
            switch (id) {
            case 0: spmv_csr<false><<<g256, BS>>>(n, rp, ci, va, x, y, part); break;
            case 1: spmv_sell<8><<<g256, BS>>>(n, s1.off, s1.len, s1.sc, s1.sv, x, y); break;
            case 2: spmv_sneg<8, 1, false><<<g256, BS>>>(n, s2.off, s2.sc, s2.sv, x, y, part); break;
            case 3: spmv_sneg<8, 2, false><<<g512, BS>>>(n, s3.off, s3.sc, s3.sv, x, y, part); break;
            case 4: spmv_csr<true><<<g256, BS>>>(n, rp, ci, va, x, y, part); break;
            case 5: spmv_sneg<8, 1, true><<<g256, BS>>>(n, s2.off, s2.sc, s2.sv, x, y, part); break;
            case 6: spmv_sneg<8, 2, true><<<g512, BS>>>(n, s3.off, s3.sc, s3.sv, x, y, part); break;
            }
        };
        for (const V &v : vs) {   // bitwise check against the CSR result
            CK(hipMemset(y, 0xff, n * 8));
            launch(v.id);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hy.data(), y, n * 8, hipMemcpyDeviceToHost));
            if (std::memcmp(hy.data(), href.data(), n * 8) != 0)
                std::printf("m=%lld %s: NOT bitwise\n", (long long)m, v.name);
        }
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int R = 5, L = m >= 8192 ? 10 : 40;
        std::vector<std::vector<float>> t(vs.size());
        for (int r = 0; r < R; ++r)
            for (size_t i = 0; i < vs.size(); ++i) {
                launch(vs[i].id);
                CK(hipEventRecord(e0));
                for (int l = 0; l < L; ++l) launch(vs[i].id);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float f;
                CK(hipEventElapsedTime(&f, e0, e1));
                t[i].push_back(f / L);
            }
        const double full = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
        for (size_t i = 0; i < vs.size(); ++i) {
            std::sort(t[i].begin(), t[i].end());
            const double best = t[i][0] * 1e-3, med = t[i][R / 2] * 1e-3;
            std::printf("m=%-6lld %-9s best %9.1f us  med %9.1f us   csr-alg %6.0f GB/s = %5.1f%% of 8 TB/s\n",
                        (long long)m, vs[i].name, best * 1e6, med * 1e6, full / best / 1e9, full / best / 8e12 * 100);
        }
        std::fflush(stdout);
        free_sell(s1);
        free_sell(s2);
        free_sell(s3);
        CK(hipFree(rp));
        CK(hipFree(ci));
        CK(hipFree(va));
        CK(hipFree(x));
        CK(hipFree(y));
        CK(hipFree(yr));
        CK(hipFree(part));
    }
    return 0;
}
