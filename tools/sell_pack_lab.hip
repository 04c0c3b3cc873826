// sell_pack_lab.hip — packed column encodings of the sliced (SELL-256) SpMV layout (development tool).
// All variants: one 256-row slice per workgroup, one row per lane, each row summed in stored order
// (bit-identical to csr_matvec; checked against the wide variant). FD matrix, every slice packable.
//   wide    : int32 columns, one 4-B load per slot (the shipped "sliced_wide")
//   pk16    : int16 deltas (column - row), one 2-B load per slot (128 B per wave instruction)
//   pk2     : two int16 deltas per int32 word (slots 2p, 2p+1 of a row), one 4-B load per slot PAIR
//   pk2v2   : pk2 + values of slots 2p, 2p+1 adjacent (one 16-B load per pair, 8-B load for an odd last)
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o tools/bin/sell_pack_lab tools/sell_pack_lab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
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

constexpr int BS = 256, S = 256, W = 8;
typedef double dv2 __attribute__((ext_vector_type(2)));

// V: 0 wide, 1 pk16, 2 pk2, 3 pk2v2. off[t] = slot offset (w*256 per slice); for pk2 the column words
// of slice t start at woff[t] (ceil(w/2)*256 words).
template <int V>
__global__ __launch_bounds__(BS) void spmv(int64_t n, const int64_t *__restrict__ off, const int64_t *__restrict__ woff,
                                           const int *__restrict__ c32, const short *__restrict__ c16,
                                           const double *__restrict__ va, const double *__restrict__ x,
                                           double *__restrict__ y) {
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x, row = t * S + tid;
    const int64_t o = off[t];
    const int w = (int)((off[t + 1] - o) / S);
    int cc[W];
    double vv[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        cc[j] = -1;
        vv[j] = 0.0;
    }
    if (V == 0 || V == 1) {
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < w) {
                if (V == 0) cc[j] = __builtin_nontemporal_load(c32 + o + j * S + tid);
                else {
                    const short d = __builtin_nontemporal_load(c16 + o + j * S + tid);
                    cc[j] = d == SHRT_MIN ? -1 : (int)row + d;
                }
                vv[j] = __builtin_nontemporal_load(va + o + j * S + tid);
            }
    } else {
        const int64_t wo = woff[t];
#pragma unroll
        for (int p = 0; p < W / 2; ++p)
            if (2 * p < w) {
                const int word = __builtin_nontemporal_load(c32 + wo + p * S + tid);
                const short d0 = (short)(word & 0xffff), d1 = (short)(word >> 16);
                cc[2 * p] = d0 == SHRT_MIN ? -1 : (int)row + d0;
                cc[2 * p + 1] = d1 == SHRT_MIN ? -1 : (int)row + d1;
                if (V == 2) {
                    vv[2 * p] = __builtin_nontemporal_load(va + o + (2 * p) * S + tid);
                    if (2 * p + 1 < w) vv[2 * p + 1] = __builtin_nontemporal_load(va + o + (2 * p + 1) * S + tid);
                } else {
                    // values: pair p at o + 2p*S (+2*tid), an odd last slot at o + (w-1)*S + tid
                    if (2 * p + 1 < w) {
                        const dv2 v2 = __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(va + o + 2 * p * S) + tid);
                        vv[2 * p] = v2.x;
                        vv[2 * p + 1] = v2.y;
                    } else {
                        vv[2 * p] = __builtin_nontemporal_load(va + o + 2 * p * S + tid);
                    }
                }
            }
    }
    double xv[W];
#pragma unroll
    for (int j = 0; j < W; ++j) xv[j] = cc[j] >= 0 ? x[cc[j]] : 0.0;
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < W; ++j)
        if (cc[j] >= 0) sum = sum + vv[j] * xv[j];
    if (row < n) __builtin_nontemporal_store(sum, y + row);
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

// all encodings of one slice per workgroup
__global__ void fill(int64_t n, const int *rp, const int *ci, const double *va, const int64_t *off,
                     const int64_t *woff, int *c32w, short *c16, int *c32p, double *vw, double *vp) {
    const int64_t t = blockIdx.x, l = threadIdx.x, row = t * S + l;
    const int64_t o = off[t], wo = woff[t];
    const int w = (int)((off[t + 1] - o) / S);
    const int a = row < n ? rp[row] : 0, L = row < n ? rp[row + 1] - a : 0;
    for (int j = 0; j < w; ++j) {
        const bool in = j < L;
        const int c = in ? ci[a + j] : -1;
        const double v = in ? va[a + j] : 0.0;
        c32w[o + (int64_t)j * S + l] = c;
        c16[o + (int64_t)j * S + l] = in ? (short)(c - row) : (short)SHRT_MIN;
        vw[o + (int64_t)j * S + l] = v;
        // pair layout of values: pair p occupies [o + 2p*S, o + 2p*S + 2S) with lane l at 2l, 2l+1
        const int p = j / 2;
        if (2 * p + 1 < w) vp[o + 2 * p * S + 2 * l + (j & 1)] = v;
        else vp[o + 2 * p * S + l] = v;
    }
    for (int p = 0; 2 * p < w; ++p) {
        const int j0 = 2 * p, j1 = 2 * p + 1;
        const short d0 = j0 < L ? (short)(ci[a + j0] - row) : (short)SHRT_MIN;
        const short d1 = j1 < L ? (short)(ci[a + j1] - row) : (short)SHRT_MIN;
        c32p[wo + (int64_t)p * S + l] = (int)(unsigned short)d0 | ((int)d1 << 16);
    }
}

int main(int argc, char **argv) {
    std::vector<int64_t> ms;
    for (int i = 1; i < argc; ++i) ms.push_back(atoll(argv[i]));
    if (ms.empty()) ms = {3163, 4096, 16384};
    for (int64_t m : ms) {
        const int64_t n = m * m, nnz = 5 * n - 4 * m;
        int *rp, *ci;
        double *va, *x, *y, *yr;
        CK(hipMalloc(&rp, (n + 1) * 4));
        CK(hipMalloc(&ci, nnz * 4));
        CK(hipMalloc(&va, nnz * 8));
        CK(hipMalloc(&x, n * 8));
        CK(hipMalloc(&y, n * 8));
        CK(hipMalloc(&yr, n * 8));
        const double h = 2.0 / (double)(m + 1);
        fd2d<<<(unsigned)((n + 256) / 256), 256>>>(m, rp, ci, va, -4.0 / h / h, 1.0 / h / h);
        fillx<<<(unsigned)((n + 255) / 256), 256>>>(n, x);
        CK(hipDeviceSynchronize());
        std::vector<int> hrp(n + 1);
        CK(hipMemcpy(hrp.data(), rp, (n + 1) * 4, hipMemcpyDeviceToHost));
        const int64_t nt = (n + S - 1) / S;
        std::vector<int64_t> hoff(nt + 1), hwoff(nt + 1);
        hoff[0] = hwoff[0] = 0;
        for (int64_t t = 0; t < nt; ++t) {
            int w = 0;
            for (int64_t r = t * S; r < std::min(n, t * S + S); ++r) w = std::max(w, hrp[r + 1] - hrp[r]);
            hoff[t + 1] = hoff[t] + (int64_t)w * S;
            hwoff[t + 1] = hwoff[t] + (int64_t)((w + 1) / 2) * S;
        }
        const int64_t slots = hoff[nt], words = hwoff[nt];
        int64_t *off, *woff;
        int *c32w, *c32p;
        short *c16;
        double *vw, *vp;
        CK(hipMalloc(&off, (nt + 1) * 8));
        CK(hipMalloc(&woff, (nt + 1) * 8));
        CK(hipMalloc(&c32w, slots * 4));
        CK(hipMalloc(&c32p, words * 4));
        CK(hipMalloc(&c16, slots * 2));
        CK(hipMalloc(&vw, slots * 8));
        CK(hipMalloc(&vp, slots * 8));
        CK(hipMemcpy(off, hoff.data(), (nt + 1) * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(woff, hwoff.data(), (nt + 1) * 8, hipMemcpyHostToDevice));
        fill<<<(unsigned)nt, S>>>(n, rp, ci, va, off, woff, c32w, c16, c32p, vw, vp);
        CK(hipDeviceSynchronize());
        auto launch = [&](int v, double *out) {
            switch (v) {
            case 0: spmv<0><<<(unsigned)nt, BS>>>(n, off, woff, c32w, c16, vw, x, out); break;
            case 1: spmv<1><<<(unsigned)nt, BS>>>(n, off, woff, c32w, c16, vw, x, out); break;
            case 2: spmv<2><<<(unsigned)nt, BS>>>(n, off, woff, c32p, c16, vw, x, out); break;
            case 3: spmv<3><<<(unsigned)nt, BS>>>(n, off, woff, c32p, c16, vp, x, out); break;
            }
        };
        const char *names[] = {"wide", "pk16", "pk2", "pk2v2"};
        const double moved[] = {12.0 * slots, 10.0 * slots, 8.0 * slots + 4.0 * words, 8.0 * slots + 4.0 * words};
        launch(0, yr);
        CK(hipDeviceSynchronize());
        std::vector<double> href(n), hy(n);
        CK(hipMemcpy(href.data(), yr, n * 8, hipMemcpyDeviceToHost));
        for (int v = 1; v < 4; ++v) {
            CK(hipMemset(y, 0xff, n * 8));
            launch(v, y);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hy.data(), y, n * 8, hipMemcpyDeviceToHost));
            if (std::memcmp(hy.data(), href.data(), n * 8) != 0) std::printf("m=%lld %s NOT bitwise\n", (long long)m, names[v]);
        }
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int R = 5, L = m >= 8192 ? 10 : 40;
        std::vector<std::vector<float>> tm(4);
        for (int r = 0; r < R; ++r)
            for (int v = 0; v < 4; ++v) {
                launch(v, y);
                CK(hipEventRecord(e0));
                for (int l = 0; l < L; ++l) launch(v, y);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float f;
                CK(hipEventElapsedTime(&f, e0, e1));
                tm[v].push_back(f / L);
            }
        const double alg = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
        for (int v = 0; v < 4; ++v) {
            std::sort(tm[v].begin(), tm[v].end());
            const double b = tm[v][0] * 1e-3, md = tm[v][R / 2] * 1e-3;
            const double mv = moved[v] + 16.0 * n + 8.0 * nt;
            std::printf("m=%-6lld %-6s best %8.1f us med %8.1f us  csr-alg %5.1f%%  moved %6.2f GB = %6.0f GB/s (%5.1f%%)\n",
                        (long long)m, names[v], b * 1e6, md * 1e6, alg / b / 8e12 * 100, mv / 1e9, mv / b / 1e9,
                        mv / b / 8e12 * 100);
        }
        std::fflush(stdout);
        for (void *p : {(void *)rp, (void *)ci, (void *)va, (void *)x, (void *)y, (void *)yr, (void *)off, (void *)woff,
                        (void *)c32w, (void *)c32p, (void *)c16, (void *)vw, (void *)vp})
            CK(hipFree(p));
    }
    return 0;
}
