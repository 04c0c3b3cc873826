// spmv_lab.hip — A/B harness for CSR SpMV schedules on gfx950 (development tool, not shipped).
// Builds FDLaplacian2D(m) on the device, runs every variant, checks each is bit-identical to
// variant A (scipy csr_matvec order), and times them in interleaved rounds in one process.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o spmv_lab tools/spmv_lab.hip
//   ./spmv_lab 3163 4096
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int BS = 256;
constexpr int PAD = 1024;   // padding entries after colidx/vals (vector loads may run past nnz)

__device__ __forceinline__ int64_t lblock() {
    const int64_t g = gridDim.x, b = blockIdx.x;
    if (g % 8 != 0) return b;
    return (b % 8) * (g / 8) + b / 8;
}

// ---------------- A: block tiles of 256 rows, 2048-entry LDS chunks (current libpsk) ---------------
__global__ __launch_bounds__(BS) void spmv_A(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                             const double* __restrict__ va, const double* __restrict__ x,
                                             double* __restrict__ y) {
    constexpr int CH = 2048, KU = CH / BS;
    __shared__ double prod[CH];
    const int tid = threadIdx.x;
    const int64_t nt = (n + 255) / 256, g = gridDim.x, lb = lblock();
    const int64_t t0 = nt * lb / g, t1 = nt * (lb + 1) / g;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n, row = r0 + tid;
        const bool has = row < r1;
        int rs = 0, re = 0;
        if (has) { rs = rp[row]; re = rp[row + 1]; }
        const int e0 = rp[r0], e1 = rp[r1];
        double sum = 0.0;
        for (int c0 = e0; c0 < e1; c0 += CH) {
            const int c1 = e1 - c0 > CH ? c0 + CH : e1;
            const int nk = (c1 - c0 + BS - 1) / BS;
            int cc[KU]; double vv[KU], xv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) { int e = c0 + k * BS + tid; int ee = e < c1 ? e : c0; cc[k] = ci[ee]; vv[k] = va[ee]; }
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) xv[k] = x[cc[k]];
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) { int e = c0 + k * BS + tid; if (e < c1) prod[k * BS + tid] = vv[k] * xv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            __syncthreads();
        }
        if (has) y[row] = sum;
    }
}

// ---------------- A2: A with the next tile's colidx/vals prefetched into registers --------------------
template <int CH, bool NT>
__global__ __launch_bounds__(BS) void spmv_A2(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                              const double* __restrict__ va, const double* __restrict__ x,
                                              double* __restrict__ y) {
    constexpr int KU = CH / BS;
    __shared__ double prod[CH];
    const int tid = threadIdx.x;
    const int64_t nt = (n + 255) / 256, g = gridDim.x, lb = lblock();
    const int64_t t0 = nt * lb / g, t1 = nt * (lb + 1) / g;
    auto ld_i = [](const int* p) { return NT ? __builtin_nontemporal_load(p) : *p; };
    auto ld_d = [](const double* p) { return NT ? __builtin_nontemporal_load(p) : *p; };
    int cc[KU]; double vv[KU];
    int ncc[KU]; double nvv[KU];
    int e0 = 0, e1 = 0;
    auto issue = [&](int64_t t, int& a, int& b, int* c_, double* v_) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n;
        a = rp[r0]; b = rp[r1];
        const int c1 = b - a > CH ? a + CH : b;
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = a + k * BS + tid; int ee = e < c1 ? e : a; c_[k] = ld_i(ci + ee); v_[k] = ld_d(va + ee); }
    };
    if (t0 < t1) issue(t0, e0, e1, cc, vv);
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n, row = r0 + tid;
        const bool has = row < r1;
        int rs = 0, re = 0;
        if (has) { rs = rp[row]; re = rp[row + 1]; }
        double sum = 0.0;
        const int ce0 = e0, ce1 = e1;
        for (int c0 = ce0; c0 < ce1; c0 += CH) {
            const int c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            if (c0 != ce0) {   // rare: tile longer than one chunk
#pragma unroll
                for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; int ee = e < c1 ? e : c0; cc[k] = ld_i(ci + ee); vv[k] = ld_d(va + ee); }
            }
            double xv[KU], pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) xv[k] = x[cc[k]];
            const bool pf = c1 == ce1 && t + 1 < t1;
            if (pf) issue(t + 1, e0, e1, ncc, nvv);       // next tile's stream issued before the gathers land
#pragma unroll
            for (int k = 0; k < KU; ++k) pv[k] = vv[k] * xv[k];
            if (pf) {
#pragma unroll
                for (int k = 0; k < KU; ++k) { cc[k] = ncc[k]; vv[k] = nvv[k]; }
            }
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; if (e < c1) prod[k * BS + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            __syncthreads();
        }
        if (has) { if (NT) __builtin_nontemporal_store(sum, y + row); else y[row] = sum; }
    }
}

// ---------------- A3: A2 with a selectable tile order --------------------------------------------------
// ORDER 0: contiguous tile range per block; 1: each XCD (blockIdx % 8) owns a contiguous slab of
// tiles and its blocks interleave inside it; 2: global interleave (tile = block + k * grid);
// 3: strips: with S = m/256 tiles per grid line, block g walks tile column c = g % S over a
// contiguous range of tile rows (tile = r*S + c), so the x[i-m] it needs was its own x[i] one
// tile earlier (same CU -> L2), needs grid % S == 0.
template <int CH, int ORDER>
__global__ __launch_bounds__(BS) void spmv_A3(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                              const double* __restrict__ va, const double* __restrict__ x,
                                              double* __restrict__ y) {
    constexpr int KU = CH / BS;
    __shared__ double prod[CH];
    const int tid = threadIdx.x;
    const int64_t nt = (n + 255) / 256, g = gridDim.x;
    int64_t tbeg, tend, tstep;
    if (ORDER == 0) { const int64_t lb = lblock(); tbeg = nt * lb / g; tend = nt * (lb + 1) / g; tstep = 1; }
    else if (ORDER == 1) {
        const int64_t xcd = blockIdx.x % 8, lb = blockIdx.x / 8, g8 = g / 8;
        const int64_t s0 = nt * xcd / 8, s1 = nt * (xcd + 1) / 8;
        tbeg = s0 + lb; tend = s1; tstep = g8;
    } else if (ORDER == 2) { tbeg = blockIdx.x; tend = nt; tstep = g; }
    else {
        const int64_t m = (int64_t)sqrt((double)n), S = m / 256 > 0 ? m / 256 : 1;
        const int64_t c = blockIdx.x % S, q = blockIdx.x / S, Q = g / S, R = (nt + S - 1) / S;
        tbeg = (R * q / Q) * S + c; tend = (R * (q + 1) / Q) * S + c; if (tend > nt) tend = nt; tstep = S;
    }
    int cc[KU], ncc[KU]; double vv[KU], nvv[KU];
    int e0 = 0, e1 = 0;
    auto issue = [&](int64_t t, int& a, int& b, int* c_, double* v_) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n;
        a = rp[r0]; b = rp[r1];
        const int c1 = b - a > CH ? a + CH : b;
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = a + k * BS + tid; int ee = e < c1 ? e : a;
            c_[k] = __builtin_nontemporal_load(ci + ee); v_[k] = __builtin_nontemporal_load(va + ee); }
    };
    if (tbeg < tend) issue(tbeg, e0, e1, cc, vv);
    for (int64_t t = tbeg; t < tend; t += tstep) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n, row = r0 + tid;
        const bool has = row < r1;
        int rs = 0, re = 0;
        if (has) { rs = rp[row]; re = rp[row + 1]; }
        double sum = 0.0;
        const int ce0 = e0, ce1 = e1;
        for (int c0 = ce0; c0 < ce1; c0 += CH) {
            const int c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            if (c0 != ce0) {
#pragma unroll
                for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; int ee = e < c1 ? e : c0;
                    cc[k] = __builtin_nontemporal_load(ci + ee); vv[k] = __builtin_nontemporal_load(va + ee); }
            }
            double xv[KU], pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) xv[k] = x[cc[k]];
            const bool pf = c1 == ce1 && t + tstep < tend;
            if (pf) issue(t + tstep, e0, e1, ncc, nvv);
#pragma unroll
            for (int k = 0; k < KU; ++k) pv[k] = vv[k] * xv[k];
            if (pf) {
#pragma unroll
                for (int k = 0; k < KU; ++k) { cc[k] = ncc[k]; vv[k] = nvv[k]; }
            }
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; if (e < c1) prod[k * BS + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            __syncthreads();
        }
        if (has) __builtin_nontemporal_store(sum, y + row);
    }
}

// ---------------- A5: A3 interleave with an UNCONDITIONAL next-tile prefetch and unconditional LDS
// stores (static vmcnt: the gathers are waited for while the prefetch stays in flight) = libpsk r1
template <int CH, int TR = 256>
__global__ __launch_bounds__(BS) void spmv_A5(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                              const double* __restrict__ va, const double* __restrict__ x,
                                              double* __restrict__ y) {
    constexpr int KU = CH / BS;
    __shared__ double prod[CH + BS];
    const int tid = threadIdx.x;
    const int64_t nt = (n + TR - 1) / TR, g = gridDim.x;
    const int last = rp[n] - 1;
    int cc[KU], ncc[KU]; double vv[KU], nvv[KU];
    int e0 = 0, e1 = 0;
    auto issue = [&](int64_t t, int& a, int& b, int* c_, double* v_) {
        const int64_t r0 = t * TR, r1 = r0 + TR < n ? r0 + TR : n;
        a = rp[r0]; b = rp[r1];
        const int c1 = b - a > CH ? a + CH : b;
        const int base = a < last ? a : last;
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = a + k * BS + tid; int ee = e < c1 ? e : base;
            c_[k] = __builtin_nontemporal_load(ci + ee); v_[k] = __builtin_nontemporal_load(va + ee); }
    };
    if ((int64_t)blockIdx.x < nt) issue(blockIdx.x, e0, e1, cc, vv);
    for (int64_t t = blockIdx.x; t < nt; t += g) {
        const int64_t r0 = t * TR, r1 = r0 + TR < n ? r0 + TR : n;
        double sum = 0.0, sum2 = 0.0;
        const int64_t row = r0 + tid, row2 = r0 + BS + tid;
        const bool has = tid < TR && row < r1, has2 = TR > BS && row2 < r1;
        const int64_t rowc2 = has2 ? row2 : r0;
        const int rs2 = rp[rowc2], re2 = rp[rowc2 + 1];
        const int64_t rowc = has ? row : r0;
        const int rs = rp[rowc], re = rp[rowc + 1];
        const int ce0 = e0, ce1 = e1;
        {
            const int c0 = ce0, c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            double xv[KU], pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) xv[k] = x[cc[k]];
            const int64_t tn = t + g < nt ? t + g : t;
            issue(tn, e0, e1, ncc, nvv);
#pragma unroll
            for (int k = 0; k < KU; ++k) pv[k] = vv[k] * xv[k];
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; prod[(e < c1 ? k * BS : CH) + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            if (has) for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            if (TR > BS) {
                const int a2 = rs2 > c0 ? rs2 : c0, b2 = re2 < c1 ? re2 : c1;
                if (has2) for (int e = a2; e < b2; ++e) sum2 = sum2 + prod[e - c0];
            }
            __syncthreads();
        }
        for (int c0 = ce0 + CH; c0 < ce1; c0 += CH) {
            const int c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            double pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; int ee = e < c1 ? e : c0;
                pv[k] = __builtin_nontemporal_load(va + ee) * x[__builtin_nontemporal_load(ci + ee)]; }
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; prod[(e < c1 ? k * BS : CH) + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            if (has) for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            if (TR > BS) {
                const int a2 = rs2 > c0 ? rs2 : c0, b2 = re2 < c1 ? re2 : c1;
                if (has2) for (int e = a2; e < b2; ++e) sum2 = sum2 + prod[e - c0];
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < KU; ++k) { cc[k] = ncc[k]; vv[k] = nvv[k]; }
        if (has) __builtin_nontemporal_store(sum, y + row);
        if (has2) __builtin_nontemporal_store(sum2, y + row2);
    }
}

// ---------------- O: one-shot — one 256-row tile per workgroup, grid = tiles (hardware dispatch
// order instead of a persistent loop; many resident workgroups hide the latency chain) ------------
template <int CH, int TPW = 1>
__global__ __launch_bounds__(BS) void spmv_O(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                             const double* __restrict__ va, const double* __restrict__ x,
                                             double* __restrict__ y) {
    constexpr int KU = CH / BS, TR = 256;
    __shared__ double prod[CH + BS];
    const int tid = threadIdx.x;
    const int64_t nt = (n + TR - 1) / TR;
    const int last = rp[n] - 1;
    int cc[TPW][KU]; double vv[TPW][KU];
    int e0[TPW], e1[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        int64_t t = (int64_t)blockIdx.x * TPW + u;
        t = t < nt ? t : nt - 1;
        const int64_t r0 = t * TR, r1 = r0 + TR < n ? r0 + TR : n;
        e0[u] = rp[r0]; e1[u] = rp[r1];
        const int c1 = e1[u] - e0[u] > CH ? e0[u] + CH : e1[u];
        const int base = e0[u] < last ? e0[u] : last;
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = e0[u] + k * BS + tid; int ee = e < c1 ? e : base;
            cc[u][k] = __builtin_nontemporal_load(ci + ee); vv[u][k] = __builtin_nontemporal_load(va + ee); }
    }
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int64_t t = (int64_t)blockIdx.x * TPW + u;
        if (t >= nt) break;
        const int64_t r0 = t * TR, r1 = r0 + TR < n ? r0 + TR : n;
        const int64_t row = r0 + tid;
        const bool has = row < r1;
        const int64_t rowc = has ? row : r0;
        const int rs = rp[rowc], re = rp[rowc + 1];
        double sum = 0.0;
        const int ce0 = e0[u], ce1 = e1[u];
        {
            const int c0 = ce0, c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            double pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) pv[k] = vv[u][k] * x[cc[u][k]];
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; prod[(e < c1 ? k * BS : CH) + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            if (has) for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            __syncthreads();
        }
        for (int c0 = ce0 + CH; c0 < ce1; c0 += CH) {
            const int c1 = ce1 - c0 > CH ? c0 + CH : ce1;
            double pv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; int ee = e < c1 ? e : c0;
                pv[k] = __builtin_nontemporal_load(va + ee) * x[__builtin_nontemporal_load(ci + ee)]; }
#pragma unroll
            for (int k = 0; k < KU; ++k) { int e = c0 + k * BS + tid; prod[(e < c1 ? k * BS : CH) + tid] = pv[k]; }
            __syncthreads();
            const int a = rs > c0 ? rs : c0, b = re < c1 ? re : c1;
            if (has) for (int e = a; e < b; ++e) sum = sum + prod[e - c0];
            __syncthreads();
        }
        if (has) __builtin_nontemporal_store(sum, y + row);
    }
}

// ---------------- A4: 3-stage pipeline: stream(t+2) | gather(t+1) | sum(t), round-robin tiles -----------
template <int CH>
__global__ __launch_bounds__(BS) void spmv_A4(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                              const double* __restrict__ va, const double* __restrict__ x,
                                              double* __restrict__ y) {
    constexpr int KU = CH / BS;
    __shared__ double prod[CH];
    const int tid = threadIdx.x;
    const int64_t nt = (n + 255) / 256, g = gridDim.x;
    // assumes every tile fits one chunk (true for the 5-point matrix: <= 1280 entries / 256 rows)
    int c0_[KU], c1_[KU]; double v0_[KU], v1_[KU];   // stream stage for tiles t+1, t+2
    double xg[KU];                                     // gathered x for tile t+1
    int a1 = 0, b1 = 0, a2 = 0, b2 = 0;
    auto stream = [&](int64_t t, int& a, int& b, int* c_, double* v_) {
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n;
        a = rp[r0]; b = rp[r1];
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = a + k * BS + tid; int ee = e < b ? e : a;
            c_[k] = __builtin_nontemporal_load(ci + ee); v_[k] = __builtin_nontemporal_load(va + ee); }
    };
    int64_t t = blockIdx.x;
    if (t < nt) stream(t, a1, b1, c0_, v0_);
    if (t < nt) {
#pragma unroll
        for (int k = 0; k < KU; ++k) xg[k] = x[c0_[k]];
    }
    if (t + g < nt) stream(t + g, a2, b2, c1_, v1_);
    for (; t < nt; t += g) {
        // products of tile t (its gathers were issued one stage earlier)
        double pv[KU];
#pragma unroll
        for (int k = 0; k < KU; ++k) pv[k] = v0_[k] * xg[k];
        const int ca = a1, cb = b1;
        // advance the pipeline: tile t+g's stream landed -> issue its gathers; stream tile t+2g
        if (t + g < nt) {
#pragma unroll
            for (int k = 0; k < KU; ++k) { xg[k] = x[c1_[k]]; c0_[k] = c1_[k]; v0_[k] = v1_[k]; }
            a1 = a2; b1 = b2;
            if (t + 2 * g < nt) stream(t + 2 * g, a2, b2, c1_, v1_);
        }
        const int64_t r0 = t * 256, r1 = r0 + 256 < n ? r0 + 256 : n, row = r0 + tid;
        const bool has = row < r1;
        int rs = 0, re = 0;
        if (has) { rs = rp[row]; re = rp[row + 1]; }
#pragma unroll
        for (int k = 0; k < KU; ++k) { int e = ca + k * BS + tid; if (e < cb) prod[k * BS + tid] = pv[k]; }
        __syncthreads();
        double sum = 0.0;
        for (int e = rs; e < re; ++e) sum = sum + prod[e - ca];
        __syncthreads();
        if (has) __builtin_nontemporal_store(sum, y + row);
    }
}

// ---------------- PCG update-like kernels (K2: 5 reads + 2 writes; K3: 3 reads + 1 write) -------------
typedef double ev2 __attribute__((ext_vector_type(2)));
template <bool NT> __device__ __forceinline__ ev2 L2(const double* p) {
    return NT ? __builtin_nontemporal_load(reinterpret_cast<const ev2*>(p)) : *reinterpret_cast<const ev2*>(p);
}
template <bool NT> __device__ __forceinline__ void S2(double* p, ev2 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<ev2*>(p)); else *reinterpret_cast<ev2*>(p) = v;
}
// MODE 0: current policy (x,Ap nt loads, x nt store); 1: all nt; 2: none nt
template <int ORDER, int MODE, int U>
__global__ __launch_bounds__(BS) void k2like(int64_t n, double* __restrict__ x, double* __restrict__ r,
                                             const double* __restrict__ p, const double* __restrict__ Ap,
                                             const double* __restrict__ d, double alpha, double* __restrict__ out) {
    constexpr bool NX = MODE != 2, NP = MODE == 1, NR = MODE == 1, NA = MODE != 2, ND = MODE == 1;
    constexpr bool SX = MODE != 2, SR = MODE == 1;
    double rr = 0, ur = 0;
    auto body = [&](int64_t i) {
        ev2 xv = L2<NX>(x + i), pv = L2<NP>(p + i), rv = L2<NR>(r + i), av = L2<NA>(Ap + i), dv = L2<ND>(d + i);
        ev2 xn = xv + alpha * pv, rn = rv - alpha * av;
        S2<SX>(x + i, xn); S2<SR>(r + i, rn);
        rr += rn.x * rn.x + rn.y * rn.y; ur += dv.x * rn.x * rn.x + dv.y * rn.y * rn.y;
    };
    if (ORDER == 0) {
        const int64_t nt = n / 512, t0 = nt * blockIdx.x / gridDim.x, t1 = nt * (blockIdx.x + 1) / gridDim.x;
        const int64_t i1 = t1 * 512;
        int64_t i = t0 * 512 + 2 * threadIdx.x;
#pragma unroll U
        for (; i < i1; i += 512) body(i);
    } else {
        const int64_t np = n / 2, gs = (int64_t)gridDim.x * BS;
#pragma unroll U
        for (int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x; q < np; q += gs) body(2 * q);
    }
    if (rr == 1.2345 && ur == 1.2345) out[0] = rr;
}

template <int ORDER, int MODE, int U>
__global__ __launch_bounds__(BS) void k3like(int64_t n, const double* __restrict__ r, double* __restrict__ p,
                                             const double* __restrict__ d, double beta) {
    constexpr bool NR = MODE != 2, NP = MODE == 1, ND = MODE != 2, SP = MODE == 1;
    auto body = [&](int64_t i) {
        ev2 rv = L2<NR>(r + i), pv = L2<NP>(p + i), dv = L2<ND>(d + i);
        S2<SP>(p + i, dv * rv + beta * pv);
    };
    if (ORDER == 0) {
        const int64_t nt = n / 512, t0 = nt * blockIdx.x / gridDim.x, t1 = nt * (blockIdx.x + 1) / gridDim.x;
        const int64_t i1 = t1 * 512;
        int64_t i = t0 * 512 + 2 * threadIdx.x;
#pragma unroll U
        for (; i < i1; i += 512) body(i);
    } else {
        const int64_t np = n / 2, gs = (int64_t)gridDim.x * BS;
#pragma unroll U
        for (int64_t q = (int64_t)blockIdx.x * BS + threadIdx.x; q < np; q += gs) body(2 * q);
    }
}

// elementwise-style stream with the same three orders (8 B x 2 per lane, 512-element tiles)
template <int ORDER>
__global__ __launch_bounds__(BS) void readOrd(int64_t n, const double* __restrict__ a, double* __restrict__ out) {
    const int64_t nt = n / 512, g = gridDim.x;
    int64_t tbeg, tend, tstep;
    if (ORDER == 0) { tbeg = nt * blockIdx.x / g; tend = nt * (blockIdx.x + 1) / g; tstep = 1; }
    else if (ORDER == 1) {
        const int64_t xcd = blockIdx.x % 8, lb = blockIdx.x / 8, g8 = g / 8;
        tbeg = nt * xcd / 8 + lb; tend = nt * (xcd + 1) / 8; tstep = g8;
    } else { tbeg = blockIdx.x; tend = nt; tstep = g; }
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2* s = reinterpret_cast<const d2*>(a);
    double acc = 0;
    int64_t t = tbeg;
    for (; t + tstep < tend; t += 2 * tstep) {
        d2 v0 = __builtin_nontemporal_load(s + t * 256 + threadIdx.x);
        d2 v1 = __builtin_nontemporal_load(s + (t + tstep) * 256 + threadIdx.x);
        acc += v0.x + v1.y;
    }
    for (; t < tend; t += tstep) acc += __builtin_nontemporal_load(s + t * 256 + threadIdx.x).x;
    if (acc == 12345.678) out[0] = acc;
}

__global__ __launch_bounds__(BS) void copy4(int64_t n, const double* __restrict__ a, double* __restrict__ b) {
    const int64_t nt = n / 2, stride = (int64_t)gridDim.x * BS;
    const double2* s = reinterpret_cast<const double2*>(a);
    double2* d = reinterpret_cast<double2*>(b);
    int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    for (; i + 3 * stride < nt; i += 4 * stride) {
        double2 v0 = s[i], v1 = s[i + stride], v2 = s[i + 2 * stride], v3 = s[i + 3 * stride];
        d[i] = v0; d[i + stride] = v1; d[i + 2 * stride] = v2; d[i + 3 * stride] = v3;
    }
    for (; i < nt; i += stride) d[i] = s[i];
}

typedef double dv2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(BS) void readU(int64_t n, const double* __restrict__ a, double* __restrict__ out) {
    const int64_t nt = n / 2, stride = (int64_t)gridDim.x * BS;
    const dv2* s = reinterpret_cast<const dv2*>(a);
    double acc = 0.0;
    int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    for (; i + (U - 1) * stride < nt; i += U * stride) {
        dv2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    if (acc == 12345.678) out[0] = acc;
}

// contiguous-range reader: each block streams its own contiguous slab (like the SpMV tiles)
template <int U, bool NT>
__global__ __launch_bounds__(BS) void readSlab(int64_t n, const double* __restrict__ a, double* __restrict__ out) {
    const int64_t nt = n / 2, per = (nt + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = blockIdx.x * per, b1 = b0 + per < nt ? b0 + per : nt;
    const dv2* s = reinterpret_cast<const dv2*>(a);
    double acc = 0.0;
    int64_t i = b0 + threadIdx.x;
    for (; i + (U - 1) * BS < b1; i += U * BS) {
        dv2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * BS) : s[i + u * BS];
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
    }
    for (; i < b1; i += BS) acc += s[i].x;
    if (acc == 12345.678) out[0] = acc;
}

__global__ __launch_bounds__(BS) void read4(int64_t n, const double* __restrict__ a, double* __restrict__ out) {
    const int64_t nt = n / 2, stride = (int64_t)gridDim.x * BS;
    const double2* s = reinterpret_cast<const double2*>(a);
    double acc = 0.0;
    int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    for (; i + 3 * stride < nt; i += 4 * stride) {
        double2 v0 = s[i], v1 = s[i + stride], v2 = s[i + 2 * stride], v3 = s[i + 3 * stride];
        acc += v0.x + v1.y + v2.x + v3.y;
    }
    if (acc == 12345.678) out[0] = acc;
}

// ---------------- B: wave-local tiles (RPW rows per wave), no block barriers ------------------------
template <int RPW, int CH>
__global__ __launch_bounds__(BS) void spmv_B(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                             const double* __restrict__ va, const double* __restrict__ x,
                                             double* __restrict__ y) {
    constexpr int KU = CH / 64, RPL = RPW / 64;
    __shared__ double slab[4][CH];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* prod = slab[w];
    const int64_t nt = (n + RPW - 1) / RPW, gw = (int64_t)gridDim.x * 4, wid = lblock() * 4 + w;
    const int64_t t0 = nt * wid / gw, t1 = nt * (wid + 1) / gw;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t r0 = t * RPW, r1 = r0 + RPW < n ? r0 + RPW : n;
        int rs[RPL], re[RPL];
        double sum[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int64_t row = r0 + q * 64 + lane;
            rs[q] = 0; re[q] = 0; sum[q] = 0.0;
            if (row < r1) { rs[q] = rp[row]; re[q] = rp[row + 1]; }
        }
        const int e0 = __builtin_amdgcn_readfirstlane(rp[r0]);
        const int e1 = __builtin_amdgcn_readfirstlane(rp[r1]);
        for (int c0 = e0; c0 < e1; c0 += CH) {
            const int c1 = e1 - c0 > CH ? c0 + CH : e1;
            const int nk = (c1 - c0 + 63) / 64;
            int cc[KU]; double vv[KU], xv[KU];
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) { int e = c0 + k * 64 + lane; int ee = e < c1 ? e : c0; cc[k] = ci[ee]; vv[k] = va[ee]; }
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) xv[k] = x[cc[k]];
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) { int e = c0 + k * 64 + lane; if (e < c1) prod[k * 64 + lane] = vv[k] * xv[k]; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int a = rs[q] > c0 ? rs[q] : c0, b = re[q] < c1 ? re[q] : c1;
                for (int e = a; e < b; ++e) sum[q] = sum[q] + prod[e - c0];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int64_t row = r0 + q * 64 + lane;
            if (row < r1) y[row] = sum[q];
        }
    }
}

// ---------------- C: wave-local tiles + 16-byte loads (4 entries per lane per step) -----------------
template <int RPW, int CH>
__global__ __launch_bounds__(BS) void spmv_C(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                             const double* __restrict__ va, const double* __restrict__ x,
                                             double* __restrict__ y) {
    constexpr int KU = CH / 256, RPL = RPW / 64;   // 4 entries per lane per k
    __shared__ double slab[4][CH + 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* prod = slab[w];
    const int64_t nt = (n + RPW - 1) / RPW, gw = (int64_t)gridDim.x * 4, wid = lblock() * 4 + w;
    const int64_t t0 = nt * wid / gw, t1 = nt * (wid + 1) / gw;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t r0 = t * RPW, r1 = r0 + RPW < n ? r0 + RPW : n;
        int rs[RPL], re[RPL];
        double sum[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int64_t row = r0 + q * 64 + lane;
            rs[q] = 0; re[q] = 0; sum[q] = 0.0;
            if (row < r1) { rs[q] = rp[row]; re[q] = rp[row + 1]; }
        }
        const int e0 = __builtin_amdgcn_readfirstlane(rp[r0]);
        const int e1 = __builtin_amdgcn_readfirstlane(rp[r1]);
        for (int c0 = e0, c1 = 0; c0 < e1; c0 = c1) {
            const int a0 = c0 & ~3;                       // 16-B aligned start (entries [a0,c0) ignored)
            c1 = e1 - a0 > CH ? a0 + CH : e1;
            const int nk = (c1 - a0 + 255) / 256;
            int4 cc[KU]; double2 v0[KU], v1[KU]; double xv[KU][4];
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) {
                const int e = a0 + 4 * (k * 64 + lane);
                cc[k] = *reinterpret_cast<const int4*>(ci + e);
                v0[k] = *reinterpret_cast<const double2*>(va + e);
                v1[k] = *reinterpret_cast<const double2*>(va + e + 2);
            }
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) {
                xv[k][0] = x[cc[k].x]; xv[k][1] = x[cc[k].y]; xv[k][2] = x[cc[k].z]; xv[k][3] = x[cc[k].w];
            }
#pragma unroll
            for (int k = 0; k < KU; ++k) if (k < nk) {
                const int e = a0 + 4 * (k * 64 + lane);
                const double p0 = v0[k].x * xv[k][0], p1 = v0[k].y * xv[k][1];
                const double p2 = v1[k].x * xv[k][2], p3 = v1[k].y * xv[k][3];
                // slab index = e - a0 (+ alignment slack); entries outside [c0,c1) are never read
                double* d = prod + (e - a0);
                if (e < c1 + 0) { d[0] = p0; d[1] = p1; d[2] = p2; d[3] = p3; }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < RPL; ++q) {
                const int a = rs[q] > c0 ? rs[q] : c0, b = re[q] < c1 ? re[q] : c1;
                for (int e = a; e < b; ++e) sum[q] = sum[q] + prod[e - a0];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int64_t row = r0 + q * 64 + lane;
            if (row < r1) y[row] = sum[q];
        }
    }
}

// ---------------- E: thread per row, direct loads, up to 8 entries in registers ---------------------
__global__ __launch_bounds__(BS) void spmv_E(int64_t n, const int* __restrict__ rp, const int* __restrict__ ci,
                                             const double* __restrict__ va, const double* __restrict__ x,
                                             double* __restrict__ y) {
    const int64_t nt = (n + BS - 1) / BS, g = gridDim.x, lb = lblock();
    const int64_t t0 = nt * lb / g, t1 = nt * (lb + 1) / g;
    for (int64_t t = t0; t < t1; ++t) {
        const int64_t row = t * BS + threadIdx.x;
        if (row >= n) continue;
        const int rs = rp[row], re = rp[row + 1];
        double sum = 0.0;
        for (int c = rs; c < re; c += 8) {
            int cc[8]; double vv[8], xv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) { int e = c + j < re ? c + j : rs; cc[j] = ci[e]; vv[j] = va[e]; }
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = x[cc[j]];
#pragma unroll
            for (int j = 0; j < 8; ++j) if (c + j < re) { const double pr = vv[j] * xv[j]; sum = sum + pr; }
        }
        y[row] = sum;
    }
}

// ---------------- bandwidth references ------------------------------------------------------------------
__global__ __launch_bounds__(BS) void copy2(int64_t n, const double* __restrict__ a, double* __restrict__ b) {
    const int64_t nt = n / 2;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nt; i += (int64_t)gridDim.x * BS)
        reinterpret_cast<double2*>(b)[i] = reinterpret_cast<const double2*>(a)[i];
}

__global__ void fd2d(int64_t m, int* rp, int* ci, double* va, double dv, double ov) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n = m * m;
    if (k > n) return;
    int64_t mk = k < m ? k : m, top = k - m * (m - 1); if (top < 0) top = 0;
    const int64_t off = 5 * k - mk - top - (k + m - 1) / m - k / m;
    rp[k] = (int)off;
    if (k == n) return;
    const int64_t ix = k % m, iy = k / m;
    int64_t p = off;
    ci[p] = (int)k; va[p++] = dv;
    if (iy > 0) { ci[p] = (int)(k - m); va[p++] = ov; }
    if (iy < m - 1) { ci[p] = (int)(k + m); va[p++] = ov; }
    if (ix > 0) { ci[p] = (int)(k - 1); va[p++] = ov; }
    if (ix < m - 1) { ci[p] = (int)(k + 1); va[p++] = ov; }
}

__global__ void fillx(int64_t n, double* x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull; h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
        x[i] = (double)(h >> 11) * (1.0 / 9007199254740992.0); }
}

typedef void (*Kern)(int64_t, const int*, const int*, const double*, const double*, double*);
typedef void (*Kern2)(int64_t, const double*, double*);

int main(int argc, char** argv) {
    std::vector<int64_t> ms;
    for (int i = 1; i < argc; ++i) ms.push_back(atoll(argv[i]));
    if (ms.empty()) ms = {3163, 4096};
    struct V { const char* name; Kern k; int grid; };
    for (int64_t m : ms) {
        const int64_t n = m * m, nnz = 5 * n - 4 * m;
        int *rp, *ci; double *va, *x, *y, *yr;
        CK(hipMalloc(&rp, (n + 1) * 4)); CK(hipMalloc(&ci, (nnz + PAD) * 4)); CK(hipMalloc(&va, (nnz + PAD) * 8));
        CK(hipMalloc(&x, n * 8)); CK(hipMalloc(&y, n * 8)); CK(hipMalloc(&yr, n * 8));
        CK(hipMemset(ci + nnz, 0, PAD * 4)); CK(hipMemset(va + nnz, 0, PAD * 8));
        const double h = 2.0 / (double)(m + 1);
        fd2d<<<(n + 256) / 256, 256>>>(m, rp, ci, va, -4.0 / h / h, 1.0 / h / h);
        fillx<<<(n + 255) / 256, 256>>>(n, x);
        CK(hipDeviceSynchronize());
        const double bytes = 12.0 * nnz + 4.0 * (n + 1) + 16.0 * n;
        std::vector<V> vs = {
            {"A blk256/ch2048", spmv_A, 2048},
            {"A3 interleave g1024", spmv_A3<1280, 2>, 1024},
            {"A5 g768", spmv_A5<1280>, 768},
            {"O oneshot", spmv_O<1280, 1>, (int)((n + 255) / 256)},
            {"O oneshot tpw2", spmv_O<1280, 2>, (int)((n + 511) / 512)},
            {"O oneshot tpw4", spmv_O<1280, 4>, (int)((n + 1023) / 1024)},
            {"A5 g1536", spmv_A5<1280>, 1536},
        };
        // reference result
        spmv_A<<<2048, BS>>>(n, rp, ci, va, x, yr);
        CK(hipDeviceSynchronize());
        std::vector<double> hr(n), hy(n);
        CK(hipMemcpy(hr.data(), yr, n * 8, hipMemcpyDeviceToHost));
        for (auto& v : vs) {
            CK(hipMemset(y, 0xff, n * 8));
            v.k<<<v.grid, BS>>>(n, rp, ci, va, x, y);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hy.data(), y, n * 8, hipMemcpyDeviceToHost));
            const bool same = memcmp(hr.data(), hy.data(), n * 8) == 0;
            printf("m=%ld %-24s grid %d bitwise=%s\n", (long)m, v.name, v.grid, same ? "yes" : "NO");
        }
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        std::vector<std::vector<float>> t(vs.size());
        const int R = 7, L = 20;
        for (int r = 0; r < R; ++r) {
            for (size_t i = 0; i < vs.size(); ++i) {
                CK(hipEventRecord(e0));
                for (int l = 0; l < L; ++l) vs[i].k<<<vs[i].grid, BS>>>(n, rp, ci, va, x, y);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t[i].push_back(ms / L);
            }
        }
        for (size_t i = 0; i < vs.size(); ++i) {
            std::sort(t[i].begin(), t[i].end());
            printf("m=%ld %-24s min %.1f us med %.1f us  -> %.0f GB/s (%.1f%% of 8 TB/s)\n", (long)m, vs[i].name,
                   t[i][0] * 1e3, t[i][R / 2] * 1e3, bytes / (t[i][0] * 1e-3) / 1e9, 100.0 * bytes / (t[i][0] * 1e-3) / 8e12);
        }
        // ---- PCG update-like kernels over 5 vectors of n doubles (K2: 5R+2W, K3: 3R+1W) ----
        if (getenv("LAB_ELEMENTWISE")) {
            double* v5; CK(hipMalloc(&v5, 5 * n * 8)); CK(hipMemset(v5, 0, 5 * n * 8));
            double *vx = v5, *vr = v5 + n, *vp = v5 + 2 * n, *va2 = v5 + 3 * n, *vd = v5 + 4 * n;
            typedef void (*K2)(int64_t, double*, double*, const double*, const double*, const double*, double, double*);
            typedef void (*K3)(int64_t, const double*, double*, const double*, double);
            struct E2 { const char* name; K2 k; int grid; };
            struct E3 { const char* name; K3 k; int grid; };
            std::vector<E2> e2 = {
                {"K2 contig cur u2 g1024", k2like<0, 0, 2>, 1024}, {"K2 contig cur u2 g2048", k2like<0, 0, 2>, 2048},
                {"K2 contig allnt u2 g1024", k2like<0, 1, 2>, 1024}, {"K2 contig nont u2 g1024", k2like<0, 2, 2>, 1024},
                {"K2 contig cur u1 g1024", k2like<0, 0, 1>, 1024}, {"K2 contig cur u4 g1024", k2like<0, 0, 4>, 1024},
                {"K2 inter cur u2 g1024", k2like<1, 0, 2>, 1024}, {"K2 inter allnt u2 g1024", k2like<1, 1, 2>, 1024},
                {"K2 contig cur u2 g512", k2like<0, 0, 2>, 512},
            };
            std::vector<E3> e3 = {
                {"K3 contig cur u2 g1024", k3like<0, 0, 2>, 1024}, {"K3 contig cur u2 g2048", k3like<0, 0, 2>, 2048},
                {"K3 contig allnt u2 g1024", k3like<0, 1, 2>, 1024}, {"K3 contig nont u2 g1024", k3like<0, 2, 2>, 1024},
                {"K3 contig cur u4 g1024", k3like<0, 0, 4>, 1024}, {"K3 inter cur u2 g1024", k3like<1, 0, 2>, 1024},
            };
            std::vector<float> b2(e2.size(), 1e9f), b3(e3.size(), 1e9f);
            for (int r = 0; r < R; ++r) {
                for (size_t i = 0; i < e2.size(); ++i) {
                    CK(hipEventRecord(e0));
                    for (int l = 0; l < L; ++l) e2[i].k<<<e2[i].grid, BS>>>(n, vx, vr, vp, va2, vd, 1e-3, y);
                    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); b2[i] = std::min(b2[i], ms / L);
                }
                for (size_t i = 0; i < e3.size(); ++i) {
                    CK(hipEventRecord(e0));
                    for (int l = 0; l < L; ++l) e3[i].k<<<e3[i].grid, BS>>>(n, vr, vp, vd, 0.5);
                    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); b3[i] = std::min(b3[i], ms / L);
                }
            }
            for (size_t i = 0; i < e2.size(); ++i)
                printf("m=%ld %-26s %.1f us -> %.0f GB/s\n", (long)m, e2[i].name, b2[i] * 1e3, 56.0 * n / (b2[i] * 1e-3) / 1e9);
            for (size_t i = 0; i < e3.size(); ++i)
                printf("m=%ld %-26s %.1f us -> %.0f GB/s\n", (long)m, e3[i].name, b3[i] * 1e3, 32.0 * n / (b3[i] * 1e-3) / 1e9);
            CK(hipFree(v5));
        }
        CK(hipFree(rp)); CK(hipFree(ci)); CK(hipFree(va)); CK(hipFree(x)); CK(hipFree(y)); CK(hipFree(yr));
    }
    return 0;
}
