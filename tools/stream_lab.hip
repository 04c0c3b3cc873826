// stream_lab.hip — A/B harness for the PCG elementwise kernels' access schedule on gfx950
// (development tool, not shipped). Streams NR f64 arrays of n elements and writes NW of them back
// in place (K2: r, Ap, DInv -> r; K3: r, p, x, DInv -> p, x), under different schedules, grids,
// loads-in-flight and cache policies, and reports HBM-level GB/s = (NR + NW) * 8n / time.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -o stream_lab tools/stream_lab.hip
//   ./stream_lab 268435456
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int BS = 256;
constexpr int TILE = 2 * BS;   // 2 doubles (16 B) per lane per tile

typedef double dv2 __attribute__((ext_vector_type(2)));

struct Ptrs {
    double *a[6];
};

template <bool NT>
__device__ __forceinline__ dv2 ld(const double *p) {
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(p));
    return *reinterpret_cast<const dv2 *>(p);
}
template <bool NT>
__device__ __forceinline__ void st(double *p, dv2 v) {
    if (NT) __builtin_nontemporal_store(v, reinterpret_cast<dv2 *>(p));
    else *reinterpret_cast<dv2 *>(p) = v;
}

// SCHED 0: contiguous share of tiles per workgroup; 1: grid-stride over tiles; 2: one-shot (grid =
// tiles / U). U tiles' loads are issued before any of their stores. NTL / NTS: non-temporal
// loads / stores (loads of arrays that are written back stay default when NTL == 1).
template <int NR, int NW, int SCHED, int U, int NTL, int NTS>
__global__ __launch_bounds__(BS) void stream_kernel(int64_t n, Ptrs P, double alpha, double *part) {
    const int64_t ntiles = n / TILE;
    int64_t t0, t1, ts;
    if (SCHED == 0) {
        t0 = ntiles * blockIdx.x / gridDim.x;
        t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
        ts = 1;
    } else if (SCHED == 1) {
        t0 = blockIdx.x;
        t1 = ntiles;
        ts = gridDim.x;
    } else {
        t0 = (int64_t)blockIdx.x * U;
        t1 = t0 + U < ntiles ? t0 + U : ntiles;
        ts = 1;
    }
    double acc = 0.0;
    for (int64_t t = t0; t < t1; t += U * ts) {
        dv2 v[U][NR];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t tt = t + u * ts;
            tt = tt < t1 ? tt : t;
            const int64_t i = tt * TILE + 2 * threadIdx.x;
#pragma unroll
            for (int q = 0; q < NR; ++q) v[u][q] = (NTL && q >= NW) ? ld<true>(P.a[q] + i) : ld<false>(P.a[q] + i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t tt = t + u * ts;
            if (tt >= t1) break;
            const int64_t i = tt * TILE + 2 * threadIdx.x;
            dv2 s = v[u][NR - 1];
#pragma unroll
            for (int q = 0; q < NR - 1; ++q) s = s + alpha * v[u][q];
            acc += s.x + s.y;
#pragma unroll
            for (int w = 0; w < NW; ++w) st<NTS != 0>(P.a[w] + i, v[u][w] + alpha * s);
        }
    }
    if (acc == 12345.678) part[blockIdx.x] = acc;   // keeps read-only variants alive
}

// the production ping-pong pipeline (pcg.hip K2/K3 shape): next tile's loads before this tile's stores
template <int NR, int NW, int NTL, int NTS>
__global__ __launch_bounds__(BS) void pingpong_kernel(int64_t n, Ptrs P, double alpha, double *part) {
    const int64_t ntiles = n / TILE;
    const int64_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    const int64_t i1 = t1 * TILE;
    int64_t i = t0 * TILE + 2 * threadIdx.x;
    double acc = 0.0;
    struct Ops {
        dv2 v[NR];
    } A{}, B{};
    auto load = [&](Ops &o, int64_t j) {
#pragma unroll
        for (int q = 0; q < NR; ++q) o.v[q] = (NTL && q >= NW) ? ld<true>(P.a[q] + j) : ld<false>(P.a[q] + j);
    };
    auto step = [&](const Ops &o, int64_t j) {
        dv2 s = o.v[NR - 1];
#pragma unroll
        for (int q = 0; q < NR - 1; ++q) s = s + alpha * o.v[q];
        acc += s.x + s.y;
#pragma unroll
        for (int w = 0; w < NW; ++w) st<NTS != 0>(P.a[w] + j, o.v[w] + alpha * s);
    };
    auto nxt = [&](int64_t j) { return (j + TILE + 1 < i1) ? j + TILE : j; };
    if (i + 1 < i1) {
        load(A, i);
        while (true) {
            load(B, nxt(i));
            step(A, i);
            i += TILE;
            if (!(i + 1 < i1)) break;
            load(A, nxt(i));
            step(B, i);
            i += TILE;
            if (!(i + 1 < i1)) break;
        }
    }
    if (acc == 12345.678) part[blockIdx.x] = acc;
}

// one-shot with a deterministic two-level reduction: every workgroup writes its partial; the last
// arriver of each group of GRP consecutive workgroups (ticket counter) sums the group's partials in
// index order and resets the ticket. WB threads per workgroup, one 2-double slot per lane.
template <int NR, int NW, int WB, int GRP>
__global__ __launch_bounds__(WB) void oneshot_kernel(int64_t n, Ptrs P, double alpha, double *part,
                                                     double *gpart, unsigned *ticket) {
    const int64_t i = (int64_t)blockIdx.x * (2 * WB) + 2 * threadIdx.x;
    dv2 v[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) v[q] = q >= NW ? ld<true>(P.a[q] + i) : ld<false>(P.a[q] + i);
    dv2 s = v[NR - 1];
#pragma unroll
    for (int q = 0; q < NR - 1; ++q) s = s + alpha * v[q];
#pragma unroll
    for (int w = 0; w < NW; ++w) st<false>(P.a[w] + i, v[w] + alpha * s);
    double acc = s.x * s.x + s.y * s.y;
    // block sum
    __shared__ double sh[WB / 64];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    __shared__ bool last;
    if (threadIdx.x == 0) {
        double b = 0.0;
        for (int w = 0; w < WB / 64; ++w) b += sh[w];
        part[blockIdx.x] = b;
        __threadfence();
        const unsigned g = blockIdx.x / GRP;
        last = atomicAdd(&ticket[g], 1u) == GRP - 1;
    }
    __syncthreads();
    if (last) {
        __threadfence();
        const unsigned g = blockIdx.x / GRP;
        double a = 0.0;
        for (int j = threadIdx.x; j < GRP; j += WB) a += __builtin_nontemporal_load(part + (int64_t)g * GRP + j);
        for (int o = 32; o > 0; o >>= 1) a += __shfl_down(a, o);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            double b = 0.0;
            for (int w = 0; w < WB / 64; ++w) b += sh[w];
            gpart[g] = b;
            ticket[g] = 0;
        }
    }
}

// as oneshot_kernel, but the hand-off avoids the release fence (buffer_wbl2 would write back the
// XCD's L2 full of streamed stores): the partial is ONE agent-scope (sc1) store, the thread waits
// for its acknowledgement (vmcnt(0)), then bumps the ticket with a relaxed agent-scope atomic; the
// last arriver reads the group's partials with agent-scope loads.
template <int NR, int NW, int WB, int GRP>
__global__ __launch_bounds__(WB) void oneshot_sc1_kernel(int64_t n, Ptrs P, double alpha, double *part,
                                                         double *gpart, unsigned *ticket) {
    const int64_t i = (int64_t)blockIdx.x * (2 * WB) + 2 * threadIdx.x;
    dv2 v[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) v[q] = q >= NW ? ld<true>(P.a[q] + i) : ld<false>(P.a[q] + i);
    dv2 s = v[NR - 1];
#pragma unroll
    for (int q = 0; q < NR - 1; ++q) s = s + alpha * v[q];
#pragma unroll
    for (int w = 0; w < NW; ++w) st<false>(P.a[w] + i, v[w] + alpha * s);
    double acc = s.x * s.x + s.y * s.y;
    __shared__ double sh[WB / 64];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    __shared__ int last;
    const unsigned g = blockIdx.x / GRP;
    if (threadIdx.x == 0) {
        double b = 0.0;
        for (int w = 0; w < WB / 64; ++w) b += sh[w];
        __hip_atomic_store(reinterpret_cast<uint64_t *>(part + blockIdx.x), (uint64_t)__double_as_longlong(b),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the partial is acknowledged
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        last = __hip_atomic_fetch_add(&ticket[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == GRP - 1;
    }
    __syncthreads();
    if (last) {
        double a = 0.0;
        for (int j = threadIdx.x; j < GRP; j += WB)
            a += __longlong_as_double((long long)__hip_atomic_load(
                reinterpret_cast<const uint64_t *>(part + (int64_t)g * GRP + j), __ATOMIC_RELAXED,
                __HIP_MEMORY_SCOPE_AGENT));
        for (int o = 32; o > 0; o >>= 1) a += __shfl_down(a, o);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            double b = 0.0;
            for (int w = 0; w < WB / 64; ++w) b += sh[w];
            gpart[g] = b;
            ticket[g] = 0;
        }
    }
}

// one-shot, deterministic two-level reduction WITHOUT tickets: each workgroup publishes its partial
// with one agent-scope 8-byte store into a slot pre-filled with a signalling-NaN sentinel; group
// g's partials are summed (index order) by a workgroup dispatched LAG ids later — workgroups are
// dispatched in id order, so every workgroup it waits for is already resident or retired and never
// waits itself: no deadlock, and with LAG above the resident capacity the wait is almost never
// taken. The reducer re-arms the slots for the next launch.
constexpr uint64_t kSentinel = 0x7FF0000000000001ull;   // sNaN: arithmetic never produces it
template <int NR, int NW, int WB, int GRP, int LAG>
__global__ __launch_bounds__(WB) void oneshot_deleg_kernel(int64_t n, Ptrs P, double alpha, double *part,
                                                           double *gpart, double *dbg) {
    const int64_t i = (int64_t)blockIdx.x * (2 * WB) + 2 * threadIdx.x;
    const int64_t nwg = gridDim.x;
    dv2 v[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) v[q] = q >= NW ? ld<true>(P.a[q] + i) : ld<false>(P.a[q] + i);
    dv2 s = v[NR - 1];
#pragma unroll
    for (int q = 0; q < NR - 1; ++q) s = s + alpha * v[q];
#pragma unroll
    for (int w = 0; w < NW; ++w) st<false>(P.a[w] + i, v[w] + alpha * s);
    double acc = s.x * s.x + s.y * s.y;
    __shared__ double sh[WB / 64];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0;
        for (int w = 0; w < WB / 64; ++w) b += sh[w];
        __hip_atomic_store(reinterpret_cast<uint64_t *>(part + blockIdx.x), (uint64_t)__double_as_longlong(b),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dbg) dbg[blockIdx.x] = b;
    }
    // groups this workgroup reduces: g with min(g*GRP + GRP-1 + LAG, nwg-1) == blockIdx.x
    const int64_t ngroups = (nwg + GRP - 1) / GRP;
    int64_t g0, g1;
    if ((int64_t)blockIdx.x < nwg - 1) {
        const int64_t t = (int64_t)blockIdx.x - (GRP - 1) - LAG;   // g*GRP == t
        if (t < 0 || t % GRP) return;
        g0 = t / GRP;
        g1 = g0 + 1;
    } else {   // the last workgroup takes every group whose reducer id would be past the grid
        const int64_t t = nwg - 1 - (GRP - 1) - LAG;
        g0 = t < 0 ? 0 : (t + GRP - 1) / GRP;
        if (t >= 0 && t % GRP == 0) g0 = t / GRP;
        g1 = ngroups;
    }
    for (int64_t g = g0; g < g1; ++g) {
        const int64_t j0 = g * GRP, j1 = j0 + GRP < nwg ? j0 + GRP : nwg;
        double a = 0.0;
        for (int64_t j = j0 + threadIdx.x; j < j1; j += WB) {
            uint64_t bits;
            int spins = 0;
            while ((bits = __hip_atomic_load(reinterpret_cast<const uint64_t *>(part + j), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) == kSentinel && ++spins < (1 << 20))
                __builtin_amdgcn_s_sleep(2);
            a += __longlong_as_double((long long)bits);
            reinterpret_cast<uint64_t *>(part)[j] = kSentinel;
        }
        for (int o = 32; o > 0; o >>= 1) a += __shfl_down(a, o);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = a;
        __syncthreads();
        if (threadIdx.x == 0) {
            double b = 0.0;
            for (int w = 0; w < WB / 64; ++w) b += sh[w];
            gpart[g] = b;
        }
        __syncthreads();
    }
}

__global__ void fill_sentinel(uint64_t *p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = kSentinel;
}

// grid-stride ping-pong: tile b, b+G, b+2G, ... (next tile's loads before this tile's stores)
template <int NR, int NW>
__global__ __launch_bounds__(BS) void gs_pingpong_kernel(int64_t n, Ptrs P, double alpha, double *part) {
    const int64_t ntiles = n / TILE;
    double acc = 0.0;
    struct Ops {
        dv2 v[NR];
    } A{}, B{};
    auto load = [&](Ops &o, int64_t t) {
        const int64_t j = t * TILE + 2 * threadIdx.x;
#pragma unroll
        for (int q = 0; q < NR; ++q) o.v[q] = q >= NW ? ld<true>(P.a[q] + j) : ld<false>(P.a[q] + j);
    };
    auto step = [&](const Ops &o, int64_t t) {
        const int64_t j = t * TILE + 2 * threadIdx.x;
        dv2 s = o.v[NR - 1];
#pragma unroll
        for (int q = 0; q < NR - 1; ++q) s = s + alpha * o.v[q];
        acc += s.x + s.y;
#pragma unroll
        for (int w = 0; w < NW; ++w) st<false>(P.a[w] + j, o.v[w] + alpha * s);
    };
    const int64_t G = gridDim.x;
    int64_t t = blockIdx.x;
    auto nxt = [&](int64_t u) { return u + G < ntiles ? u + G : u; };
    if (t < ntiles) {
        load(A, t);
        while (true) {
            load(B, nxt(t));
            step(A, t);
            t += G;
            if (t >= ntiles) break;
            load(A, nxt(t));
            step(B, t);
            t += G;
            if (t >= ntiles) break;
        }
    }
    if (acc == 12345.678) part[blockIdx.x] = acc;
}

// 1R1W into a separate array (the guide's copy figure)
__global__ __launch_bounds__(BS) void copy_kernel(int64_t n, Ptrs P, double alpha, double *part) {
    const int64_t i = (int64_t)blockIdx.x * TILE + 2 * threadIdx.x;
    st<false>(P.a[1] + i, alpha * ld<true>(P.a[0] + i));
}

typedef void (*KFn)(int64_t, Ptrs, double, double *);
struct Var {
    std::string name;
    KFn k;
    int grid;
    int nr, nw;
};

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 268435456LL;
    const int R = argc > 2 ? atoi(argv[2]) : 3, L = argc > 3 ? atoi(argv[3]) : 4;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cu = prop.multiProcessorCount;
    Ptrs P;
    for (int q = 0; q < 6; ++q) {
        CK(hipMalloc(&P.a[q], n * 8));
        CK(hipMemset(P.a[q], 0x3f, n * 8));   // 0x3f3f.. = 1.2e-4: finite, nonzero
    }
    double *part;
    CK(hipMalloc(&part, 1 << 26));
    const int64_t ntiles = n / TILE;
    std::vector<Var> vs;
#define ADD(NR, NW, S, U, NTL, NTS, G)                                                                        \
    vs.push_back({std::string("R") + #NR + "W" + #NW + " sched" + #S + " U" + #U + " ntl" + #NTL + " nts" + #NTS + \
                      " g" + std::to_string(G),                                                              \
                  stream_kernel<NR, NW, S, U, NTL, NTS>, (int)(G), NR, NW})
#define ADDPP(NR, NW, NTL, NTS, G)                                                                     \
    vs.push_back({std::string("R") + #NR + "W" + #NW + " pingpong ntl" + #NTL + " nts" + #NTS + " g" + \
                      std::to_string(G),                                                              \
                  pingpong_kernel<NR, NW, NTL, NTS>, (int)(G), NR, NW})
    unsigned *ticket;
    double *gpart;
    CK(hipMalloc(&ticket, 1 << 22));
    CK(hipMemset(ticket, 0, 1 << 22));
    CK(hipMalloc(&gpart, 1 << 22));
    static unsigned *s_ticket;
    static double *s_gpart;
    s_ticket = ticket;
    s_gpart = gpart;
#define ADDOS(NR, NW, WB, GRP)                                                                                 \
    vs.push_back({std::string("R") + #NR + "W" + #NW + " oneshot+ticket wb" + #WB + " grp" + #GRP,            \
                  [](int64_t n_, Ptrs P_, double al, double *pt) {                                           \
                      oneshot_kernel<NR, NW, WB, GRP><<<n_ / (2 * WB), WB>>>(n_, P_, al, pt, s_gpart, s_ticket); \
                  },                                                                                          \
                  -1, NR, NW})
    static double *s_part2;
    CK(hipMalloc(&s_part2, 1 << 26));
    fill_sentinel<<<(1 << 23) / 256, 256>>>(reinterpret_cast<uint64_t *>(s_part2), 1 << 23);
    static double *s_dbg = nullptr;
#define ADDDG(NR, NW, WB, GRP, LAG)                                                                            \
    vs.push_back({std::string("R") + #NR + "W" + #NW + " oneshot+deleg wb" + #WB + " grp" + #GRP + " lag" + #LAG, \
                  [](int64_t n_, Ptrs P_, double al, double *pt) {                                           \
                      oneshot_deleg_kernel<NR, NW, WB, GRP, LAG><<<n_ / (2 * WB), WB>>>(n_, P_, al, s_part2,   \
                                                                                         s_gpart, s_dbg);    \
                  },                                                                                          \
                  -1, NR, NW})
    ADDPP(3, 1, 1, 0, 3 * cu);
    ADD(3, 1, 2, 1, 1, 0, ntiles);
    ADDDG(3, 1, 256, 256, 4096);
    ADDDG(3, 1, 256, 512, 4096);
    ADDDG(3, 1, 256, 256, 0);
    ADDDG(3, 1, 512, 256, 2048);
    ADDPP(4, 2, 1, 0, 3 * cu);
    ADD(4, 2, 2, 1, 1, 0, ntiles);
    ADDDG(4, 2, 256, 256, 4096);
    std::vector<float> best(vs.size(), 1e30f);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&](const Var &v) {
        if (v.grid < 0) v.k(n, P, 1e-3, part);
        else v.k<<<v.grid, BS>>>(n, P, 1e-3, part);
    };
    for (auto &v : vs) launch(v);   // warm
    CK(hipDeviceSynchronize());
    for (int r = 0; r < R; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            CK(hipEventRecord(e0));
            for (int l = 0; l < L; ++l) launch(vs[i]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best[i] = std::min(best[i], ms / L);
        }
    CK(hipGetLastError());
    {   // verify the last delegated variant's group sums against its own partials
        const Var &v = vs.back();
        CK(hipMalloc(&s_dbg, 1 << 26));
        launch(v);
        CK(hipDeviceSynchronize());
        const int64_t nwg = n / (2 * 256), ng = (nwg + 255) / 256;
        std::vector<double> hp(nwg), hg(ng);
        CK(hipMemcpy(hp.data(), s_dbg, nwg * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hg.data(), gpart, ng * 8, hipMemcpyDeviceToHost));
        std::vector<uint64_t> hs(nwg);
        CK(hipMemcpy(hs.data(), s_part2, nwg * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0, unarmed = 0;
        for (int64_t j = 0; j < nwg; ++j) unarmed += hs[j] != kSentinel;
        for (int64_t g = 0; g < ng; ++g) {
            double w[4];
            for (int q = 0; q < 4; ++q) {
                double l[64];
                for (int j = 0; j < 64; ++j) l[j] = hp[g * 256 + q * 64 + j];
                for (int o = 32; o > 0; o >>= 1)
                    for (int j = 0; j < o; ++j) l[j] += l[j + o];
                w[q] = l[0];
            }
            const double ref = ((w[0] + w[1]) + w[2]) + w[3];
            bad += ref != hg[g];
        }
        printf("verify %s: %lld of %lld group sums differ, %lld slots not re-armed\n", v.name.c_str(), (long long)bad,
               (long long)ng, (long long)unarmed);
    }
    printf("n=%lld CUs=%d (best of %d rounds x %d launches)\n", (long long)n, cu, R, L);
    for (size_t i = 0; i < vs.size(); ++i) {
        const double bytes = (double)(vs[i].nr + vs[i].nw) * 8.0 * (double)(ntiles * TILE);
        printf("%-40s %9.1f us -> %6.0f GB/s\n", vs[i].name.c_str(), best[i] * 1e3, bytes / (best[i] * 1e-3) / 1e9);
    }
    return 0;
}
