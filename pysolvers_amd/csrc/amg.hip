// amg.hip — smoothed-aggregation AMG preconditioner apply on the device, and its O(nnz) host setup.
//
// apply(v) restates AMGPreconditioner.apply (AMGPreconditioner.py:46-51) -> AMGVCycleSolver.solve
// with CommonSolverArgs(maxiter=numIters, failOnMaxiter=False) (VCycleSolver.py:52-95):
//     x = copy(v);  for k < numIters: x = runLevel(v, x, L-1); r = v - A x;
//                   if ||r|| < tau ||v||: return x
// runLevel (VCycleManager.py:31-62): level 0 -> direct solve; else pre-smooth, r = f - A x,
// f2 = R r, x2 = runLevel(f2, 0, lev-1), x = x + P x2, post-smooth. A smoothing sweep is
// x <- x + S^-1 (f - A x) for both of the reference's smoothers (ClassicSmoothers.py:5-36:
// Jacobi S^-1 = DInv*, Gauss-Seidel S^-1 = spsolve(triu(A), .)).
//
// Everything stays on one stream with no host synchronisation: the early exit is a device flag.
// After each non-final cycle a one-workgroup kernel compares the fused residual norm (SpMV
// epilogue) with tau ||v|| and, the first time it holds, the current x is copied to the output;
// later cycles still run (their result is discarded), which keeps the launch sequence fixed.
//
// Host setup: psk_sa_aggregate restates BuildAggregates + BuildFilteredMatrix
// (SmoothedAggregation.py:41-183) in O(nnz) instead of the reference's set loops (quadratic in
// phase 2), with identical results (oracle/amg.py pins both against the reference).
#include "psk_internal.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace psk {

// A level whose two consecutive Gauss-Seidel sweeps run as one launch (gs_pair_kernel below)
struct GsPairLevel {
    bool eligible = false, on = false;
    int64_t m = 0, H = 0, nbands = 0;
    int role[5] = {};     // A's stored diagonals in stored order: 0 = d, 1 = -m, 2 = +m, 3 = -1, 4 = +1
    int ord = -1;         // gs_pair_kernel's ORD: role == gp_role(ord, .)
    double v[5] = {};
    DevBuf pub;           // [nbands][3][m] publications of each band's last owned line
};

struct AmgHierarchy {
    int L = 0, num_iters = 0, nu_pre = 0, nu_post = 0;
    double tau = 0.0;
    std::vector<psk_csr *> A, P, R;
    std::vector<psk_prec *> S;
    psk_prec *coarse = nullptr;
    std::vector<DevBuf> x, f, r, t;   // per level (f unused on the finest level: f = v)
    DevBuf scal;                      // [0] = ||v||^2, [1] = flag (as int64), partials after
    std::vector<GsPairLevel> gp;      // per level
};

void amg_free(AmgHierarchy *h) {
    if (!h) return;
    for (auto &b : h->x) b.release();
    for (auto &b : h->f) b.release();
    for (auto &b : h->r) b.release();
    for (auto &b : h->t) b.release();
    for (auto &g : h->gp) g.pub.release();
    h->scal.release();
    delete h;
}

// ---- two Gauss-Seidel sweeps in one launch (round 6) -------------------------------------------
// For a level whose operator is a 5-point stencil on an m x H grid with one value per diagonal (A's diagonal
// layout, its presence masks exactly the grid's; the smoother's triu(A) carries TriFactor::fd5_*), the pair
//     x1 = x0 + U^-1 (f - A x0),   x2 = x1 + U^-1 (f - A x1)           (ClassicSmoothers.py:31-36, twice)
// runs as ONE launch after the first residual r = f - A x0 (launch_spmv). The upper solve goes from row n - 1
// backwards: solve-order line Y = H - 1 - iy, position a = m - 1 - ix; (Y, a) depends on (Y, a - 1) (column
// i + 1) and (Y - 1, a) (column i + m). A band of 63 lines is one workgroup of five waves (one per CU: its LDS),
// lane j on line Y0 + j, stepping a skewed wavefront (step s: position a = s - j):
//  * first sweep (kGpW1st): dx1 from its own previous step (a - 1) and lane j - 1's previous step (line above) by a
//    DPP wave shift — no memory on the dependency chain; x1 = x0 + dx1 into ring1. Lane 63 recomputes the next
//    band's first line, which the second sweep's residual needs (its -m neighbour).
//  * residual (kGpWRes): at step t, r2 = f - A x1 of the lane's row of step t - 1, from x1 of three steps of its own
//    line and of lanes j -/+ 1 (DPP), the row's five entries in A's stored order from 0.0 with rounded products,
//    absent entries skipped (the SpMV's bits); (x1, r2) into ring2.
//  * second sweep (kGpW2nd): dx2 by the same DPP recurrence on r2, x2 = x1 + dx2 into an output slot.
//  * stream (kGpWStream): r, x0 and f into LDS ahead of the sweeps, 16 steps x 64 lines a chunk, and x2 back out
//    once the second sweep has passed a chunk. A line's 16 steps are 16 consecutive rows, so each load and store
//    instruction covers four lines' 128 B with 16 lanes each; read straight by the sweep lanes (one row of 64
//    distinct lines per instruction) the same traffic held a step to ~0.8 us.
//  * poller (wave 0): the band above's publications (dx1, x1, dx2 of its last owned line, sentinel-armed, stored
//    once per 8-step block) into LDS for the lanes 0 of the other waves.
// Every value is the serialized path's: U's off-diagonal sum formed as the factor's current schedule forms it
// (gp_uacc: the grid / band / levels fma chain, or the sync-free / LDS / partitioned lane partials),
// (r - acc) / d by IEEE division (the grid kernel's Markstein quotient is the IEEE one), x + dx. Bands are drawn
// from the U factor's ticket counter (sched_next_block's protocol: a band waits only on the band drawn before
// it), so the launch needs no co-residency; every wait is bounded and
// reports through the smoother's error word (ilu_check_error).
// kGpC: steps per streamed chunk; kGpNB: chunk slots per streamed array; kGpBlk: steps between progress
// announcements and waits (the band below trails by its publication latency plus up to one of these)
constexpr int kGpOwn = 63, kGpRing = 32, kGpRW = 66, kGpExt = 256, kGpBlk = 8, kGpC = 16, kGpNB = 3, kGpSR = 65;
constexpr size_t kGpStage = (size_t)kGpNB * kGpC * kGpSR;   // doubles of one streamed array's slots
constexpr size_t kGpOffRing = 4 * kGpStage * 8, kGpOffExt = kGpOffRing + (size_t)kGpRing * kGpRW * 24,
                 kGpOffCtl = kGpOffExt + 3 * (size_t)kGpExt * 8, kGpLds = kGpOffCtl + 8 * 8;
static_assert(kGpLds <= 160 * 1024, "one workgroup's LDS");
// the waves' roles: the three compute waves on waves 1..3, the light polling (0) and streaming waves (4) (the
// five waves of a workgroup share four SIMDs; wave w runs on SIMD w % 4)
constexpr int kGpW1st = 1, kGpWRes = 2, kGpW2nd = 3, kGpWStream = 4;
constexpr uint32_t kGpOOB = 0xFFFFFFFFu;   // a buffer offset out of range: loads 0, drops the store
constexpr uint64_t kGpSentinel = 0x7FF4DEAD0000BEEFull;   // ilu.hip's sentinel: an sNaN payload
constexpr int64_t kGpMaxSpins = 1ll << 22, kGpDone = INT64_MAX / 4;

struct GsPairArgs {
    int64_t n, m, H, nbands;
    double d, a1, am;   // U = triu(A): the diagonal, the +1 and +m values
    int mfirst;         // U stores its +m entry before its +1 entry
    int role[5];
    double v[5];
    const double *f, *r;   // right-hand side; r = f - A x0
    double *x;             // x0 in, x2 out
    double *pub;
    uint32_t *tick;
    int32_t *err;
};

__device__ __forceinline__ double gp_load(const double *p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void gp_store(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gp_sent(double v) { return (uint64_t)__double_as_longlong(v) == kGpSentinel; }
__device__ __forceinline__ int64_t gp_get(const int64_t *c) {
    return __hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void gp_set(int64_t *c, int64_t v) {
    __hip_atomic_store(c, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wave-uniform: wait until *c >= want; false after the bound (error reported)
__device__ __forceinline__ bool gp_wait(const int64_t *c, int64_t want, int32_t *err, int code, int64_t band) {
    int64_t spins = 0;
    while (!__builtin_amdgcn_readfirstlane((int)(gp_get(c) >= want))) {
        if (++spins > kGpMaxSpins) {
            if ((threadIdx.x & 63) == 0) atomicExch(err, (code << 24) | (int)(band & 0xffffff));
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}
// buffer (bounds-checked) loads and stores: every lane issues every one of them with no branch around it, so
// the compiler's vmcnt waits count exactly the operations in flight (ilu.hip, the grid kernel's note)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gp_rsrc(const double *p, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), (short)0, (int)(uint32_t)(n * 8), 0x00020000);
}
__device__ __forceinline__ double gp_bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
typedef unsigned int gp_u2 __attribute__((ext_vector_type(2)));
template <int CPOL>   // 0x10: sc1 (agent-scope write-through: the publications), 0: plain
__device__ __forceinline__ void gp_bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(gp_u2, v), r, off, 0, CPOL);
}
// lane l <- lane l - 1 (wave_shr:1); lane 0 <- edge
__device__ __forceinline__ double gp_shr1(double v, double edge) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(edge), __double2loint(v), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(edge), __double2hiint(v), 0x138, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// lane l's value, to every lane (two readlanes: no branch, no exec change)
__device__ __forceinline__ double gp_lane(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
// lane l <- lane l + 1 (wave_shl:1); lane 63 <- 0
__device__ __forceinline__ double gp_shl1(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// U's off-diagonal sum of one row as the serialized schedule forms it: LANES = false, the grid / band / levels
// kernels' fma chain over the stored order from 0.0; LANES = true, the sync-free / LDS / partitioned kernels'
// lane partials (entry k's product in lane k, fma(v, x, 0.0)) added by the wave reduction (ilu.hip row_total:
// with two entries the one sum p0 + p1, the other lanes' zeros adding exactly nothing). An absent entry comes
// with coefficient 0: fma(0, v, acc) = acc for a finite v and an acc that is not -0 (acc starts at +0, and an
// fma onto +0 never rounds to -0), exactly the grid kernel's padding entries; the selects stay off the chain.
template <bool LANES, bool MF>
__device__ __forceinline__ double gp_uacc(double c1, double left, double cm, double up) {
    if (LANES) {
        const double q1 = fma(c1, left, 0.0), qm = fma(cm, up, 0.0);
        return MF ? qm + q1 : q1 + qm;
    }
    return MF ? fma(c1, left, fma(cm, up, 0.0)) : fma(cm, up, fma(c1, left, 0.0));
}
// relaxed look at a progress word (the fast path of a block's waits; an acquire fence follows)
__device__ __forceinline__ int gp_ready(const int64_t *c, int64_t want) {
    return (int)(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= want);   // combined with &
}

#ifdef PSK_GP_PROF   // profile build (scripts/build_variant.sh gpprof -DPSK_GP_PROF): per band, s_memrealtime (100 MHz)
// at the start, the first sweep's end and the second's end, then s_memtime cycles spent in each wave's waits:
// ring capacity, the band above's dx1, the first sweep's progress, the band above's dx2; the XCD
__device__ unsigned long long g_gp_prof[4096 * 16];
extern "C" int psk_gp_prof_read(unsigned long long *out, int nbands) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gp_prof), sizeof(unsigned long long) * 16 * (size_t)nbands) ==
                   hipSuccess ? 0 : -1;
}
#define GP_PROF(...) __VA_ARGS__
#else
#define GP_PROF(...)
#endif
// A's stored orders the kernel is built for (role of each stored diagonal): the reference's FD order
// [d, -m, +m, -1, +1] (FDLaplacian2D) and column order [-m, -1, d, +1, +m] (a sorted CSR)
__host__ __device__ constexpr int gp_role(int ord, int t) {
    return ord == 0 ? t : (t == 0 ? 1 : t == 1 ? 3 : t == 2 ? 0 : t == 3 ? 4 : 2);
}
template <bool LANES, int ORD, bool MF>
__global__ __launch_bounds__(320) void gs_pair_kernel(GsPairArgs g) {
    extern __shared__ __align__(16) unsigned char gsm[];
    double *st_r = reinterpret_cast<double *>(gsm), *st_x = st_r + kGpStage, *st_f = st_x + kGpStage,
           *st_o = st_f + kGpStage;   // [slot][step][line], row stride kGpSR
    // ring1: x1 of step s, lane j at [s % kGpRing][j + 1] (first sweep -> residual wave); ring2: (x1, r2) of step s
    // at [s % kGpRing][2 (j + 1)] (residual wave -> second sweep)
    double(*ring1)[kGpRW] = reinterpret_cast<double(*)[kGpRW]>(gsm + kGpOffRing);
    double(*ring2)[2 * kGpRW] = reinterpret_cast<double(*)[2 * kGpRW]>(gsm + kGpOffRing + (size_t)kGpRing * kGpRW * 8);
    double *e1d = reinterpret_cast<double *>(gsm + kGpOffExt), *e1x = e1d + kGpExt, *e2d = e1x + kGpExt;
    // done through step: [0] first sweep, [1] second; known through position: [2] dx1 and x1, [3] all three;
    // chunks: [4] loaded through, [5] stored through; [6] the band; [7] residuals done through step
    int64_t *ctl = reinterpret_cast<int64_t *>(gsm + kGpOffCtl);
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int j = threadIdx.x & 63;
    const int64_t m = g.m, n = g.n, S = m + kGpOwn, nch = (S + kGpC - 1) / kGpC;
    auto slot = [](int64_t c, int e, int line) { return ((int)(c % kGpNB) * kGpC + e) * kGpSR + line; };
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t t = __hip_atomic_fetch_add(g.tick + kSchedTicket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((int64_t)t == g.nbands + (int64_t)gridDim.x - 1)
                __hip_atomic_store(g.tick + kSchedTicket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ctl[6] = t;
            ctl[0] = ctl[1] = -1;
            ctl[2] = ctl[3] = t > 0 ? -1 : kGpDone;
            ctl[4] = ctl[5] = ctl[7] = -1;
        }
        for (int i = threadIdx.x; i < 3 * kGpExt; i += blockDim.x) e1d[i] = 0.0;   // finite values at positions
        __syncthreads();                                                           // no band publishes
        const int64_t b = ctl[6];
        if (b >= g.nbands) break;
        const int64_t Y0 = b * kGpOwn, Y = Y0 + j;
        double *pb = g.pub + b * 3 * m;
        bool dead = false;   // a wait ran out (error reported): finish the band without waiting
        GP_PROF(unsigned long long wcyc[4] = {0, 0, 0, 0};
                const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
                const unsigned long long c_start = __builtin_amdgcn_s_memtime();)
        auto wait = [&](const int64_t *c, int64_t want, int code) {
            GP_PROF(const unsigned long long tw = __builtin_amdgcn_s_memtime();)
            if (!dead && !gp_wait(c, want, g.err, code, b)) dead = true;
            GP_PROF(wcyc[(code - 5) & 3] += __builtin_amdgcn_s_memtime() - tw;)
        };
        if (wave == kGpW1st) {
            // ---------------- first sweep: lanes 0..63 (lane 63: the next band's first line)
            double prev = 0.0;
            for (int64_t s0 = 0; s0 < S; s0 += kGpBlk) {
                const int64_t c = s0 / kGpC;
                if (s0 > 0) {
                    __builtin_amdgcn_s_waitcnt(0xc07f);   // the ring writes before the announcement
                    if (j == 0) gp_set(&ctl[0], s0 - 1);
                }
                {   // the chunk's r and x0 in LDS, ring1 rows free (read by the residual wave), the band above's dx1
                    const int64_t w2 = b > 0 ? ((s0 + kGpBlk - 1 < m - 1) ? s0 + kGpBlk - 1 : m - 1) : -1;
                    if (!__builtin_amdgcn_readfirstlane((int)(gp_ready(&ctl[4], c) & gp_ready(&ctl[7], s0 + kGpBlk - kGpRing) &
                                                              gp_ready(&ctl[2], w2)))) {
                        wait(&ctl[4], c, 10);
                        wait(&ctl[7], s0 + kGpBlk - kGpRing, 5);
                        wait(&ctl[2], w2, 6);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
                double rr[kGpBlk], xx[kGpBlk], e1[kGpBlk], pdx[kGpBlk];
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const int e = (int)((s0 + k) % kGpC);
                    rr[k] = st_r[slot(c, e, j)];
                    xx[k] = st_x[slot(c, e, j)];
                    e1[k] = e1d[(s0 + k) & (kGpExt - 1)];   // dx1 of (Y0 - 1, s): lane 0's line above
                }
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const int64_t t = s0 + k, a = t - j;
                    const double up = gp_shr1(prev, e1[k]);   // dx1 of (Y - 1, a): lane j - 1, step t - 1
                    const double acc = gp_uacc<LANES, MF>(a > 0 ? g.a1 : 0.0, prev, Y > 0 ? g.am : 0.0, up);
                    const double dx = (rr[k] - acc) / g.d;
                    const double x1 = xx[k] + dx;
                    ring1[t & (kGpRing - 1)][j + 1] = x1;
                    pdx[k] = gp_lane(dx, kGpOwn - 1);
                    prev = dx;   // finite on every lane (absent neighbours carry coefficient 0)
                }
                // the band below's line above: lane 62's dx1 and x1 of the block's steps, stored by lanes 0..7 once per
                // block (one store each instead of a one-lane branch per step)
                {
                    double pd = pdx[0];
#pragma unroll
                    for (int k = 1; k < kGpBlk; ++k) pd = j == k ? pdx[k] : pd;
                    const int64_t a = s0 + j - (kGpOwn - 1);
                    if (j < kGpBlk && Y0 + kGpOwn - 1 < g.H && (uint64_t)a < (uint64_t)m) {
                        gp_store(pb + a, pd);
                        gp_store(pb + m + a, ring1[(s0 + j) & (kGpRing - 1)][kGpOwn]);
                    }
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (j == 0) gp_set(&ctl[0], kGpDone);
            GP_PROF(if (j == 0 && b < 4096) {
                g_gp_prof[b * 16 + 0] = t_start;
                g_gp_prof[b * 16 + 1] = __builtin_amdgcn_s_memrealtime();
                g_gp_prof[b * 16 + 3] = wcyc[0];
                g_gp_prof[b * 16 + 4] = wcyc[1];
                g_gp_prof[b * 16 + 7] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;
                g_gp_prof[b * 16 + 8] = __builtin_amdgcn_s_memtime() - c_start;
            })
        } else if (wave == kGpWRes) {
            // ---------------- the second sweep's residual: at step t lane j forms r2 = f - A x1 of its row of step
            // t - 1 from x1 of steps t - 2, t - 1, t of its own line (ring, then registers) and of lanes j -/+ 1 (DPP)
            double x1p = 0.0, x1pp = 0.0;
            for (int64_t s0 = 0; s0 < S; s0 += kGpBlk) {
                if (s0 > 0) {
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    if (j == 0) gp_set(&ctl[7], s0 - 1);
                }
                {   // ring1 rows through s0 + 7, ring2 rows free, the band above's x1
                    const int64_t w0 = (s0 + kGpBlk - 1 < S - 1) ? s0 + kGpBlk - 1 : S - 1;
                    const int64_t w2 = b > 0 ? ((s0 + kGpBlk - 2 < m - 1) ? s0 + kGpBlk - 2 : m - 1) : -1;
                    if (!__builtin_amdgcn_readfirstlane((int)(gp_ready(&ctl[0], w0) & gp_ready(&ctl[1], s0 + kGpBlk - kGpRing) &
                                                              gp_ready(&ctl[2], w2)))) {
                        wait(&ctl[0], w0, 14);
                        wait(&ctl[1], s0 + kGpBlk - kGpRing, 16);
                        wait(&ctl[2], w2, 15);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
                double xc[kGpBlk], ff[kGpBlk], ex[kGpBlk];
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const int64_t t = s0 + k, tp = t > 0 ? t - 1 : 0;
                    xc[k] = ring1[t & (kGpRing - 1)][j + 1];
                    ff[k] = st_f[slot(tp / kGpC, (int)(tp % kGpC), j)];
                    ex[k] = e1x[(t - 1) & (kGpExt - 1)];   // x1 of (Y0 - 1, t - 1)
                }
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const int64_t t = s0 + k, ap = t - 1 - j;
                    const double x1 = xc[k];
                    // x1 by role (0 d, 1 -m, 2 +m, 3 -1, 4 +1) around (Y, ap)
                    const double xr[5] = {x1p, gp_shl1(x1), gp_shr1(x1pp, ex[k]), x1, x1pp};
                    const bool pr[5] = {true, Y < g.H - 1, Y > 0, ap < m - 1, ap > 0};
                    double sum = 0.0;
#pragma unroll
                    for (int q = 0; q < 5; ++q) {   // A's stored order, rounded products, absent entries skipped
                        const int ro = gp_role(ORD, q);
                        const double u = sum + g.v[q] * xr[ro];
                        sum = pr[ro] ? u : sum;
                    }
                    dv2 w;
                    w.x = x1p;
                    w.y = ff[k] - sum;
                    *reinterpret_cast<dv2 *>(&ring2[(t - 1) & (kGpRing - 1)][2 * (j + 1)]) = w;
                    x1pp = x1p;
                    x1p = x1;
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (j == 0) gp_set(&ctl[7], kGpDone);
            GP_PROF(if (j == 0 && b < 4096) {
                g_gp_prof[b * 16 + 10] = __builtin_amdgcn_s_memtime() - c_start;
                g_gp_prof[b * 16 + 11] = wcyc[1];   // waits on the first sweep
                g_gp_prof[b * 16 + 12] = wcyc[2];   // waits on the band above's x1
            })
        } else if (wave == kGpW2nd) {
            // ---------------- second sweep: lanes 0..62, x1 and r2 from the rings
            const int64_t S1 = m + kGpOwn - 1;
            double prev = 0.0;
            for (int64_t s0 = 0; s0 < S1; s0 += kGpBlk) {
                const int64_t c = s0 / kGpC;
                if (s0 > 0) {
                    __builtin_amdgcn_s_waitcnt(0xc07f);   // the x2 slot writes before the announcement
                    if (j == 0) gp_set(&ctl[1], s0 - 1);
                }
                {   // the chunk's output slot stored, r2 rows through s0 + 7, the band above's dx2
                    const int64_t w7 = (s0 + kGpBlk < S - 1) ? s0 + kGpBlk : S - 1;
                    const int64_t w3 = b > 0 ? ((s0 + kGpBlk - 1 < m - 1) ? s0 + kGpBlk - 1 : m - 1) : -1;
                    if (!__builtin_amdgcn_readfirstlane((int)(gp_ready(&ctl[5], c - kGpNB) & gp_ready(&ctl[7], w7) &
                                                              gp_ready(&ctl[3], w3)))) {
                        wait(&ctl[5], c - kGpNB, 12);
                        wait(&ctl[7], w7, 7);
                        wait(&ctl[3], w3, 8);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                }
                double xv[kGpBlk], rv[kGpBlk], e2[kGpBlk], pdx[kGpBlk];
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const dv2 w = *reinterpret_cast<const dv2 *>(&ring2[(s0 + k) & (kGpRing - 1)][2 * (j + 1)]);
                    xv[k] = w.x;
                    rv[k] = w.y;
                    e2[k] = e2d[(s0 + k) & (kGpExt - 1)];
                }
#pragma unroll
                for (int k = 0; k < kGpBlk; ++k) {
                    const int64_t s = s0 + k, a = s - j;
                    const double up = gp_shr1(prev, e2[k]);
                    const double acc = gp_uacc<LANES, MF>(a > 0 ? g.a1 : 0.0, prev, Y > 0 ? g.am : 0.0, up);
                    const double dx = (rv[k] - acc) / g.d;
                    st_o[slot(c, (int)(s % kGpC), j)] = xv[k] + dx;   // x2
                    pdx[k] = gp_lane(dx, kGpOwn - 1);
                    prev = dx;   // finite on every lane (absent neighbours carry coefficient 0)
                }
                {   // lane 62's dx2 of the block's steps, stored by lanes 0..7
                    double pd = pdx[0];
#pragma unroll
                    for (int k = 1; k < kGpBlk; ++k) pd = j == k ? pdx[k] : pd;
                    const int64_t a = s0 + j - (kGpOwn - 1);
                    if (j < kGpBlk && Y0 + kGpOwn - 1 < g.H && (uint64_t)a < (uint64_t)m) gp_store(pb + 2 * m + a, pd);
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (j == 0) gp_set(&ctl[1], kGpDone);
            GP_PROF(if (j == 0 && b < 4096) {
                g_gp_prof[b * 16 + 2] = __builtin_amdgcn_s_memrealtime();
                g_gp_prof[b * 16 + 5] = wcyc[2];
                g_gp_prof[b * 16 + 6] = wcyc[3];
                g_gp_prof[b * 16 + 9] = __builtin_amdgcn_s_memtime() - c_start;
            })
        } else if (wave == kGpWStream) {
            // ---------------- streaming: lane l -> line J = 4q + l / 16 of instruction q, step e = l % 16 of the chunk
            const __amdgpu_buffer_rsrc_t rr = gp_rsrc(g.r, n), rx = gp_rsrc(g.x, n), rf = gp_rsrc(g.f, n);
            const int e = j & 15;
            auto off = [&](int64_t c, int J, bool own) {   // byte offset of line J's row at step 16c + e, or OOB
                const int64_t s = c * kGpC + e, YJ = Y0 + J;
                const bool ok = YJ < g.H && (uint64_t)(s - J) < (uint64_t)m && (!own || J < kGpOwn);
                return ok ? (uint32_t)((n - 1 - YJ * m - (s - J)) * 8) : kGpOOB;
            };
            int64_t cl = 0, cs = 0, spins = 0;
            while (cs < nch) {
                bool moved = false;
                const int64_t need = (cl - kGpNB + 1) * kGpC;   // the residual wave (behind the first sweep, reading f a
                                                                // step late) past chunk cl - kGpNB
                if (cl < nch && __builtin_amdgcn_readfirstlane((int)(gp_get(&ctl[7]) >= need))) {
                    double vr[16], vx[16], vf[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int J = 4 * q + (j >> 4);
                        const uint32_t o = off(cl, J, false);
                        vr[q] = gp_bload(rr, o);
                        vx[q] = gp_bload(rx, o);
                        vf[q] = gp_bload(rf, o);
                    }
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int J = 4 * q + (j >> 4);
                        st_r[slot(cl, e, J)] = vr[q];
                        st_x[slot(cl, e, J)] = vx[q];
                        st_f[slot(cl, e, J)] = vf[q];
                    }
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    if (j == 0) gp_set(&ctl[4], cl);
                    ++cl;
                    moved = true;
                }
                if (cs < cl && __builtin_amdgcn_readfirstlane((int)(gp_get(&ctl[1]) >= cs * kGpC + kGpC - 1))) {
                    double vo[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q) vo[q] = st_o[slot(cs, e, 4 * q + (j >> 4))];
#pragma unroll
                    for (int q = 0; q < 16; ++q) gp_bstore<0>(rx, off(cs, 4 * q + (j >> 4), true), vo[q]);
                    if (j == 0) gp_set(&ctl[5], cs);   // the slot's values are in the stores' registers
                    ++cs;
                    moved = true;
                }
                if (moved) {
                    spins = 0;
                } else {
                    if (++spins > kGpMaxSpins) {
                        if (j == 0) atomicExch(g.err, (13 << 24) | (int)(b & 0xffffff));
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
        } else if (b > 0) {
            // ---------------- poller: the band above's dx1 / x1 (cursor c1) and dx2 (cursor c2), 64 positions a chunk
            const double *pa = g.pub + (b - 1) * 3 * m;
            int64_t c1 = 0, c2 = 0, k1 = -1, k2 = -1, spins = 0;
            bool got1 = false, got2 = false;
            while (c1 < m || c2 < m) {
                const int64_t w1 = gp_get(&ctl[1]);   // slots of positions <= w1 have been consumed
                bool moved = false;
                if (c1 < m && c1 + 63 - kGpExt <= w1) {
                    const int64_t a = c1 + j;
                    if (!got1) {
                        if (a >= m) {
                            got1 = true;
                        } else {
                            const double d1 = gp_load(pa + a), v1 = gp_load(pa + m + a);
                            if (!gp_sent(d1) && !gp_sent(v1)) {
                                e1d[a & (kGpExt - 1)] = d1;
                                e1x[a & (kGpExt - 1)] = v1;
                                got1 = true;
                            }
                        }
                    }
                    const uint64_t nr = __ballot(!got1);
                    const int64_t k = c1 + (nr ? __builtin_ctzll(nr) : 64) - 1;
                    moved = k > k1;
                    k1 = k;
                    if (!nr) {
                        c1 += 64;
                        got1 = false;
                    }
                }
                if (c2 < m && c2 + 63 - kGpExt <= w1) {
                    const int64_t a = c2 + j;
                    if (!got2) {
                        if (a >= m) {
                            got2 = true;
                        } else {
                            const double d2 = gp_load(pa + 2 * m + a);
                            if (!gp_sent(d2)) {
                                e2d[a & (kGpExt - 1)] = d2;
                                got2 = true;
                            }
                        }
                    }
                    const uint64_t nr = __ballot(!got2);
                    const int64_t k = c2 + (nr ? __builtin_ctzll(nr) : 64) - 1;
                    moved = moved || k > k2;
                    k2 = k;
                    if (!nr) {
                        c2 += 64;
                        got2 = false;
                    }
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);   // LDS writes before the announcements
                if (j == 0) {
                    gp_set(&ctl[2], k1 < m - 1 ? k1 : m - 1);
                    gp_set(&ctl[3], (k1 < k2 ? k1 : k2) < m - 1 ? (k1 < k2 ? k1 : k2) : m - 1);
                }
                if (moved) {
                    spins = 0;
                } else {
                    if (++spins > kGpMaxSpins) {
                        if (j == 0) atomicExch(g.err, (9 << 24) | (int)(b & 0xffffff));
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (j == 0) {
                gp_set(&ctl[2], kGpDone);
                gp_set(&ctl[3], kGpDone);
            }
        }
    }
}

__global__ void gp_fill_kernel(int64_t n, double *p) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) reinterpret_cast<uint64_t *>(p)[i] = kGpSentinel;
}

// presence masks of A's diagonal layout == the m x H grid's (roles as GsPairLevel::role)
struct GpRoles {
    int role[8];
};
__global__ void gp_mask_check_kernel(int64_t n, int64_t m, int K, GpRoles R, const uint8_t *__restrict__ mask,
                                     int32_t *bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t ix = i % m, iy = i / m, H = n / m;
    uint32_t want = 0;
    for (int t = 0; t < K; ++t) {
        const int ro = R.role[t];
        const bool p = ro == 0 || (ro == 1 && iy > 0) || (ro == 2 && iy < H - 1) || (ro == 3 && ix > 0) ||
                       (ro == 4 && ix < m - 1);
        want |= (uint32_t)p << t;
    }
    if (mask[i] != want) atomicOr(bad, 1);
}

// the pair's eligibility (host, at AMG creation): see the comment above gs_pair_kernel
static int gs_pair_setup(psk_csr *A, psk_prec *S, GsPairLevel &g, hipStream_t s) {
    g = GsPairLevel();
    if (!A || !S || S->kind != PSK_PREC_ILU || S->lo.present || !S->up.present || S->up.fd5_m <= 0) return PSK_OK;
    if (S->gather_in || S->gather_out || !S->up.sched || !S->err || A->comm || !A->dg_mask || A->dg_K != 5) return PSK_OK;

    const TriFactor &U = S->up;
    const int64_t n = A->n, m = U.fd5_m;
    if (S->n != n || n % m != 0 || A->ncols != n || n > ((int64_t)1 << 29)) return PSK_OK;   // 32-bit byte offsets
    auto same = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    GpRoles R{};
    int seen = 0;
    for (int t = 0; t < 5; ++t) {
        const int64_t d = A->dg_d[t];
        const int ro = d == 0 ? 0 : d == -m ? 1 : d == m ? 2 : d == -1 ? 3 : d == 1 ? 4 : -1;
        if (ro < 0 || (seen >> ro) & 1) return PSK_OK;
        seen |= 1 << ro;
        R.role[t] = ro;
        g.role[t] = ro;
        g.v[t] = A->dg_v[t];
        if ((ro == 0 && !same(A->dg_v[t], U.fd5_d)) || (ro == 2 && !same(A->dg_v[t], U.fd5_am)) ||
            (ro == 4 && !same(A->dg_v[t], U.fd5_a1)))
            return PSK_OK;
    }
    if (m < 2) return PSK_OK;
    for (int o = 0; o < 2 && g.ord < 0; ++o) {
        bool same_order = true;
        for (int t = 0; t < 5; ++t) same_order = same_order && g.role[t] == gp_role(o, t);
        if (same_order) g.ord = o;
    }
    if (g.ord < 0) return PSK_OK;   // a stored order the kernel is not built for
    DevBuf bad;
    PSK_TRY(bad.ensure(sizeof(int32_t)));
    PSK_HIP(hipMemsetAsync(bad.p, 0, sizeof(int32_t), s));
    hipLaunchKernelGGL(gp_mask_check_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, m, 5, R,
                       A->dg_mask, bad.as<int32_t>());
    PSK_HIP(hipGetLastError());
    int32_t hb = 1;
    PSK_HIP(hipMemcpyAsync(&hb, bad.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    bad.release();
    if (hb) return PSK_OK;
    g.m = m;
    g.H = n / m;
    g.nbands = (g.H + kGpOwn - 1) / kGpOwn;
    PSK_TRY(g.pub.ensure((size_t)(3 * m * g.nbands) * sizeof(double)));
    g.eligible = g.on = true;
    return PSK_OK;
}

// x <- two sweeps from x, given r = f - A x
static int gs_pair_launch(const Context *c, const GsPairLevel &gl, const psk_prec *S, const double *f, const double *r,
                          double *x, hipStream_t s) {
    const TriFactor &U = S->up;
    GsPairArgs g{};
    g.n = gl.m * gl.H;
    g.m = gl.m;
    g.H = gl.H;
    g.nbands = gl.nbands;
    g.d = U.fd5_d;
    g.a1 = U.fd5_a1;
    g.am = U.fd5_am;
    g.mfirst = U.fd5_mfirst;
    for (int t = 0; t < 5; ++t) {
        g.role[t] = gl.role[t];
        g.v[t] = gl.v[t];
    }
    g.f = f;
    g.r = r;
    g.x = x;
    g.pub = gl.pub.as<double>();
    g.tick = U.sched;
    g.err = S->err;
    const int64_t np = 3 * gl.m * gl.nbands;
    hipLaunchKernelGGL(gp_fill_kernel, dim3((unsigned)((np + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, np, g.pub);
    PSK_HIP(hipGetLastError());
    const int64_t grid = std::min<int64_t>(gl.nbands, (int64_t)c->num_cus);   // one workgroup per CU (its LDS)
    // the arithmetic of the schedule the serialized sweep would run now (psk_prec_trisolve_schedule may change it)
    const bool lanes = U.schedule == kSchedSyncFree || U.schedule == kSchedLds || U.schedule == kSchedPart;
    const void *k = nullptr;
#define PSK_GP_K(L, O, F) reinterpret_cast<const void *>(&gs_pair_kernel<L, O, F>)
    if (lanes) k = gl.ord == 0 ? (g.mfirst ? PSK_GP_K(true, 0, true) : PSK_GP_K(true, 0, false))
                               : (g.mfirst ? PSK_GP_K(true, 1, true) : PSK_GP_K(true, 1, false));
    else k = gl.ord == 0 ? (g.mfirst ? PSK_GP_K(false, 0, true) : PSK_GP_K(false, 0, false))
                         : (g.mfirst ? PSK_GP_K(false, 1, true) : PSK_GP_K(false, 1, false));
#undef PSK_GP_K
    void *args[] = {&g};
    PSK_HIP(hipLaunchKernel(k, dim3((unsigned)grid), dim3(320), args, kGpLds, s));
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

__global__ void amg_add_kernel(int64_t n, double *__restrict__ x, const double *__restrict__ d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] + d[i];   // x + dx (ClassicSmoothers.py:14, :34)
}

// ||v||^2 partials, and x = copy(v) (VCycleSolver.py:69) in the same pass
__global__ __launch_bounds__(kBlock) void amg_sqnorm_partial_kernel(int64_t n, const double *__restrict__ v,
                                                                    double *__restrict__ part,
                                                                    double *__restrict__ x) {
    __shared__ double sh[kWaves];
    int64_t t0, t1;
    const int64_t ntiles = (n + kVecTile - 1) / kVecTile;
    block_range(ntiles, t0, t1);
    const int64_t i0 = t0 * kVecTile, i1 = (t1 * kVecTile < n) ? t1 * kVecTile : n;
    double acc = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) {
        const double vi = v[i];
        x[i] = vi;
        acc = fma(vi, vi, acc);
    }
    const double s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// scal[0] = sum of np partials (||v||^2); flag = 0
__global__ __launch_bounds__(kBlock) void amg_init_kernel(const double *part, int np, double *scal,
                                                          int64_t *flag) {
    __shared__ double sh[kWaves];
    const double s = reduce_partials(part, np, 1, sh);
    if (threadIdx.x == 0) {
        scal[0] = s;
        *flag = 0;
    }
}

// convergence test after a non-final cycle (VCycleSolver.py:134-142): 0 -> 1 the first time
__global__ __launch_bounds__(kBlock) void amg_check_kernel(const double *part, int np, const double *scal,
                                                           double tau, int64_t *flag) {
    __shared__ double sh[kWaves];
    const double rr = reduce_partials(part, np, 1, sh);
    if (threadIdx.x == 0 && *flag == 0 && sqrt(rr) < tau * sqrt(scal[0])) *flag = 1;
}

// out = x when flag == want (a converged snapshot (1), or the final x when never converged (0))
__global__ void amg_copy_if_kernel(int64_t n, const int64_t *flag, int64_t want, const double *__restrict__ x,
                                   double *__restrict__ out) {
    if (*flag != want) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = x[i];
}

__global__ void amg_promote_kernel(int64_t *flag) {
    if (*flag == 1) *flag = 2;
}

static inline dim3 vgrid(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

// nu sweeps of x <- x + S^-1 (f - A x) on level lev
static int amg_smooth(const AmgHierarchy *h, const Context *c, int lev, const double *f, double *x, int nu,
                      hipStream_t s) {
    psk_csr *A = h->A[lev];
    const int64_t n = A->n;
    double *r = h->r[lev].as<double>(), *t = h->t[lev].as<double>();
    int it = 0;
    if ((size_t)lev < h->gp.size() && h->gp[lev].on)   // two sweeps per launch (gs_pair_kernel)
        for (; it + 2 <= nu; it += 2) {
            PSK_TRY(launch_spmv(A, kSpmvResid, x, r, nullptr, f, nullptr, nullptr, s));
            PSK_TRY(gs_pair_launch(c, h->gp[lev], h->S[lev], f, r, x, s));
        }
    for (; it < nu; ++it) {
        PSK_TRY(launch_spmv(A, kSpmvResid, x, r, nullptr, f, nullptr, nullptr, s));
        // (round 3: x += U^-1 r fused into the solve's last gather, profiles/r3_amg_fuse_ab.txt)
        if (h->S[lev] && h->S[lev]->kind == PSK_PREC_ILU) {   // Gauss-Seidel: x += U^-1 r in the last gather
            PSK_TRY(ilu_apply_add(h->S[lev], r, x, s));
            continue;
        }
        PSK_TRY(prec_apply_dev(h->S[lev], n, r, t, s));
        hipLaunchKernelGGL(amg_add_kernel, vgrid(n), dim3(kBlock), 0, s, n, x, t);
        PSK_HIP(hipGetLastError());
    }
    return PSK_OK;
}

// x <- runLevel(f, x, lev) (VCycleManager.py:31-62)
static int amg_level(const AmgHierarchy *h, const Context *c, int lev, const double *f, double *x,
                     hipStream_t s) {
    if (lev == 0) return prec_apply_dev(h->coarse, h->A[0]->n, f, x, s);   // spsolve(A_c, f) (:34-37)
    psk_csr *A = h->A[lev];
    PSK_TRY(amg_smooth(h, c, lev, f, x, h->nu_pre, s));                         // :41
    double *r = h->r[lev].as<double>();
    PSK_TRY(launch_spmv(A, kSpmvResid, x, r, nullptr, f, nullptr, nullptr, s));   // :44
    double *f2 = h->f[lev - 1].as<double>(), *x2 = h->x[lev - 1].as<double>();
    psk_csr *R = h->R[lev - 1], *P = h->P[lev - 1];
    PSK_TRY(launch_spmv(R, kSpmvPlain, r, f2, nullptr, nullptr, nullptr, nullptr, s));   // :47
    if (lev - 1 > 0 && h->A[lev - 1]->n > 0)
        PSK_HIP(hipMemsetAsync(x2, 0, (size_t)h->A[lev - 1]->n * sizeof(double), s));   // zeros_like (:50)
    PSK_TRY(amg_level(h, c, lev - 1, f2, x2, s));                                  // :51
    PSK_TRY(launch_spmv(P, kSpmvAdd, x2, x, nullptr, x, nullptr, nullptr, s));   // :54
    return amg_smooth(h, c, lev, f, x, h->nu_post, s);                            // :59
}

int amg_apply(const psk_prec *M, const double *v, double *out, hipStream_t s) {
    const AmgHierarchy *h = M->amg;
    const int64_t n = M->n;
    if (n == 0) return PSK_OK;
    Context *c;
    PSK_TRY(ctx(&c));
    const int top = h->L - 1;
    psk_csr *A = h->A[top];
    double *x = h->x[top].as<double>(), *r = h->r[top].as<double>();
    double *scal = h->scal.as<double>();
    int64_t *flag = reinterpret_cast<int64_t *>(scal + 1);
    double *part = scal + 2;
    const int gv = grid_for_rows(c, n, kVecTile), ga = 1;   // the residual SpMV's sum: in-launch
    hipLaunchKernelGGL(amg_sqnorm_partial_kernel, dim3(gv), dim3(kBlock), 0, s, n, v, part, x);   // + x = copy(b) (:69)
    PSK_HIP(hipGetLastError());
    hipLaunchKernelGGL(amg_init_kernel, dim3(1), dim3(kBlock), 0, s, part, gv, scal, flag);
    PSK_HIP(hipGetLastError());
    for (int k = 0; k < h->num_iters; ++k) {
        PSK_TRY(amg_level(h, c, top, v, x, s));                                            // runCycle (:79)
        if (k + 1 < h->num_iters) {
            PSK_TRY(launch_spmv(A, kSpmvResid, x, r, nullptr, v, part, nullptr, s));   // r = b - A x (:82)
            hipLaunchKernelGGL(amg_check_kernel, dim3(1), dim3(kBlock), 0, s, part, ga, scal, h->tau, flag);
            PSK_HIP(hipGetLastError());
            hipLaunchKernelGGL(amg_copy_if_kernel, vgrid(n), dim3(kBlock), 0, s, n, flag, (int64_t)1, x, out);
            PSK_HIP(hipGetLastError());
            hipLaunchKernelGGL(amg_promote_kernel, dim3(1), dim3(1), 0, s, flag);
            PSK_HIP(hipGetLastError());
        }
    }
    // the last cycle's test does not matter: converged or not (failOnMaxiter=False) x is returned
    hipLaunchKernelGGL(amg_copy_if_kernel, vgrid(n), dim3(kBlock), 0, s, n, flag, (int64_t)0, x, out);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

int amg_gs_pair(psk_prec *M, int set, int *on, int *eligible) {
    if (!M || M->kind != PSK_PREC_AMG) return fail(PSK_ERR_ARG, "amg_gs_pair: not an AMG preconditioner");
    int a = 0, e = 0;
    for (GsPairLevel &g : M->amg->gp) {
        if (set >= 0) g.on = g.eligible && set != 0;
        a += g.on;
        e += g.eligible;
    }
    if (on) *on = a;
    if (eligible) *eligible = e;
    return PSK_OK;
}

int prec_check_error(const psk_prec *M, hipStream_t s) {
    if (!M) return PSK_OK;
    if (M->kind == PSK_PREC_ILU) return ilu_check_error(M, s);
    if (M->kind == PSK_PREC_DENSE) return dense_check_error(M, s);
    if (M->kind == PSK_PREC_AMG) {
        const AmgHierarchy *h = M->amg;
        for (psk_prec *S : h->S)
            if (S && S->kind == PSK_PREC_ILU) PSK_TRY(ilu_check_error(S, s));
        if (h->coarse && h->coarse->kind == PSK_PREC_ILU) PSK_TRY(ilu_check_error(h->coarse, s));
        if (h->coarse && h->coarse->kind == PSK_PREC_DENSE) PSK_TRY(dense_check_error(h->coarse, s));
    }
    return PSK_OK;
}

}  // namespace psk

using namespace psk;

extern "C" int psk_prec_create_amg(int32_t num_levels, psk_csr *const *A, psk_csr *const *P, psk_csr *const *R,
                                   psk_prec *const *smoother, psk_prec *coarse, int32_t num_iters, int32_t nu_pre,
                                   int32_t nu_post, double tau, psk_prec **out) {
    if (!out || num_levels < 1 || !A || !coarse || num_iters < 0 || nu_pre < 0 || nu_post < 0)
        return fail(PSK_ERR_ARG, "psk_prec_create_amg: bad arguments");
    if (num_levels > 1 && (!P || !R || !smoother)) return fail(PSK_ERR_ARG, "psk_prec_create_amg: NULL level arrays");
    const int L = num_levels;
    for (int k = 0; k < L; ++k) {
        if (!A[k]) return fail(PSK_ERR_ARG, "psk_prec_create_amg: NULL level matrix");
        if (A[k]->comm) return fail(PSK_ERR_UNSUPPORTED, "psk_prec_create_amg: sharded matrices (replicas only)");
        if (A[k]->ncols != A[k]->n) return fail(PSK_ERR_ARG, "psk_prec_create_amg: level matrix not square");
    }
    for (int k = 0; k + 1 < L; ++k) {
        if (!P[k] || !R[k]) return fail(PSK_ERR_ARG, "psk_prec_create_amg: NULL transfer operator");
        if (P[k]->n != A[k + 1]->n || P[k]->ncols != A[k]->n)
            return fail(PSK_ERR_ARG, "psk_prec_create_amg: P[k] must be n_{k+1} x n_k");
        if (R[k]->n != A[k]->n || R[k]->ncols != A[k + 1]->n)
            return fail(PSK_ERR_ARG, "psk_prec_create_amg: R[k] must be n_k x n_{k+1}");
    }
    for (int k = 1; k < L; ++k) {
        psk_prec *S = smoother[k];
        if (!S || S->n != A[k]->n || S->kind == PSK_PREC_AMG)
            return fail(PSK_ERR_ARG, "psk_prec_create_amg: smoother[k] missing, of the wrong size or an AMG");
    }
    if (coarse->n != A[0]->n || coarse->kind == PSK_PREC_AMG)
        return fail(PSK_ERR_ARG, "psk_prec_create_amg: coarse solver of the wrong size");
    Context *c;
    PSK_TRY(ctx(&c));
    AmgHierarchy *h = new AmgHierarchy();
    h->L = L;
    h->num_iters = num_iters;
    h->nu_pre = nu_pre;
    h->nu_post = nu_post;
    h->tau = tau;
    h->A.assign(A, A + L);
    if (L > 1) {
        h->P.assign(P, P + L - 1);
        h->R.assign(R, R + L - 1);
        h->S.assign(smoother, smoother + L);
        h->S[0] = nullptr;   // built but never used by the reference (VCycleManager.py:23-24)
    }
    h->coarse = coarse;
    h->x.resize(L);
    h->f.resize(L);
    h->r.resize(L);
    h->t.resize(L);
    int rc = PSK_OK;
    for (int k = 0; k < L && rc == PSK_OK; ++k) {
        const size_t bytes = (size_t)std::max<int64_t>(A[k]->n, 1) * sizeof(double);
        rc = h->x[k].ensure(bytes);
        if (rc == PSK_OK && k < L - 1) rc = h->f[k].ensure(bytes);
        if (rc == PSK_OK && (k > 0 || L == 1)) rc = h->r[k].ensure(bytes);
        if (rc == PSK_OK && k > 0) rc = h->t[k].ensure(bytes);
    }
    if (rc == PSK_OK) rc = h->r[L - 1].ensure((size_t)std::max<int64_t>(A[L - 1]->n, 1) * sizeof(double));
    if (rc == PSK_OK) rc = h->scal.ensure((size_t)(2 + kMaxGrid) * sizeof(double));
    h->gp.resize(L);
    for (int k = 1; k < L && rc == PSK_OK; ++k) rc = gs_pair_setup(h->A[k], h->S[k], h->gp[k], c->stream);
    if (rc != PSK_OK) {
        amg_free(h);
        return rc;
    }
    psk_prec *M = new psk_prec();
    M->kind = PSK_PREC_AMG;
    M->n = A[L - 1]->n;
    M->amg = h;
    *out = M;
    return PSK_OK;
}

// ---------------------------------------------------------------------------------------------
// host setup: SmoothedAggregation.py:41-183 in O(nnz)
extern "C" int psk_sa_aggregate(int64_t n, const int32_t *rowptr, const int32_t *colidx, const double *vals,
                                double tol, int32_t *agg_out, int64_t *count_out, double *af_vals) {
    if (n < 0 || !rowptr || !agg_out || !count_out || (n > 0 && rowptr[n] > 0 && (!colidx || !vals)))
        return fail(PSK_ERR_ARG, "psk_sa_aggregate: bad arguments");
    const int64_t nnz = n > 0 ? rowptr[n] : 0;
    for (int64_t i = 0; i < n; ++i)
        if (rowptr[i + 1] < rowptr[i]) return fail(PSK_ERR_ARG, "psk_sa_aggregate: rowptr not monotone");
    for (int64_t k = 0; k < nnz; ++k)
        if (colidx[k] < 0 || colidx[k] >= n) return fail(PSK_ERR_ARG, "psk_sa_aggregate: column out of range");
    // A.diagonal(): sum of the row's diagonal entries in stored order (scipy csr_diagonal)
    std::vector<double> d(n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
            if (colidx[k] == i) d[i] += vals[k];
    // strength (getNeighborhood, :49-54): abs(a_ij) >= tol*sqrt(a_ii*a_jj); N_i = {i} U strong
    std::vector<uint8_t> strong(nnz, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
            strong[k] = std::fabs(vals[k]) >= tol * std::sqrt(d[i] * d[colidx[k]]);
    auto in_n = [&](int64_t i, int32_t j, auto &&pred) {   // iterate N_i: i itself, then strong columns
        if (!pred((int32_t)i)) return false;
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
            if (strong[k] && !pred(colidx[k])) return false;
        return true;
    };
    std::vector<int32_t> agg(n, -1);
    std::vector<uint8_t> in_r(n, 1), late(n, 0);
    std::vector<int64_t> root;
    // isolated nodes: |N_i| == 1 (:73-77)
    for (int64_t i = 0; i < n; ++i) {
        bool iso = true;
        for (int32_t k = rowptr[i]; k < rowptr[i + 1] && iso; ++k)
            if (strong[k] && colidx[k] != i) iso = false;
        if (iso) {
            agg[i] = (int32_t)root.size();
            in_r[i] = 0;
            root.push_back(i);
        }
    }
    // phase 1 (:84-89): N_i entirely unaggregated -> new aggregate N_i
    for (int64_t i = 0; i < n; ++i) {
        if (!in_r[i]) continue;
        if (!in_n(i, 0, [&](int32_t j) { return in_r[j] != 0; })) continue;
        const int32_t id = (int32_t)root.size();
        in_n(i, 0, [&](int32_t j) {
            agg[j] = id;
            in_r[j] = 0;
            return true;
        });
        root.push_back(i);
    }
    const int64_t count = (int64_t)root.size();
    if (count == 0 && n > 0) return fail(PSK_ERR_ARG, "psk_sa_aggregate: no aggregates (reference: aggregates[-1] IndexError)");
    if (count >= INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "psk_sa_aggregate: too many aggregates");
    // phase 2 (:104-127) against the phase-1 snapshot: candidates = aggregates meeting N_i; strength
    // of a candidate = max |A[i,k]| over its members k (A[i,k] sums duplicate entries); strictly
    // largest wins, first in list order on ties; none positive -> aggregates[-1]
    std::vector<int32_t> snap(agg);
    std::vector<int32_t> cand;
    std::vector<std::pair<int32_t, double>> colsum;   // (k, A[i,k]) for members of candidates
    for (int64_t i = 0; i < n; ++i) {
        if (!in_r[i]) continue;
        cand.clear();
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k)
            if (strong[k] && snap[colidx[k]] >= 0) cand.push_back(snap[colidx[k]]);
        std::sort(cand.begin(), cand.end());
        cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
        colsum.clear();
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            const int32_t j = colidx[k];
            if (snap[j] < 0 || !std::binary_search(cand.begin(), cand.end(), snap[j])) continue;
            bool merged = false;
            for (auto &e : colsum)
                if (e.first == j) {
                    e.second += vals[k];
                    merged = true;
                    break;
                }
            if (!merged) colsum.emplace_back(j, vals[k]);
        }
        double best = 0.0;
        int32_t best_c = -1;
        for (const int32_t cc : cand)   // list order
            for (const auto &e : colsum)
                if (snap[e.first] == cc && std::fabs(e.second) > best) {
                    best = std::fabs(e.second);
                    best_c = cc;
                }
        agg[i] = best_c >= 0 ? best_c : (int32_t)(count - 1);
        late[i] = 1;
    }
    std::copy(agg.begin(), agg.end(), agg_out);
    *count_out = count;
    if (!af_vals) return PSK_OK;
    // BuildFilteredMatrix (:157-183). neighborhoods[i] as it reads them: the original N_i, grown by
    // the phase-2 members of aggregate c when i is c's root (the reference's aggregate list holds
    // the neighbourhood set objects themselves, :75/:88, and phase 2 adds to them, :126).
    std::vector<int32_t> root_of(n, -1);
    for (int64_t cidx = 0; cidx < count; ++cidx) root_of[root[cidx]] = (int32_t)cidx;
    std::copy(vals, vals + nnz, af_vals);
    int64_t iptr = -1;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t s = rowptr[i], e = rowptr[i + 1];
        for (int32_t k = s; k < e; ++k)
            if (colidx[k] == i) {
                iptr = k;
                break;
            }
        for (int32_t k = s; k < e; ++k) {
            const int32_t j = colidx[k];
            bool keep = (j == i);
            for (int32_t q = s; q < e && !keep; ++q) keep = strong[q] && colidx[q] == j;
            if (!keep && root_of[i] >= 0 && late[j] && agg[j] == root_of[i]) keep = true;
            if (keep) continue;
            if (iptr < 0) return fail(PSK_ERR_ARG, "psk_sa_aggregate: row without a diagonal entry (reference: NameError)");
            af_vals[iptr] -= af_vals[k];
            af_vals[k] = 0.0;
        }
    }
    return PSK_OK;
}
