// ilu.hip — sparse triangular-solve chains on the device: right-ILUT apply
// (RightILUTPreconditioner.applyRight, ILUTPreconditioner.py:70-78), RightIC apply
// (ICPreconditioner.py:58-63), the Gauss-Seidel smoother's U^-1 (ClassicSmoothers.py:28-36) and the
// AMG coarse-level SuperLU solve (VCycleManager.py:34-37) are all "gather, lower solve, upper solve,
// gather" with some stages absent (psk_prec_create_trisolve).
//
// The reference calls SuperLU's ILU.solve(v) (scipy SuperLU, dgstrs): with Pr A Pc ~= L U,
//     bb[perm_r[i]] = v[i];  y = L^-1 bb (unit lower);  z = U^-1 y;  out[i] = z[perm_c[i]].
// The factors come from the same third-party factorisation on the host (scipy spilu, exactly the
// reference's call, ILUTPreconditioner.py:51-53): they are uploaded once per form() and the two
// triangular solves run on the GPU.
//
// Publication protocol (both schedules): the output is pre-filled with a signalling-NaN sentinel that
// arithmetic never produces; each x[i] is written by ONE 8-byte agent-scope store (sc1) and read by
// agent-scope relaxed loads that bypass the non-coherent L1 (MI355X_MICROARCH.md, hand-off granule
// R2: "the data IS the flag"). Every spin is bounded and reports PSK_ERR instead of hanging.
//
// Schedule 1, sync-free (sptrsv_kernel): one wave per row, rows dealt to a co-resident grid in a
// level-sorted topological order computed on the host (k-th row of that order -> wave k mod W; every
// row depends only on rows earlier in the order, so the first unsolved row can always proceed).
// Level order instead of index order cut the apply at FD m=1024 from 255 ms to 17 ms. Each
// dependency level costs about one cross-CU hand-off (~1 us, MI355X_MICROARCH.md "handoff-1to1").
//
// Schedule 2, band (sptrsv_band_kernel): the solve order is cut into contiguous blocks, one
// workgroup per block; the workgroup walks the block's LOCAL dependency levels with a barrier
// between levels, so a dependency inside the block costs a barrier and an LDS-ring read instead of
// a hand-off; only dependencies on earlier blocks go through the published values. For the
// Gauss-Seidel factor triu(A) of a 5-point grid (2m-1 levels, each up to m rows wide) this is what
// makes the smoother usable at m = 8192.
//
// Also below: the single-workgroup LDS schedule (small factors, x in LDS), the grid schedule (2-D
// stencil factors: one wave per band of 64 lines along a skewed coordinate) and the partitioned
// schedule (strips of the natural index, one workgroup per CU, in-strip hand-offs through LDS). The
// host simulates the schedules with measured per-level / per-row costs and keeps the fastest
// (TriFactor::schedule; psk_prec_trisolve_schedule reports and overrides it).
#include "psk_internal.hpp"

#include <algorithm>
#include <chrono>
#include <unordered_map>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <queue>
#include <vector>

namespace psk {

constexpr uint64_t kSentinel = 0x7FF4DEAD0000BEEFull;   // sNaN payload: never an arithmetic result
constexpr int64_t kMaxSpins = 1ll << 24;
constexpr int kRingMaxWords = 16384;                     // 128 KiB LDS ring (then 1 workgroup / CU)

__device__ __forceinline__ double load_pub(const double *p) {
    const uint64_t b = __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    return __longlong_as_double((long long)b);
}

__device__ __forceinline__ void store_pub(double *p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t *>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool is_sentinel(double v) { return (uint64_t)__double_as_longlong(v) == kSentinel; }

__device__ __forceinline__ double wait_pub(const double *p, int32_t *err) {
    double xv = load_pub(p);
    int64_t spins = 0;
    while (is_sentinel(xv)) {
        if (++spins > kMaxSpins) {
            atomicExch(err, 1);
            return 0.0;
        }
        __builtin_amdgcn_s_sleep(4);   // sleep 1 / 4 / 12 between polls: AMG 8192^2 2.90 / 2.92 / 2.90 it/s
        xv = load_pub(p);
    }
    return xv;
}

// ---- forward progress without co-residency (round 5) ---------------------
// The spin-waiting schedules no longer assume that every workgroup of their grid is resident at once (a
// plain launch promises nothing: a caller's kernels on other streams, a second process on the device or
// the halo exchange's kernels may hold CUs). Each takes its work from counters in TriFactor::sched (words
// on separate 256-B lines, zero between launches):
//  * band / narrow band / grid: a workgroup draws its next block (band) from a ticket counter instead of
//    deriving it from blockIdx.x. A block waits only on earlier blocks, and every earlier block was drawn
//    by a workgroup that has started and runs to completion, so the lowest unfinished block can always
//    proceed. The drawer of the launch's last ticket re-arms the counter.
//  * sync-free: a row may wait on ANY earlier position, so rows are dealt round-robin over the waves that
//    ENROLLED: the first workgroup to start waits until all gridDim.x have enrolled or kEnrollWaitTicks
//    have passed, closes the enrolment and publishes the count R; positions are dealt over those 4R waves,
//    and workgroups that arrive later leave at once. Every row is then held by a running wave. The last
//    workgroup to leave re-arms the words.
// The grid is unchanged when the device is free (all workgroups enrol within a few us); under contention
// the solve runs on fewer waves instead of waiting on workgroups that cannot start.
// kSchedTicket / kSchedPub / kSchedExit / kSchedLast / kSchedWords: psk_internal.hpp (the lab library reads kSchedLast)
constexpr uint32_t kEnrollClosed = 0x80000000u;
constexpr uint64_t kEnrollWaitTicks = 2000;   // s_memrealtime (100 MHz): 20 us

__device__ __forceinline__ uint32_t sched_add(uint32_t *w, uint32_t v) {
    return __hip_atomic_fetch_add(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t sched_load(const uint32_t *w) {
    return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sched_store(uint32_t *w, uint32_t v) {
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// thread 0: the next block of a ticket-dealt launch (every workgroup draws until it gets one >= nblocks,
// so the launch draws exactly nblocks + gridDim.x tickets; the last drawer re-arms the counter)
__device__ __forceinline__ int64_t sched_next_block(uint32_t *sched, int64_t nblocks) {
    const uint32_t t = sched_add(sched + kSchedTicket, 1u);
    if ((int64_t)t == nblocks + (int64_t)gridDim.x - 1) sched_store(sched + kSchedTicket, 0u);
    return t;
}

// thread 0: the block of a launch in which every workgroup draws exactly one (the grid schedule's bands);
// the drawer of ticket gridDim.x - 1 re-arms the counter
__device__ __forceinline__ int64_t sched_one_block(uint32_t *sched) {
    const uint32_t t = sched_add(sched + kSchedTicket, 1u);
    if (t == gridDim.x - 1) sched_store(sched + kSchedTicket, 0u);
    return t;
}

// every thread: enrol this workgroup (see above); returns its worker rank (-1: arrived after the close) and
// the worker count R in *R. Bounded: the decider waits at most kEnrollWaitTicks.
__device__ __forceinline__ int sched_enroll(uint32_t *sched, uint32_t *R, int32_t *err) {
    __shared__ int s_rank;
    __shared__ uint32_t s_R;
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x;
        const uint32_t old = sched_add(sched + kSchedTicket, 1u);
        if (old & kEnrollClosed) {
            s_rank = -1;
            s_R = 0;
        } else if (old == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while ((sched_load(sched + kSchedTicket) & ~kEnrollClosed) < G &&
                   __builtin_amdgcn_s_memrealtime() - t0 < kEnrollWaitTicks)
                __builtin_amdgcn_s_sleep(2);
            const uint32_t r = __hip_atomic_fetch_or(sched + kSchedTicket, kEnrollClosed, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) & ~kEnrollClosed;
            sched_store(sched + kSchedPub, r);
            sched_store(sched + kSchedLast, r);   // kept after the launch (psk_lab_trisolve_workers)
            s_rank = 0;
            s_R = r;
        } else {
            uint32_t r;
            int64_t spins = 0;
            while ((r = sched_load(sched + kSchedPub)) == 0) {
                if (++spins > kMaxSpins) {
                    atomicExch(err, 4 << 24);
                    r = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_rank = (int)old;
            s_R = r;
        }
    }
    __syncthreads();
    *R = s_R;
    return s_rank;
}

// every thread, at the very end of an enrolled launch (after the workgroup's last use of the words)
__device__ __forceinline__ void sched_leave(uint32_t *sched) {
    __syncthreads();
    if (threadIdx.x == 0 && sched_add(sched + kSchedExit, 1u) == gridDim.x - 1) {
        sched_store(sched + kSchedTicket, 0u);
        sched_store(sched + kSchedPub, 0u);
        sched_store(sched + kSchedExit, 0u);
    }
}

__global__ void fill_sentinel_kernel(int64_t n, double *x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) reinterpret_cast<uint64_t *>(x)[i] = kSentinel;
}

// Branch-free row pipeline (the LDS kernel's, SfSrc below). The compiler's vmcnt waits count only
// the memory operations it knows were issued; a load under a divergent branch (a lane test, a row
// past the end) is not counted, so the wait for a row's first dependency became vmcnt(0) — it also
// waited for the prefetch of the rows D ahead issued after it, which is what the pipeline exists to
// hide. Every load of SfSrc is issued by every lane at a clamped, valid address (the value selected
// afterwards), the row header is loaded per lane (VMEM, counted in order, not SMEM), and the rare
// slow path (a row longer than the register chunks) ends with an explicit vmcnt(0), so the fast
// path's counts survive its join.
__device__ __forceinline__ void drain_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // vmcnt(0) only
__device__ __forceinline__ int32_t opaque_zero() {
    int32_t z;
    __asm__ volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

struct SfHead {
    int32_t row, s, e;
};
constexpr int kSfChunks = 3;   // 64-entry chunks of a row held in registers (longer rows loop)
struct SfBody {
    int32_t row, s, e, ri, c[kSfChunks];
    double v[kSfChunks], d;
};

constexpr int kSfTail = 4;

// Row total of the sync-free family (sync-free, LDS, partitioned kernels: the same function, so the
// three give identical bits): the DPP wave total (psk_internal.hpp), ~130 cycles on the dependency
// chain where a butterfly of ds_bpermute shuffles took ~700 (tools/part_micro.py trace, FD chain).
__device__ __forceinline__ double row_total(double v) { return wave_total(v); }

// the loads of a row (positions clamped into [0, n), entries into [0, nnz); callers select)
struct SfSrc {
    int64_t n;
    int32_t last;   // nnz - 1 (>= 0)
    const int32_t *krp, *kci, *krow, *ridx;   // ridx: rhs_idx, or krow (any valid int array of n)
    const double *kva, *dg;                   // dg: diag, or rhs (any valid double array of n)
    bool has_ri, has_d;
    int32_t zv;                               // opaque zero: per-lane header loads
    __device__ void head(int64_t k, SfHead &h) const {
        const int64_t kk = (k < n ? k : n - 1) + zv;
        h.row = krow[kk];
        h.s = krp[kk];
        h.e = krp[kk + 1];
    }
    __device__ void body(const SfHead &h, SfBody &b, int lane) const {
        b.row = h.row;
        b.s = h.s;
        b.e = h.e;
        // lanes past the row's end re-read its first entry (the line lane 0 reads; an empty row: the
        // entry before it), never one shared address (a hot line every wave would hit)
        const int32_t fb = h.s < h.e ? h.s : (h.e > 0 ? h.e - 1 : 0);
#pragma unroll
        for (int j = 0; j < kSfChunks; ++j) {
            const int32_t idx = h.s + 64 * j + lane;
            const bool ok = idx < h.e;
            const int32_t ic = ok ? idx : fb;
            const int32_t c = kci[ic];
            const double v = kva[ic];
            b.c[j] = ok ? c : -1;
            b.v[j] = ok ? v : 0.0;
        }
        const int32_t ri = ridx[h.row];
        const double d = dg[h.row];
        b.ri = has_ri ? ri : h.row;
        b.d = has_d ? d : 1.0;
    }
};

// Sync-free: x_i = (rhs_i - sum_j T_ij x_j) / diag_i  (diag == nullptr: unit), rhs_i = rhs[rhs_idx[i]]
// when rhs_idx is given. The factor is stored in SOLVE ORDER (host-built): position k holds row
// krow[k] with entries [krp[k], krp[k+1]) of kci/kva, so a wave's rows stream. Wave w takes positions
// w, w+W, ... and software-pipelines them: while it waits on the dependencies of position k it already
// has position k+W's row, entries, right-hand side and diagonal in flight (stage B) and position
// k+2W's row header (stage A), so a row costs one hand-off round trip instead of a chain of dependent
// HBM loads (order -> rowptr -> entries -> rhs index -> rhs). Its loads stay under lane tests: the
// branch-free form of the LDS kernel below (SfSrc) measured 27.0 -> 27.9-28.9 ms on configs[2]'s ILU
// apply (profiles/r3_grid_phase_probe.txt), where the hand-off, not the compiler's waits, bounds a row.
struct SfRow {
    int32_t row, s, e, c[kSfChunks];
    double v[kSfChunks], b, d;
};

__device__ __forceinline__ void sptrsv_rows(int64_t n, const int32_t *__restrict__ krp, const int32_t *__restrict__ kci,
                                            const double *__restrict__ kva, const double *__restrict__ diag,
                                            const double *__restrict__ rhs, const int32_t *__restrict__ rhs_idx, double *x,
                                            int32_t *err, const int32_t *__restrict__ krow, int64_t wave, int64_t W) {
    const int lane = threadIdx.x & 63;
    if (wave >= n) return;
    auto head = [&](int64_t k, SfHead &h) {
        if (k < n) {
            h.row = krow[k];
            h.s = krp[k];
            h.e = krp[k + 1];
        }
    };
    auto body = [&](int64_t k, const SfHead &h, SfRow &b) {
        if (k < n) {
            b.row = h.row;
            b.s = h.s;
            b.e = h.e;
#pragma unroll
            for (int j = 0; j < kSfChunks; ++j) {
                const int32_t idx = h.s + 64 * j + lane;
                b.c[j] = idx < h.e ? kci[idx] : -1;
                b.v[j] = idx < h.e ? kva[idx] : 0.0;
            }
            if (lane == 0) {
                b.b = rhs[rhs_idx ? rhs_idx[h.row] : h.row];
                b.d = diag ? diag[h.row] : 1.0;
            }
        }
    };
    SfHead ha, hb;
    SfRow cur, nxt;
    head(wave, ha);
    body(wave, ha, cur);
    head(wave + W, hb);
    for (int64_t k = wave; k < n; k += W) {
        // the first poll of this row goes out before the prefetches, so waiting for it does not
        // wait for them (loads complete in order)
        uint64_t bits[kSfChunks];
#pragma unroll
        for (int j = 0; j < kSfChunks; ++j)
            bits[j] = cur.c[j] >= 0 ? __hip_atomic_load(reinterpret_cast<const uint64_t *>(x + cur.c[j]),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                    : 0;
        body(k + W, hb, nxt);       // stage B of k+W (its header arrived an iteration ago)
        head(k + 2 * W, hb);        // stage A of k+2W
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < kSfChunks; ++j)   // lane's entries in stored order: lane, lane+64, ...
            if (cur.c[j] >= 0) {
                double xv = __longlong_as_double((long long)bits[j]);
                if (is_sentinel(xv)) xv = wait_pub(x + cur.c[j], err);
                acc = fma(cur.v[j], xv, acc);
            }
        // longer rows: kSfTail chunks of entries, then their x values, in flight at once
        for (int32_t base = cur.s + 64 * kSfChunks; base < cur.e; base += 64 * kSfTail) {
            int32_t tc[kSfTail];
            double tv[kSfTail];
            uint64_t tb[kSfTail];
#pragma unroll
            for (int t = 0; t < kSfTail; ++t) {
                const int32_t idx = base + 64 * t + lane;
                tc[t] = idx < cur.e ? kci[idx] : -1;
                tv[t] = idx < cur.e ? kva[idx] : 0.0;
            }
#pragma unroll
            for (int t = 0; t < kSfTail; ++t)
                tb[t] = tc[t] >= 0 ? __hip_atomic_load(reinterpret_cast<const uint64_t *>(x + tc[t]), __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0;
#pragma unroll
            for (int t = 0; t < kSfTail; ++t)
                if (tc[t] >= 0) {
                    double xv = __longlong_as_double((long long)tb[t]);
                    if (is_sentinel(xv)) xv = wait_pub(x + tc[t], err);
                    acc = fma(tv[t], xv, acc);
                }
        }
        const double sum = row_total(acc);
        if (lane == 0) {
            double r = cur.b - sum;
            if (diag) r = r / cur.d;
            store_pub(x + cur.row, r);
        }
        cur = nxt;
    }
}

__global__ __launch_bounds__(kBlock) void sptrsv_kernel(int64_t n, const int32_t *__restrict__ krp,
                                                        const int32_t *__restrict__ kci, const double *__restrict__ kva,
                                                        const double *__restrict__ diag, const double *__restrict__ rhs,
                                                        const int32_t *__restrict__ rhs_idx, double *x,
                                                        int32_t *err, const int32_t *__restrict__ krow,
                                                        uint32_t *sched) {
    // positions dealt over the waves of the workgroups that enrolled (sched_enroll), not over the grid
    uint32_t R = 0;
    const int rank = sched_enroll(sched, &R, err);
    if (rank >= 0) sptrsv_rows(n, krp, kci, kva, diag, rhs, rhs_idx, x, err, krow, (int64_t)rank * kWaves + (threadIdx.x >> 6),
                               (int64_t)R * kWaves);
    sched_leave(sched);
}

// LDS-resident: a factor small enough for x to live in LDS (the AMG coarse LU: 16.6k rows, 3008
// levels, ~140 entries per row) is solved by ONE workgroup of 16 waves running the sync-free
// schedule above with x in LDS: a dependency hand-off is an LDS write seen by another wave's LDS
// poll (~0.1 us) instead of a device-scope store seen by a polling load (~1-2 us). Each wave still
// prefetches its next rows' entries from HBM while it waits. x is copied out at the end.
constexpr int kLdsThreads = 1024;
constexpr int kLdsTail = 8;
constexpr int kLdsDepth = 3;   // rows in flight per wave (PSK_LDS_DEPTH=1..3 overrides)
constexpr int64_t kLdsMaxRows = 18432;   // 144 KiB of x

template <int D>
__global__ __launch_bounds__(kLdsThreads) void sptrsv_lds_kernel(int64_t n, const int32_t *__restrict__ krp,
                                                                 const int32_t *__restrict__ kci,
                                                                 const double *__restrict__ kva,
                                                                 const double *__restrict__ diag,
                                                                 const double *__restrict__ rhs,
                                                                 const int32_t *__restrict__ rhs_idx, double *x,
                                                                 int32_t *err, const int32_t *__restrict__ krow) {
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t *xs = reinterpret_cast<uint64_t *>(smem);
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t wave = tid >> 6, W = kLdsThreads / 64;
    for (int64_t i = tid; i < n; i += kLdsThreads) xs[i] = kSentinel;
    __syncthreads();
    auto lds_wait = [&](int32_t c) -> double {
        uint64_t b = __hip_atomic_load(xs + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        int64_t spins = 0;
        while (b == kSentinel) {
            if (++spins > kMaxSpins) {
                atomicExch(err, 1);
                return 0.0;
            }
            __builtin_amdgcn_s_sleep(1);
            b = __hip_atomic_load(xs + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return __longlong_as_double((long long)b);
    };
    const int32_t nnz = krp[n];
    if (nnz == 0) {   // diagonal factor: no dependencies
        for (int64_t k = wave; k < n; k += W) {
            const int32_t row = krow[k];
            double r = rhs[rhs_idx ? rhs_idx[row] : row];
            if (diag) r = r / diag[row];
            if (lane == 0) x[row] = r;
        }
        return;
    }
    const SfSrc src{n, nnz - 1, krp, kci, krow, rhs_idx ? rhs_idx : krow, kva, diag ? diag : rhs,
                    rhs_idx != nullptr, diag != nullptr, opaque_zero()};
    // register ring of D rows per wave: row k's entries are loaded D rows (D*W positions) before
    // it is solved and its header 2D rows before, so a wave keeps D rows of HBM loads in flight
    // while it waits on LDS hand-offs (one row in flight cost one HBM round trip per row); all of
    // them branch-free (see SfSrc), so the compiler's vmcnt waits leave them in flight
    SfHead hq[D];
    SfBody bq[D];
#pragma unroll
    for (int t = 0; t < D; ++t) src.head(wave + t * W, hq[t]);
#pragma unroll
    for (int t = 0; t < D; ++t) src.body(hq[t], bq[t], lane);
#pragma unroll
    for (int t = 0; t < D; ++t) src.head(wave + (D + t) * W, hq[t]);
    for (int64_t k0 = wave; k0 < n; k0 += D * W) {
#pragma unroll
        for (int t = 0; t < D; ++t) {
            const int64_t k = k0 + t * W;
            if (k >= n) break;
            const SfBody cur = bq[t];
            const double bv = rhs[cur.ri];   // goes out before the prefetches (loads complete in order)
            src.body(hq[t], bq[t], lane);
            src.head(k + 2 * D * W, hq[t]);
            // all of this row's first LDS reads go out together; only a sentinel among them waits
            uint64_t bits[kSfChunks];
#pragma unroll
            for (int j = 0; j < kSfChunks; ++j)
                bits[j] = __hip_atomic_load(xs + (cur.c[j] >= 0 ? cur.c[j] : 0), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < kSfChunks; ++j)   // lane's entries in stored order: lane, lane+64, ...
                if (cur.c[j] >= 0)
                    acc = fma(cur.v[j],
                              bits[j] == kSentinel ? lds_wait(cur.c[j]) : __longlong_as_double((long long)bits[j]), acc);
            // longer rows (the dense tail of an LU factor, uniform): kLdsTail chunks of entries in flight at once
            if (cur.e - cur.s > 64 * kSfChunks) {
                for (int32_t base = cur.s + 64 * kSfChunks; base < cur.e; base += 64 * kLdsTail) {
                    int32_t tc[kLdsTail];
                    double tv[kLdsTail];
                    uint64_t tb[kLdsTail];
#pragma unroll
                    for (int u = 0; u < kLdsTail; ++u) {
                        const int32_t idx = base + 64 * u + lane;
                        tc[u] = idx < cur.e ? kci[idx] : -1;
                        tv[u] = idx < cur.e ? kva[idx] : 0.0;
                    }
#pragma unroll
                    for (int u = 0; u < kLdsTail; ++u)
                        tb[u] = tc[u] >= 0 ? __hip_atomic_load(xs + tc[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0;
#pragma unroll
                    for (int u = 0; u < kLdsTail; ++u)
                        if (tc[u] >= 0)
                            acc = fma(tv[u], tb[u] == kSentinel ? lds_wait(tc[u]) : __longlong_as_double((long long)tb[u]),
                                      acc);
                }
                drain_vm();
            }
            const double sum = row_total(acc);
            double r = bv - sum;
            if (diag) r = r / cur.d;
            // every lane: the same value to the same LDS word
            __hip_atomic_store(xs + cur.row, (uint64_t)__double_as_longlong(r), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    __syncthreads();
    for (int64_t i = tid; i < n; i += kLdsThreads) x[i] = __longlong_as_double((long long)xs[i]);
}

// Partitioned (sptrsv_part_kernel): the rows are cut into P strips of the NATURAL index (the
// matrix's own numbering before the factorisation's permutations: for ILU the original equation /
// unknown of every factor row), one strip per workgroup of 16 waves, one workgroup per CU. A strip of
// a mesh-like matrix is a band of the mesh, so most dependencies of its rows are rows of the same
// strip: those hand-offs go through LDS (~0.1 us) instead of a device-scope store seen by a polling
// load (~1 us). Each workgroup runs its rows in ASAP order (earliest finish under the cost model,
// host-computed: a topological order), dealt round-robin to its waves; every wave runs the sync-free
// row pipeline above. Entry codes: c >= 0 = another strip's row, read from x with the sentinel
// protocol; c < 0 = the strip's own row at local position qd = -c-1, read from an LDS cache of
// kPartSlots results (slot qd mod kPartSlots) whose tag is the local position it holds. Rows write x
// (the output) and the cache; the tag goes to kPartWriting while a slot is rewritten, so a reader
// that sees the same tag before and after reading the value has that row's value, a newer tag means
// the slot was reused (the value is then read from x), an older one that the row is not done. Same
// per-row arithmetic as sync-free (same entry order, lane partials, row_total), so bit-identical to it.
// Progress: all P workgroups are co-resident (one per CU, P <= CUs); the globally ASAP-first unsolved
// row has all its dependencies solved and every earlier row of its wave is ASAP-earlier.
constexpr int kPartThreads = 1024;
constexpr int kPartWaves = kPartThreads / 64;
constexpr int kPartSlots = 8192;                // 64 KiB of values + 32 KiB of tags
constexpr int32_t kPartPad = INT32_MIN;         // padding lane
constexpr int32_t kPartEmpty = -1, kPartWriting = -2;
constexpr size_t kPartLds = (size_t)kPartSlots * (sizeof(double) + sizeof(int32_t));

// Every load of the row pipeline is unconditional (clamped positions, entry arrays padded by
// kPartPadEntries on the host, the right-hand side pre-gathered): a load under a divergent branch
// makes the compiler wait for ALL outstanding loads (vmcnt(0)) at the join, which would serialise
// the prefetch of the next rows behind this row's dependency polls.
#ifdef PSK_PART_PROF
// development probe: [0] wave cycles, [1] local-wait cycles, [2] remote-wait cycles, [3] rows,
// [4] local waits, [5] remote waits, [6] slot reuses, [7] max wave cycles (summed over the launch)
__device__ unsigned long long g_part_prof[8];
extern "C" int psk_part_prof_read(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_part_prof), sizeof(g_part_prof)) != hipSuccess) return -1;
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_part_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// per-position phase stamps (clock64) of the first 2^17 positions, 8 words each: [0] the row's turn
// (its wave's pipeline loads for later rows issued), [1] local (LDS) dependencies read, [2] every
// entry's x value in and the lane partial summed (remote polls included), [3] row total (DPP),
// [4] quotient, [5] x and the LDS cache written (issued); [6] 1 if the spin waited, [7] spins
constexpr int kPartTraceWords = 8;
__device__ unsigned long long g_part_trace[kPartTraceWords << 17];
extern "C" int psk_part_trace_read(unsigned long long *out, int64_t n) {
    if (n > (1 << 17)) n = 1 << 17;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_part_trace), (size_t)n * 8 * kPartTraceWords) == hipSuccess ? 0 : -1;
}
#define PART_PROF(...) __VA_ARGS__
#else
#define PART_PROF(...)
#endif
constexpr int kPtChunks = 2;   // 64-entry chunks of a row held in registers (4 rows in flight per wave)
constexpr int kPartPadEntries = 64 * kPtChunks;
struct PtBody {
    int32_t row, s, e, c[kPtChunks];
    double v[kPtChunks], b, d;
};

template <bool UNIT>
__global__ __launch_bounds__(kPartThreads) void sptrsv_part_kernel(
    const int64_t *__restrict__ seg, const int32_t *__restrict__ krp, const int32_t *__restrict__ kcode,
    const double *__restrict__ kva, const double *__restrict__ diag, const double *__restrict__ rhs, double *x,
    int32_t *err, const int32_t *__restrict__ krow) {
    extern __shared__ __align__(16) unsigned char smem[];
    // LDS accesses are workgroup-scope relaxed atomics: ds_read / ds_write in program order, no waits
    // between them (a wave's LDS operations execute in issue order)
    uint64_t *sv = reinterpret_cast<uint64_t *>(smem);
    int32_t *st = reinterpret_cast<int32_t *>(smem + kPartSlots * sizeof(double));
    auto ld_tag = [&](int32_t s) { return __hip_atomic_load(st + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto ld_val = [&](int32_t s) {
        return __longlong_as_double((long long)__hip_atomic_load(sv + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t wave = tid >> 6;
    for (int i = tid; i < kPartSlots; i += kPartThreads) st[i] = kPartEmpty;   // before the barrier: plain
    __syncthreads();
    const int64_t base = seg[blockIdx.x], R = seg[blockIdx.x + 1] - base;
    if (wave >= R) return;
    PART_PROF(const unsigned long long pt0 = clock64(); unsigned long long plw = 0, prw = 0, pnl = 0, pnr = 0, pev = 0;)
    auto head = [&](int64_t q, SfHead &h) {   // q >= R: a valid position whose row is never used
        const int64_t k = base + (q < R ? q : R - 1);
        h.row = krow[k];
        h.s = krp[k];
        h.e = krp[k + 1];
    };
    auto body = [&](const SfHead &h, PtBody &b) {
        b.row = h.row;
        b.s = h.s;
        b.e = h.e;
#pragma unroll
        for (int j = 0; j < kPtChunks; ++j) {
            const int32_t idx = h.s + 64 * j + lane;   // < nnz + kPartPadEntries
            const int32_t c = kcode[idx];
            b.v[j] = kva[idx];
            b.c[j] = idx < h.e ? c : kPartPad;
        }
        b.b = rhs[h.row];
        b.d = UNIT ? 1.0 : diag[h.row];
    };
    // an entry's x value: bits/t1/v/t2 are its first reads (issued together for the whole row)
    auto resolve = [&](int32_t c, uint64_t bits, int32_t t1, double v, int32_t t2) -> double {
        if (c >= 0) {
            const double xv = __longlong_as_double((long long)bits);
            return is_sentinel(xv) ? wait_pub(x + c, err) : xv;
        }
        const int32_t qd = ~c, slot = qd & (kPartSlots - 1);   // ~c == -c-1
        int64_t spins = 0;
        PART_PROF(const unsigned long long w0 = clock64(); if (!(t1 == qd && t2 == qd)) pnl++;)
        while (!(t1 == qd && t2 == qd)) {
            if (t1 > qd || t1 == qd) {
                PART_PROF(pev++;)
                return wait_pub(x + krow[base + qd], err);   // slot reused: x has it
            }
            if (++spins > kMaxSpins) {
                atomicExch(err, 2);
                return 0.0;
            }
            __builtin_amdgcn_s_sleep(1);
            t1 = ld_tag(slot);
            v = ld_val(slot);
            t2 = ld_tag(slot);
        }
        PART_PROF(plw += clock64() - w0;)
        return v;
    };
    // Software pipeline over the wave's rows u = 0, 1, ... (position wave + u*W): in iteration u the
    // wave issues the first x polls of row u+1, the entries of row u+3 and the header of row u+5, then
    // resolves row u. Every load a step waits for was issued at least one iteration earlier and the
    // polls go out first, so (loads completing in order) resolving row u waits only for its own polls
    // and what was issued two iterations before: a wave keeps ~3 rows of loads in flight and a row
    // whose dependencies are done costs no memory round trip of its own. Rings: bodies and headers 4,
    // polls 2; the loop is unrolled by 4 so every ring index is a constant.
    auto poll = [&](const PtBody &b, uint64_t *bits) {   // first polls of the remote entries
#pragma unroll
        for (int j = 0; j < kPtChunks; ++j)
            bits[j] = __hip_atomic_load(reinterpret_cast<const uint64_t *>(x + (b.c[j] >= 0 ? b.c[j] : 0)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    constexpr int64_t W = kPartWaves;
    SfHead H[4];
    PtBody B[4];
    uint64_t P[2][kPtChunks];
    head(wave, H[0]);
    head(wave + W, H[1]);
    head(wave + 2 * W, H[2]);
    body(H[0], B[0]);
    body(H[1], B[1]);
    body(H[2], B[2]);
    head(wave + 3 * W, H[3]);
    head(wave + 4 * W, H[0]);
    poll(B[0], P[0]);
    for (int64_t q0 = wave; q0 < R; q0 += 4 * W) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t q = q0 + t * W;
            if (q >= R) break;
            poll(B[(t + 1) & 3], P[(t + 1) & 1]);   // row u+1 (entries issued two iterations ago)
            body(H[(t + 3) & 3], B[(t + 3) & 3]);   // row u+3 (header issued two iterations ago)
            head(q + 5 * W, H[(t + 1) & 3]);         // row u+5
            const PtBody &cur = B[t];
            const uint64_t *pc = P[t & 1];
            PART_PROF(const unsigned long long ph0 = clock64(); unsigned long long nspin = 0;)
            // x values of the row's register chunks: remote ones from the early polls, local ones from
            // the LDS cache, polled by the whole wave until every local entry is present (the spin's
            // control flow is uniform); reused slots and unpublished remote values then wait on x
            double xv[kPtChunks];
            bool pend[kPtChunks];
#pragma unroll
            for (int j = 0; j < kPtChunks; ++j) {
                xv[j] = 0.0;   // remote values are read from the polls only below (no wait for them here)
                pend[j] = cur.c[j] < 0 && cur.c[j] != kPartPad;   // local, not yet read
            }
            PART_PROF(const unsigned long long w0 = clock64(); bool waited = false;)
            for (int64_t spins = 0;; ++spins) {
                bool left = false;
#pragma unroll
                for (int j = 0; j < kPtChunks; ++j)
                    if (pend[j]) {
                        const int32_t qd = ~cur.c[j], slot = qd & (kPartSlots - 1);
                        const int32_t t1 = ld_tag(slot);
                        const double v = ld_val(slot);
                        const int32_t t2 = ld_tag(slot);
                        if (t1 == qd && t2 == qd) {
                            xv[j] = v;
                            pend[j] = false;
                        } else if (t1 >= qd) {   // slot reused (or being rewritten): x holds the value
                            xv[j] = wait_pub(x + krow[base + qd], err);
                            pend[j] = false;
                            PART_PROF(pev++;)
                        } else {
                            left = true;
                        }
                    }
                if (!__any(left)) break;
                if (spins > kMaxSpins) {
                    if (lane == 0) atomicExch(err, 2);
                    break;
                }
                PART_PROF(waited = true; ++nspin;)
#ifndef PSK_PART_SLEEP
#define PSK_PART_SLEEP 1
#endif
                __builtin_amdgcn_s_sleep(PSK_PART_SLEEP);
            }
            PART_PROF(if (waited) { plw += clock64() - w0; pnl++; }
                      for (int j = 0; j < kPtChunks; ++j) __asm__ volatile("" ::"v"(xv[j]));
                      const unsigned long long ph1 = clock64();)
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < kPtChunks; ++j) {
                const int32_t c = cur.c[j];
                if (c == kPartPad) continue;
                if (c >= 0) {
                    xv[j] = __longlong_as_double((long long)pc[j]);
                    if (is_sentinel(xv[j])) {
                        PART_PROF(const unsigned long long w1 = clock64(); pnr++;)
                        xv[j] = wait_pub(x + c, err);
                        PART_PROF(prw += clock64() - w1;)
                    }
                }
                acc = fma(cur.v[j], xv[j], acc);
            }
            for (int32_t b0 = cur.s + 64 * kPtChunks; b0 < cur.e; b0 += 64 * kSfTail) {   // long rows
                int32_t tc[kSfTail];
                double tv[kSfTail];
#pragma unroll
                for (int u = 0; u < kSfTail; ++u) {
                    const int32_t idx = b0 + 64 * u + lane;
                    tc[u] = idx < cur.e ? kcode[idx] : kPartPad;
                    tv[u] = idx < cur.e ? kva[idx] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < kSfTail; ++u)
                    if (tc[u] != kPartPad) {
                        const int32_t c = tc[u], slot = ~c & (kPartSlots - 1);
                        const uint64_t bt = c >= 0 ? __hip_atomic_load(reinterpret_cast<const uint64_t *>(x + c),
                                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                   : 0;
                        const int32_t a1 = c < 0 ? ld_tag(slot) : 0;
                        const double vv = c < 0 ? ld_val(slot) : 0.0;
                        const int32_t a2 = c < 0 ? ld_tag(slot) : 0;
                        acc = fma(tv[u], resolve(c, bt, a1, vv, a2), acc);
                    }
            }
            PART_PROF(__asm__ volatile("" ::"v"(acc)); const unsigned long long ph2 = clock64();)
            const double sum = row_total(acc);
            PART_PROF(__asm__ volatile("" ::"v"(sum)); const unsigned long long ph3 = clock64();)
            if (lane == 0) {
                double r = cur.b - sum;
                if (!UNIT) r = r / cur.d;
                PART_PROF(__asm__ volatile("" ::"v"(r)); const unsigned long long ph4 = clock64();)
                store_pub(x + cur.row, r);
                const int32_t slot = (int32_t)(q & (kPartSlots - 1));
                __hip_atomic_store(st + slot, kPartWriting, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(sv + slot, (uint64_t)__double_as_longlong(r), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(st + slot, (int32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                PART_PROF(if (base + q < (1 << 17)) {
                    const unsigned long long ph5 = clock64();
                    unsigned long long *tr = g_part_trace + kPartTraceWords * (base + q);
                    tr[0] = ph0;
                    tr[1] = ph1;
                    tr[2] = ph2;
                    tr[3] = ph3;
                    tr[4] = ph4;
                    tr[5] = ph5;
                    tr[6] = waited ? 1 : 0;
                    tr[7] = nspin;
                })
            }
        }
    }
#ifdef PSK_PART_PROF
    unsigned long long vals[6] = {clock64() - pt0, plw, prw, pnl, pnr, pev};
    for (int i = 0; i < 6; ++i)
        for (int o = 32; o > 0; o >>= 1) vals[i] = max(vals[i], (unsigned long long)__shfl_xor((long long)vals[i], o));
    if (lane == 0) {
        atomicAdd(&g_part_prof[0], vals[0]);
        atomicAdd(&g_part_prof[1], vals[1]);
        atomicAdd(&g_part_prof[2], vals[2]);
        atomicAdd(&g_part_prof[4], vals[3]);
        atomicAdd(&g_part_prof[5], vals[4]);
        atomicAdd(&g_part_prof[6], vals[5]);
        atomicMax(&g_part_prof[7], vals[0]);
        atomicAdd(&g_part_prof[3], (unsigned long long)((R - wave + kPartWaves - 1) / kPartWaves));
    }
#endif
}


// Band: workgroup g takes blocks g, g+G, ... in solve order. Position of row i in solve order: i
// (lower) or n-1-i (upper); block b = positions [b*B, (b+1)*B). The block's rows come as a RECORD
// stream in local-level order (SoA, host-built): row, end of its level (relative to the block),
// K off-diagonal (column, value) pairs (column -1 = padding), diagonal. Records are staged into LDS in
// chunks of kBandChunk (one per thread), double-buffered, the next chunk's global loads issued a
// whole chunk ahead, so a level costs LDS reads + barrier instead of dependent global loads. One
// thread per record of a level (levels are at most kBandChunk wide, host-checked). In-block results
// go to an LDS ring (position & ring_mask, host-verified reuse distance) as well as to x; dependencies
// on earlier blocks are waited on through x.
constexpr int kBandChunk = kBlock;   // records per staged chunk = widest level = threads
#ifdef PSK_BAND_PROF
__device__ unsigned long long g_band_prof[8];   // development probe: cycles per phase of block 100's levels
extern "C" int psk_band_prof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_band_prof), sizeof(g_band_prof)) == hipSuccess ? 0 : -1;
}
#endif

template <int K>
struct BandChunkRegs {
    int32_t row = 0, end = 0, c[K];
    double v[K], e[K], d = 1.0, b = 0.0;   // e: snapshot of external dependencies (sentinel = not yet)
};

template <int K>
__global__ __launch_bounds__(kBlock) void sptrsv_band_kernel(
    int64_t n, int upper, const double *__restrict__ rhs, const int32_t *__restrict__ rhs_idx, double *x,
    int32_t *err, const int32_t *__restrict__ rec_row, const int32_t *__restrict__ rec_end,
    const int32_t *__restrict__ rec_c, const double *__restrict__ rec_v, const double *__restrict__ rec_d,
    int64_t nblocks, int64_t B, int ring_mask, uint32_t *sched) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int64_t s_blk;
    const int ring_words = ring_mask + 1;
    double *ring = reinterpret_cast<double *>(smem);
    // two chunk buffers, SoA: v[K][C], d[C], b[C], e[K][C] (doubles) then row[C], end[C], c[K][C] (ints)
    constexpr int kD = 2 * K + 2;
    double *dbuf = ring + ring_words;
    int32_t *ibuf = reinterpret_cast<int32_t *>(dbuf + 2 * kD * kBandChunk);
    const int tid = threadIdx.x;
    const double sentinel = __longlong_as_double((long long)kSentinel);
    // global -> registers, a chunk ahead of use; dependencies on earlier blocks are loaded too (their
    // producers usually finished them long before this block reaches them; if not, the snapshot is the
    // sentinel and the consumer waits at use time)
    auto stage_load = [&](int64_t q, int64_t q_end, int64_t p_lo, BandChunkRegs<K> &r) {
        if (q < q_end) {
            r.row = rec_row[q];
            r.end = rec_end[q];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                r.c[k] = rec_c[(int64_t)k * n + q];
                r.v[k] = rec_v[(int64_t)k * n + q];
                const int32_t c = r.c[k];
                r.e[k] = (c >= 0 && (upper ? (n - 1 - c) : c) < p_lo) ? load_pub(x + c) : sentinel;
            }
            r.d = rec_d ? rec_d[q] : 1.0;
            r.b = rhs_idx ? rhs[rhs_idx[r.row]] : rhs[r.row];
        }
    };
    auto stage_store = [&](int buf, const BandChunkRegs<K> &r) {             // registers -> LDS
        double *db = dbuf + buf * kD * kBandChunk;
        int32_t *ib = ibuf + buf * (K + 2) * kBandChunk;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            db[k * kBandChunk + tid] = r.v[k];
            db[(K + 2 + k) * kBandChunk + tid] = r.e[k];
            ib[(2 + k) * kBandChunk + tid] = r.c[k];
        }
        db[K * kBandChunk + tid] = r.d;
        db[(K + 1) * kBandChunk + tid] = r.b;
        ib[tid] = r.row;
        ib[kBandChunk + tid] = r.end;
    };
    for (;;) {   // blocks drawn from the ticket counter (sched_next_block): forward progress at any residency
        if (tid == 0) s_blk = sched_next_block(sched, nblocks);
        __syncthreads();
        const int64_t blk = s_blk;
        if (blk >= nblocks) break;
        const int64_t p_lo = blk * B, p_hi = (p_lo + B < n) ? p_lo + B : n, nrec = p_hi - p_lo;
        const int64_t nchunks = (nrec + kBandChunk - 1) / kBandChunk;
        BandChunkRegs<K> next;
        stage_load(p_lo + tid, p_hi, p_lo, next);
        stage_store(0, next);
        if (nchunks > 1) stage_load(p_lo + kBandChunk + tid, p_hi, p_lo, next);   // chunk 1 in flight
        int64_t have = 1;   // chunks [0, have) staged; chunk c lives in buffer c & 1
        __syncthreads();
        int64_t a = 0;
        auto advance = [&]() {   // stage chunk `have` (loads issued a chunk ago), issue the next one
            stage_store((int)(have & 1), next);
            if (have + 1 < nchunks) stage_load(p_lo + (have + 1) * kBandChunk + tid, p_hi, p_lo, next);
            ++have;
            __syncthreads();
        };
        while (a < nrec) {
#ifdef PSK_BAND_PROF
            const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
            if (a / kBandChunk >= have) advance();                      // level starts in the next chunk
            const int64_t ca = a / kBandChunk;
            const int32_t *iba = ibuf + (ca & 1) * (K + 2) * kBandChunk;
            const int64_t bnd = iba[kBandChunk + (a % kBandChunk)];   // end of this level (relative)
            if ((bnd - 1) / kBandChunk >= have) advance();              // level reaches into the next chunk
#ifdef PSK_BAND_PROF
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            uint64_t t2 = t1;
#endif
            const int64_t r = a + tid;
            if (r < bnd) {
                const int cb = (int)((r / kBandChunk) & 1), sl = (int)(r % kBandChunk);
                const double *db = dbuf + cb * kD * kBandChunk;
                const int32_t *ib = ibuf + cb * (K + 2) * kBandChunk;
                // every LDS read of the record first (one round trip), then every ring read (a
                // second one; entries that are not in-block read slot 0, unused), then the sum in
                // stored order: a local level is ~3 dependent LDS round trips instead of ~10
                const int32_t row = ib[sl];
                int32_t cc[K];
                int64_t pc[K];
                double vv[K], ee[K], rg[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    cc[k] = ib[(2 + k) * kBandChunk + sl];
                    vv[k] = db[k * kBandChunk + sl];
                    ee[k] = db[(K + 2 + k) * kBandChunk + sl];
                }
                const double bb = db[(K + 1) * kBandChunk + sl];
                const double dd = rec_d ? db[K * kBandChunk + sl] : 1.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    pc[k] = upper ? (n - 1 - cc[k]) : cc[k];
                    rg[k] = ring_mask >= 0 ? ring[(cc[k] >= 0 && pc[k] >= p_lo ? pc[k] : 0) & ring_mask] : 0.0;
                }
#ifdef PSK_BAND_PROF
                __builtin_amdgcn_s_waitcnt(0xc07f);
                t2 = __builtin_amdgcn_s_memtime();
#endif
                double acc = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (cc[k] >= 0) {
                        double xv;
                        if (pc[k] < p_lo) {   // earlier block: the staged snapshot, else wait for it
                            xv = ee[k];
                            if (is_sentinel(xv)) xv = wait_pub(x + cc[k], err);
                        } else {
                            xv = ring_mask >= 0 ? rg[k] : wait_pub(x + cc[k], err);
                        }
                        acc = fma(vv[k], xv, acc);
                    }
                }
                double res = bb - acc;
                if (rec_d) res = res / dd;
                if (ring_mask >= 0) ring[(upper ? (n - 1 - row) : row) & ring_mask] = res;
                store_pub(x + row, res);
            }
#ifdef PSK_BAND_PROF
            const uint64_t t3 = __builtin_amdgcn_s_memtime();
#endif
            // LDS results of this level visible to the next; x stores may still be in flight
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
#ifdef PSK_BAND_PROF
            if (tid == 0 && blk == 100) {
                const uint64_t t4 = __builtin_amdgcn_s_memtime();
                g_band_prof[0] += t1 - t0;
                g_band_prof[1] += t2 - t1;
                g_band_prof[2] += t3 - t2;
                g_band_prof[3] += t4 - t3;
                g_band_prof[4] += 1;
            }
#endif
            a = bnd;
        }
        __syncthreads();   // ring and buffers reused by the next block of this workgroup
    }
}

// Narrow band: the band schedule for factors whose local levels are at most one wave wide (the
// Gauss-Seidel factor triu(A) of a 2-D grid, any block of lines). Wave 0 solves the block's levels
// alone, with no workgroup barrier between levels (LDS traffic of one wave is in order); waves 1-3
// stage the record chunks into kNarrowBufs LDS buffers ahead of it and, while they wait for a free
// buffer, re-poll the external snapshots still holding the sentinel, so the solving wave finds its
// dependencies on earlier blocks in LDS instead of paying an agent-scope load round trip per level
// (tools/band_prof.py: that round trip was ~60% of a band level). Hand-shakes through LDS counters:
// ctl[b] = stager waves that finished staging buffer b (3 per round), ctl[NB] = last chunk the solver
// finished, ctl[NB+1] = block done.
constexpr int kNarrowBufs = 3;
constexpr int kNarrowChunk = 128;   // records per buffer
constexpr int kNarrowWidth = 64;    // widest local level (one wave)

__device__ __forceinline__ int32_t lds_load_acq(int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int K>
__global__ __launch_bounds__(kBlock) void sptrsv_band_narrow_kernel(
    int64_t n, int upper, const double *__restrict__ rhs, const int32_t *__restrict__ rhs_idx, double *x,
    int32_t *err, const int32_t *__restrict__ rec_row, const int32_t *__restrict__ rec_end,
    const int32_t *__restrict__ rec_c, const double *__restrict__ rec_v, const double *__restrict__ rec_d,
    int64_t nblocks, int64_t B, int ring_mask, uint32_t *sched) {
    constexpr int C = kNarrowChunk, NB = kNarrowBufs, kD = 2 * K + 2;
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int64_t s_blk;
    const int ring_words = ring_mask + 1;
    double *ring = reinterpret_cast<double *>(smem);
    double *dbuf = ring + ring_words;                                        // NB x [v[K], d, b, e[K]] x C
    int32_t *ibuf = reinterpret_cast<int32_t *>(dbuf + NB * kD * C);         // NB x [row, end, c[K]] x C
    int32_t *ctl = ibuf + NB * (K + 2) * C;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const double sentinel = __longlong_as_double((long long)kSentinel);
    for (;;) {   // blocks drawn from the ticket counter (sched_next_block)
        if (tid == 0) s_blk = sched_next_block(sched, nblocks);
        __syncthreads();
        const int64_t blk = s_blk;
        if (blk >= nblocks) break;
        const int64_t p_lo = blk * B, p_hi = (p_lo + B < n) ? p_lo + B : n, nrec = p_hi - p_lo;
        const int64_t nchunks = (nrec + C - 1) / C;
        if (tid <= NB + 1) ctl[tid] = tid == NB ? -1 : 0;
        __syncthreads();
        if (wave == 0) {
            int64_t seen = -1, cur = 0, a = 0;
            auto wait_chunk = [&](int64_t q) {
                if (q <= seen) return;
                const int32_t need = 3 * (int32_t)(q / NB + 1);
                int64_t spins = 0;
                while (lds_load_acq(&ctl[q % NB]) < need) {
                    if (++spins > kMaxSpins) {
                        atomicExch(err, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                seen = q;
            };
            while (a < nrec) {
#ifdef PSK_BAND_PROF
                const uint64_t t0 = __builtin_amdgcn_s_memtime();
                int hits = 0;
#endif
                const int64_t q = a / C;
                if (q > cur) {   // every level of chunks < q is done: their buffers may be restaged
                    if (lane == 0) __hip_atomic_store(&ctl[NB], (int32_t)(q - 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    cur = q;
                }
                wait_chunk(q);
                const int64_t bnd = ibuf[(q % NB) * (K + 2) * C + C + (a % C)];
                if ((bnd - 1) / C > q) wait_chunk(q + 1);
#ifdef PSK_BAND_PROF
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                uint64_t t2 = t1;
#endif
                const int64_t r = a + lane;
                if (r < bnd) {
                    const int bf = (int)((r / C) % NB), sl = (int)(r % C);
                    const double *db = dbuf + bf * kD * C;
                    const int32_t *ib = ibuf + bf * (K + 2) * C;
                    const int32_t row = ib[sl];
                    int32_t cc[K];
                    int64_t pc[K];
                    double vv[K], ee[K], rg[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        cc[k] = ib[(2 + k) * C + sl];
                        vv[k] = db[k * C + sl];
                        ee[k] = __longlong_as_double((long long)__hip_atomic_load(
                            reinterpret_cast<const uint64_t *>(db + (K + 2 + k) * C + sl), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP));
                    }
                    const double bb = db[(K + 1) * C + sl];
                    const double dd = rec_d ? db[K * C + sl] : 1.0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        pc[k] = upper ? (n - 1 - cc[k]) : cc[k];
                        rg[k] = ring[(cc[k] >= 0 && pc[k] >= p_lo ? pc[k] : 0) & ring_mask];
                    }
#ifdef PSK_BAND_PROF
                    __builtin_amdgcn_s_waitcnt(0xc07f);
                    t2 = __builtin_amdgcn_s_memtime();
#endif
                    double acc = 0.0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (cc[k] >= 0) {
                            double xv;
                            if (pc[k] < p_lo) {
                                xv = ee[k];
#ifdef PSK_BAND_PROF
                                if (is_sentinel(xv)) ++hits;
#endif
                                if (is_sentinel(xv)) xv = wait_pub(x + cc[k], err);
                            } else {
                                xv = rg[k];
                            }
                            acc = fma(vv[k], xv, acc);
                        }
                    }
                    double res = bb - acc;
                    if (rec_d) res = res / dd;
                    ring[(upper ? (n - 1 - row) : row) & ring_mask] = res;
                    store_pub(x + row, res);
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);   // this level's ring writes before the next level's reads
                __builtin_amdgcn_wave_barrier();
#ifdef PSK_BAND_PROF
                {
                    const uint64_t t3 = __builtin_amdgcn_s_memtime();
                    t2 = __shfl(t2, 0, 64);
                    hits = __reduce_add_sync(0xffffffffffffffffull, hits);
                    if (lane == 0 && blk == 100) {
                        g_band_prof[0] += t1 - t0;
                        g_band_prof[1] += t2 - t1;
                        g_band_prof[2] += t3 - t2;
                        g_band_prof[3] += (uint64_t)hits;
                        g_band_prof[4] += 1;
                    }
                }
#endif
                a = bnd;
            }
            if (lane == 0) {
                __hip_atomic_store(&ctl[NB], (int32_t)(nchunks - 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(&ctl[NB + 1], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else {
            // stager thread st owns slot st of every buffer (and slot st + 192 < C: none for C = 128)
            const int st = tid - 64;
            const bool owns = st < C;
            int64_t last_q[NB];
            uint32_t pending[NB];   // bit k: entry k of the owned slot still holds the sentinel
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                last_q[b] = -1;
                pending[b] = 0;
            }
            auto refresh = [&]() {
                const int32_t done_q = lds_load_acq(&ctl[NB]);
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (pending[b] == 0 || last_q[b] <= done_q) continue;
                    const int32_t *ib = ibuf + b * (K + 2) * C;
                    double *db = dbuf + b * kD * C;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (pending[b] & (1u << k)) {
                            const double v = load_pub(x + ib[(2 + k) * C + st]);
                            if (!is_sentinel(v)) {
                                __hip_atomic_store(reinterpret_cast<uint64_t *>(db + (K + 2 + k) * C + st),
                                                   (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP);
                                pending[b] &= ~(1u << k);
                            }
                        }
                }
            };
            for (int64_t q = 0; q < nchunks; ++q) {
                const int b = (int)(q % NB);
                int64_t spins = 0;
                while (lds_load_acq(&ctl[NB]) < q - NB) {   // buffer b still holds chunk q - NB
                    refresh();
                    if (++spins > kMaxSpins) {
                        atomicExch(err, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                const int64_t rq = p_lo + q * C + st;
                pending[b] = 0;
                last_q[b] = q;
                if (owns && rq < p_hi) {
                    double *db = dbuf + b * kD * C;
                    int32_t *ib = ibuf + b * (K + 2) * C;
                    const int32_t row = rec_row[rq];
                    ib[st] = row;
                    ib[C + st] = rec_end[rq];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int32_t c = rec_c[(int64_t)k * n + rq];
                        ib[(2 + k) * C + st] = c;
                        db[k * C + st] = rec_v[(int64_t)k * n + rq];
                        double e = sentinel;
                        if (c >= 0 && (upper ? (n - 1 - c) : c) < p_lo) {
                            e = load_pub(x + c);
                            if (is_sentinel(e)) pending[b] |= 1u << k;
                        }
                        db[(K + 2 + k) * C + st] = e;
                    }
                    db[K * C + st] = rec_d ? rec_d[rq] : 1.0;
                    db[(K + 1) * C + st] = rhs_idx ? rhs[rhs_idx[row]] : rhs[row];
                }
                __builtin_amdgcn_s_waitcnt(0xc07f);   // this wave's LDS writes done
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) __hip_atomic_fetch_add(&ctl[b], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            int64_t spins = 0;
            while (lds_load_acq(&ctl[NB + 1]) == 0) {
                refresh();
                if (++spins > kMaxSpins) {
                    atomicExch(err, 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();   // ring, buffers and counters reused by the next block of this workgroup
    }
}

// Grid: a factor whose dependencies, in solve order q, form a 2-D stencil: with q = y*w + x (w
// positions per line), every off-diagonal entry of row q refers to q' = q - (yd*w + xd) with
// 0 <= yd < 64 lines back and, for the skew chosen by the host, ud = xd + g(y) - g(y - yd) >= 1 steps
// back along u = x + g(y) (the 5-point Gauss-Seidel factor triu(A): (0,1), (1,0), g(y) = y; an
// SA coarse operator of a 2-D grid: up to 2 lines back with diagonal neighbours). The skew may be a
// half integer, g(y) = (sigma2 * y + phase) >> 1 with sigma2 odd: SA level 3 of -FD 4096^2 (2048 lines
// of 1366) has a dependency (1 line, 2 positions ahead) on every other line only, which an integer
// skew can only meet with g(y) = 3y; g(y) = (5y + 1) >> 1 meets it with 13.6% fewer steps. One wave per band
// of 64 lines; lane j owns line y0+j and all lanes advance together along u, so step s solves 64
// rows that do not depend on each other; a dependency on the same band is a read of the LDS ring
// holding the band's last `ring` steps (ring[(s mod ring)*64 + lane]); only lanes j < yd reach into
// the band above, through the published values (pre-filled sentinel, agent-scope store / poll as
// the other schedules), prefetched D steps ahead with everything else a step needs. The critical
// path is the u range (w + g(H) steps) plus one hand-off lag per band, instead of one hand-off
// per dependency level. Per-row arithmetic is the band kernels': fma over the entries in stored
// order from 0.0, then (b - acc) / diag, so results are bit-identical to the band schedule.
constexpr int kGridLanes = 64;
constexpr int kGridMaxRing = 128;   // ring rows the plan may ask for (the kernel's mirrored kGridRing)
#ifdef PSK_GRID_PROF
// development probe (tools/grid_probe.py): per band start / end s_memtime, waits and cycles waited
// 8 words per band: start, end, waits on the band above, cycles waited, then the solver's cycles per
// step phase summed over the band: records + rhs ready, LDS ring reads, arithmetic (fma chain and
// division), ring write + x store issued
__device__ unsigned long long g_grid_prof[8192 * 8];
extern "C" int psk_grid_prof_read(unsigned long long *out, int nbands) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_grid_prof), sizeof(unsigned long long) * 8 * (size_t)nbands) ==
                   hipSuccess ? 0 : -1;
}
#endif

// Records of one step of a band: three contiguous 64-lane fields — K 16-bit pattern codes per lane,
// K values per lane (stored entry order), the diagonal — so each field load is one contiguous access
// (one 32-B record per lane, loaded as two 16-B halves, touched twice the cache lines and ran the
// 5-point sweep 1.6x slower).
template <int K>
struct GridStep {
    static constexpr int64_t kCode = 0;                                   // uint16 [64][K]
    static constexpr int64_t kCoef = kGridLanes * 2 * K;                  // double [64][K]
    static constexpr int64_t kDiag = kCoef + kGridLanes * 8 * K;          // double [64]
    static constexpr int64_t kBytes = kDiag + kGridLanes * 8;
};

// Two waves per band. The SOLVER wave (lanes = the band's 64 lines) advances along u. Its records
// are stored in its access order — slot = (band * S_full + step) * 64 + lane — one 16-B-multiple
// record per slot, so a step's records are one contiguous 64-lane stream, prefetched D steps ahead;
// rhs and x stay in natural order (each lane walks its own line). Dependencies come from ONE LDS ring
// of kGridRing steps x kGridRW columns: columns [8 - maxyd, 8) hold the band above's last maxyd lines,
// written by the POLLER wave as their values get published (64 u-positions polled at a time, the ready
// prefix announced through an LDS counter after every round trip), column 8 + j the solver's lane j; a
// dependency (yd lines, ud steps back) of lane j is column 8 + j - yd of ring row (s - ud) whoever
// produced it. The ring is MIRRORED (every row written at r and r + kGridRing, one ds_write2st64), so a
// dependency's byte address is the step's row base plus a per-entry constant (kept per dictionary
// record): one VALU add per entry instead of the modular row arithmetic and an integer multiply.
// The step is bound by its instruction count (one wave, in order: ~160 instructions per step ran the
// 5-point sweep at ~630 cycles per step), so everything the step does not need per lane is scalar: the
// ring row, the wait test on the band above (a step limit), the index prefetch (a buffer load with a
// scalar offset). The solver's waits are scalar LDS spins. Padding entries (value 0, code 0 = the lane's
// own column of the current row: finite) add exactly +-0 to the fma chain. Per-row arithmetic is the
// band kernels': fma over the entries in stored order from 0.0, then (b - acc) / diag — bit-identical.
// DICT: the records come from a dictionary (TriFactor::grid_dict_n): per lane-step ONE 32-bit index
// load instead of the three record loads (codes, values, diagonal), the dictionary in LDS as one
// 64/128-B record per entry (values, diagonal, RN(1/diagonal), ring offsets), the next step's record
// looked up while the current step's ring reads are in flight.
constexpr int kGridRW = 72;                          // ring columns: 8 for the band above + 64 lanes
constexpr int kGridRing = 128;                       // ring rows (steps); the LDS holds 2 x 128 (mirror)
constexpr uint32_t kGridMirror = kGridRing * kGridRW * 8;   // bytes between a row and its mirror
template <int K>
struct GridDict {   // LDS record of a dictionary entry
    static constexpr int kBytes = K == 8 ? 128 : 64;
    // [0, 8K) values, [8K, 8K + 16) diagonal and RN(1/diagonal), then K uint32 ring offsets
    static constexpr int kDg = 8 * K, kOff = 8 * K + 16;
};
template <int K>
struct GridRec {
    uint32_t off[K];      // byte offset of each entry's ring word from the step's lane base
    double cf[K], d, rd;  // rd = RN(1 / d), DICT only
};
// ring byte offset of a dependency coded ud*64 + yd, from the lane base (lower copy of the current row,
// column 8 + j): the upper copy of row s - ud, column 8 + j - yd
__device__ __forceinline__ uint32_t grid_ring_off(uint32_t c) {
    return (uint32_t)(kGridRing - (int)(c >> 6)) * (kGridRW * 8) - (c & 63) * 8;
}
// the skewed step of line y's first position: g(y) = (sigma2 * y + phase) >> 1 (sigma2 = twice the skew)
__host__ __device__ __forceinline__ int64_t grid_g(int64_t sigma2, int64_t phase, int64_t y) {
    return (sigma2 * y + phase) >> 1;
}
// (b - acc) / d on the solver's dependency chain without the IEEE division sequence (two
// dependent scale steps, the reciprocal, five fmas and the fix-up): q0 = RN(r * rd) from the
// correctly rounded reciprocal rd = RN(1/d) (computed once per dictionary entry, off the chain), then
// two Markstein corrections q <- RN(q + RN(r - q d) rd) with the remainder exact in an fma. With rd
// correctly rounded, a correction from any q within one ulp of r/d returns RN(r/d), and q0 is within
// 1.5 ulp, so the second correction returns the IEEE quotient; r = +-0 keeps q0 (the signed zero).
// tools/markstein_check.c: 0 mismatches against r / d in 2e8 random pairs after ONE correction.
// Exactness needs 1/d, r/d and the remainder normal: the host keeps the dictionary only for
// diagonals 2^-100 <= |d| <= 2^100, and a right-hand side r must be zero or inside [2^-900, 2^901)
// (biased exponent in [123, 1923]; tools/markstein_check.c covers both ends of the range and the
// zero/subnormal/infinite edges). The range test is NOT on the dependency chain: each lane ORs it into
// a flag (integer work on r's exponent beside the correction chain), the launch reports it at its end,
// and a conditional pass re-solves the factor with the IEEE division when any step was out of range
// (never, for a stencil solve) — the result is then that pass's, bit for bit the IEEE one. (A
// per-step branch around the IEEE division, round 4's first guard, put 22 instructions and two
// branches on every step: +13% per sweep.)
// The test: frexp's exponent (r = f 2^ex, 0.5 <= |f| < 1; 0 for zero, inf and NaN) in [-899, 901],
// and r not inf / NaN (a class test) — two VALU compares beside the chain, OR-ed into a scalar mask.
__device__ __forceinline__ double div_markstein(double r, double d, double rd, uint64_t &out_of_range) {
    const double q0 = r * rd;
    const double q1 = fma(fma(-q0, d, r), rd, q0);
    const double q2 = fma(fma(-q1, d, r), rd, q1);
    const int ex = __builtin_amdgcn_frexp_exp(r);
    out_of_range |= __builtin_amdgcn_ballot_w64((uint32_t)(ex + 899) > 1800u);
    out_of_range |= __builtin_amdgcn_ballot_w64(__builtin_amdgcn_class(r, 0x207));   // s/qNaN, -inf, +inf
    return r == 0.0 ? q0 : q2;
}
// Buffer (bounds-checked) access for the solver wave's rhs loads and x stores: an out-of-range
// offset loads 0 / drops the store in hardware, so every lane issues every load and store with no
// branch around it. The compiler's vmcnt waits count only memory operations it knows were issued:
// with the rhs load and the two x stores under divergent branches it assumed one operation per step
// (the record index) and waited with vmcnt(10) — i.e. for stores and loads issued ~3 steps before,
// write-through stores included — where the prefetch runs D steps ahead. Byte offsets are 32-bit:
// the grid schedule takes factors of at most kGridMaxRows rows (host check).
constexpr uint32_t kBufOOB = 0xFFFFFFFFu;
constexpr int64_t kGridMaxRows = (int64_t)1 << 29;
typedef unsigned int grid_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t grid_rsrc(const double *p, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), (short)0, (int)(uint32_t)(n * 8), 0x00020000);
}
__device__ __forceinline__ double grid_bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <int CPOL>   // 0x10: sc1 (agent-scope write-through, the publication store), 0: plain
__device__ __forceinline__ void grid_bstore(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(grid_u2, v), r, off, 0, CPOL);
}

// MK (DICT only): Markstein quotient, range flag OR-ed into *rflag at the end (see div_markstein); !MK:
// IEEE division. gate != nullptr: the conditional re-solve, a no-op unless *gate is set.
template <int K, int D, bool DICT, bool MK>
__global__ __launch_bounds__(2 * kGridLanes) void sptrsv_grid_kernel(
    int64_t n, int64_t w, int64_t H, int64_t sigma2, int64_t phase, int64_t off, int64_t S_full, int upper, int pe,
    int maxyd,
    int unit, const double *__restrict__ rhs, double *x, int32_t *err, const double *__restrict__ grec,
    GridExt ext, const uint32_t *__restrict__ gidx, const double *__restrict__ gdict, int ndict, int32_t *rflag,
    const int32_t *gate, uint32_t *sched) {
    if (gate && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;   // uniform
    extern __shared__ __align__(16) unsigned char smem[];
    // the bands this workgroup solves: drawn one after the other from the ticket counter (band b waits only on
    // band b - 1, drawn earlier by a running workgroup; sched_next_block) until they run out. A workgroup
    // that finishes its band takes the next one itself: the launch never needs a workgroup that has not
    // started (round 5: with one band per workgroup, a launch beside a kernel holding most CUs stalled —
    // the dispatcher did not start its later workgroups on the CUs its finished ones freed, tests/
    // test_gpu_progress.py, profiles/r5_progress_probe.txt)
    __shared__ int64_t s_band;
    double *ring = reinterpret_cast<double *>(smem);                  // [2 * kGridRing][kGridRW]
    int64_t *ctl = reinterpret_cast<int64_t *>(smem + 2 * kGridMirror);
    unsigned char *dict = smem + 2 * kGridMirror + 16;                // DICT: ndict GridDict<K> records
    // gdict (host layout): [ndict][K] values, [ndict] diagonals, [ndict][K/2] code words
    if (DICT) {
        const uint32_t *gcode = reinterpret_cast<const uint32_t *>(gdict + (size_t)ndict * (K + 1));
        for (int i = threadIdx.x; i < ndict; i += 2 * kGridLanes) {
            unsigned char *rec = dict + (size_t)i * GridDict<K>::kBytes;
            double *cf = reinterpret_cast<double *>(rec);
            for (int k = 0; k < K; ++k) cf[k] = gdict[(size_t)i * K + k];
            const double dg = gdict[(size_t)ndict * K + i];
            reinterpret_cast<double *>(rec + GridDict<K>::kDg)[0] = dg;
            reinterpret_cast<double *>(rec + GridDict<K>::kDg)[1] = 1.0 / dg;
            uint32_t *ro = reinterpret_cast<uint32_t *>(rec + GridDict<K>::kOff);
            for (int k = 0; k < K; ++k) ro[k] = grid_ring_off((gcode[(size_t)i * (K / 2) + k / 2] >> (16 * (k & 1))) & 0xffff);
        }
    }
    const int64_t nbands = (H + kGridLanes - 1) / kGridLanes;
    auto run_band = [&](const int64_t band) {
        // ctl[0]: last u of the band above present in the ring (poller -> solver)
        // ctl[1]: last u the solver has finished (solver -> poller, ring capacity)
        const int tid = threadIdx.x, j = tid & 63;
        const int64_t y0 = band * kGridLanes;
        const int64_t ylast = (y0 + kGridLanes - 1 < H - 1) ? y0 + kGridLanes - 1 : H - 1;
        const int64_t u_lo = grid_g(sigma2, phase, y0), u_hi = (w - 1) + grid_g(sigma2, phase, ylast);
        const int S = (int)(u_hi - u_lo + 1);
        int min_ud = 1 << 30, max_ud = 0;
        for (int e = 0; e < pe; ++e) {
            const int ud = ext.delta[e] >> 6;
            min_ud = ud < min_ud ? ud : min_ud;
            max_ud = ud > max_ud ? ud : max_ud;
        }
        const bool has_ext = band > 0 && pe > 0;
        for (int i = tid; i < 2 * kGridRing * kGridRW; i += 2 * kGridLanes) ring[i] = 0.0;
        if (tid == 0) {
            ctl[0] = has_ext ? u_lo - max_ud - 1 : INT64_MAX / 2;
            ctl[1] = u_lo - 1;
        }
        __syncthreads();
    #ifdef PSK_GRID_PROF
        const unsigned long long t_start = __builtin_amdgcn_s_memtime();
        const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
        unsigned long long n_wait = 0, c_wait = 0;
    #endif
        if (tid >= kGridLanes) {
            // ---------------- poller: u positions [u_lo - max_ud, u_hi - min_ud] of lines y0-maxyd .. y0-1
            if (!has_ext) return;
            const int64_t ua = u_lo - max_ud, ub = u_hi - min_ud;
            for (int64_t base = ua; base <= ub; base += kGridLanes) {
                const int64_t u = base + j;
                double *row_lo = ring + (size_t)((u - u_lo) & (kGridRing - 1)) * kGridRW + (8 - maxyd);
                double *row_hi = row_lo + kGridRing * kGridRW;
                // ring capacity: row (u - u_lo) last held u - kGridRing, which the solver reads until it passes
                // that position + max_ud
                int64_t spins = 0;
                while (__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
                       base + kGridLanes - 1 - kGridRing + max_ud) {
                    if (++spins > kMaxSpins) { atomicExch(err, (2 << 24) | (int)band); return; }
                    __builtin_amdgcn_s_sleep(2);
                }
                uint32_t pending = 0;   // lines of this lane's u still to fetch
                for (int L = 0; L < maxyd; ++L) {
                    const int64_t yl = y0 - maxyd + L, xl = u - grid_g(sigma2, phase, yl), q = yl * w + xl - off;
                    const bool valid = u <= ub && yl >= 0 && xl >= 0 && xl < w && q >= 0 && q < n;
                    if (valid) {
                        pending |= 1u << L;
                    } else {
                        row_lo[L] = 0.0;
                        row_hi[L] = 0.0;
                    }
                }
                spins = 0;
                while (true) {
                    for (int L = 0; L < maxyd; ++L)
                        if (pending & (1u << L)) {
                            const int64_t yl = y0 - maxyd + L, q = yl * w + (u - grid_g(sigma2, phase, yl)) - off;
                            const double v = load_pub(x + (upper ? n - 1 - q : q));
                            if (!is_sentinel(v)) {
                                row_lo[L] = v;
                                row_hi[L] = v;
                                pending &= ~(1u << L);
                            }
                        }
                    // ready prefix of this chunk: lanes 0..r-1 have every line
                    const uint64_t notready = __ballot(pending != 0);
                    const int r = notready ? __builtin_ctzll(notready) : kGridLanes;
                    __builtin_amdgcn_s_waitcnt(0xc07f);   // ring writes before the announcement
                    if (j == 0 && r > 0)
                        __hip_atomic_store(&ctl[0], base + r - 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (!notready) break;
                    if (++spins > kMaxSpins) { atomicExch(err, (3 << 24) | (int)band); return; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            return;
        }
        // ---------------- solver
        const int64_t y = y0 + j;
        // lane j's line holds grid positions [y*w, y*w + w) of [off, n + off) (the first `off` positions of
        // the first line are empty: a partial line leading the solve order); it is active for steps
        // [s_beg, s_end): x = s - gy in [x_lo, x_hi), gy = g(y) - g(y0) (the line's first step in the band)
        const int64_t x_lo = y * w < off ? off - y * w : 0;
        const int64_t x_hi = n + off - y * w < w ? n + off - y * w : w;
        const bool live = y < H && x_hi > x_lo;
        const int64_t gy = grid_g(sigma2, phase, y) - u_lo;
        const int s_beg = (int)(gy + (live ? x_lo : 0)), s_end = live ? (int)(gy + x_hi) : s_beg;
        const uint32_t s_len = (uint32_t)(s_end - s_beg);
        // byte offset of step s's row: rb8 + rs8 * s (32-bit: n <= kGridMaxRows; step indices < 2^23, so a
        // 24-bit multiply), q = y*w + s - gy - off; a line-less lane reads out of range (loads 0)
        const int64_t qb = y * w - gy - off;
        const uint32_t rb8 = live ? (uint32_t)((upper ? n - 1 - qb : qb) * 8) : kBufOOB - 8;
        const int32_t rs8 = live ? (upper ? -8 : 8) : 0;
        const bool pub = j >= kGridLanes - maxyd;   // the lines the band below reads: agent-scope stores
        const uint32_t lane8 = (uint32_t)(8 + j) * 8;
        const unsigned char *pstep = reinterpret_cast<const unsigned char *>(grec) +
                                     band * S_full * GridStep<K>::kBytes;
        // the index stream of this band: a buffer with the step in the scalar offset
        const __amdgpu_buffer_rsrc_t ridx = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(DICT ? gidx + band * S_full * kGridLanes : gidx), (short)0,
            DICT ? (int)(uint32_t)(S_full * kGridLanes * 4) : 0, 0x00020000);
        const __amdgpu_buffer_rsrc_t rrhs = grid_rsrc(rhs, n), rx = grid_rsrc(x, n);
        // steps up to s_ok need nothing more from the band above (uniform)
        int s_ok = has_ext ? -max_ud - 1 + min_ud : INT32_MAX / 2;
        uint64_t rbad = 0;   // MK: lanes with a step's right-hand side outside the Markstein range (div_markstein)
        struct Slot {
            uint32_t idx;   // DICT: the record index
            uint32_t code[K / 2];
            double cf[K], d, b;
        };
        auto fetch = [&](int s, Slot &sl) {
            const int sc = s < S ? s : S - 1;   // past the end: re-read the last step (unused)
            const int sa = __builtin_elementwise_max(__builtin_elementwise_min(s, s_end - 1), s_beg);
            sl.b = grid_bload(rrhs, rb8 + (uint32_t)__mul24(rs8, sa));
            if (DICT) {
                sl.idx = __builtin_amdgcn_raw_buffer_load_b32(ridx, (uint32_t)j * 4, (uint32_t)sc * (kGridLanes * 4), 0);
                return;
            }
            const unsigned char *st = pstep + (int64_t)sc * GridStep<K>::kBytes;
            const uint32_t *pc = reinterpret_cast<const uint32_t *>(st + GridStep<K>::kCode) + j * (K / 2);
    #pragma unroll
            for (int k = 0; k < K / 2; ++k) sl.code[k] = pc[k];
            const dv2 *pf = reinterpret_cast<const dv2 *>(st + GridStep<K>::kCoef) + j * (K / 2);
    #pragma unroll
            for (int k = 0; k < K; k += 2) {
                const dv2 c = pf[k / 2];
                sl.cf[k] = c.x;
                sl.cf[k + 1] = c.y;
            }
            sl.d = reinterpret_cast<const double *>(st + GridStep<K>::kDiag)[j];
        };
        auto lookup = [&](uint32_t idx, GridRec<K> &rc) {   // DICT: the record of a step, from LDS
            const unsigned char *rec = dict + idx * GridDict<K>::kBytes;
    #pragma unroll
            for (int k = 0; k < K; k += 2) {
                const dv2 c = *reinterpret_cast<const dv2 *>(rec + 8 * k);
                rc.cf[k] = c.x;
                rc.cf[k + 1] = c.y;
            }
            const dv2 dd = *reinterpret_cast<const dv2 *>(rec + GridDict<K>::kDg);
            rc.d = dd.x;
            rc.rd = dd.y;
    #pragma unroll
            for (int k = 0; k < K; ++k) rc.off[k] = reinterpret_cast<const uint32_t *>(rec + GridDict<K>::kOff)[k];
        };
        // the ring values of step t are requested right after step t-1's ring write (one wave: the LDS
        // queue is in order, so they see it), and the step's other work — the x stores, the prefetch D
        // steps ahead, the dictionary lookup two steps ahead — runs while they are in flight: the chain
        // per step is the LDS round trip and the arithmetic, not the step's whole instruction stream
        auto wait_ext = [&](int t) {
            if (t > s_ok && t < S) {   // uniform: the band above not yet in the ring
    #ifdef PSK_GRID_PROF
                const unsigned long long tw = __builtin_amdgcn_s_memtime();
    #endif
                int64_t spins = 0;
                do {
                    const int known = __builtin_amdgcn_readfirstlane(
                        (int)(__hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) - u_lo));
                    s_ok = known + min_ud;   // ext_known >= u - min_ud  <=>  t <= known + min_ud
                    if (t <= s_ok) break;
                    if (++spins > kMaxSpins) { atomicExch(err, (1 << 24) | (int)band); break; }
                    __builtin_amdgcn_s_sleep(1);
                } while (true);
    #ifdef PSK_GRID_PROF
                n_wait += 1;
                c_wait += __builtin_amdgcn_s_memtime() - tw;
    #endif
            }
        };
        auto request = [&](int t, const Slot &sl, const GridRec<K> &rec, double *v) {
            const uint32_t base = lane8 + (uint32_t)(t & (kGridRing - 1)) * (kGridRW * 8);   // lower copy, row t
    #pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t ro = DICT ? rec.off[k] : grid_ring_off((sl.code[k >> 1] >> (16 * (k & 1))) & 0xffff);
                v[k] = *reinterpret_cast<const double *>(smem + base + ro);
            }
        };
        auto solve = [&](int s, const Slot &sl, const GridRec<K> &rec, const double *v) -> double {
            double acc = 0.0;
    #pragma unroll
            for (int k = 0; k < K; ++k) acc = fma(DICT ? rec.cf[k] : sl.cf[k], v[k], acc);   // stored order; padding adds +-0
            double r = sl.b - acc;
            const double d = DICT ? rec.d : sl.d;
            if (DICT && MK) {   // a select, not a branch, on `unit` (the chain stays branch-free)
                const double q = div_markstein(r, d, rec.rd, rbad);
                r = unit ? r : q;
            } else if (!unit) {
                r = r / d;
            }
            // both copies of the row (the mirror is kGridMirror bytes above)
            const uint32_t base = lane8 + (uint32_t)(s & (kGridRing - 1)) * (kGridRW * 8);
            *reinterpret_cast<double *>(smem + base) = r;
            *reinterpret_cast<double *>(smem + base + kGridMirror) = r;
            return r;
        };
        auto store_x = [&](int s, double r) {   // the lines the band below reads are published
            const bool act = (uint32_t)(s - s_beg) < s_len;
            const uint32_t o = rb8 + (uint32_t)__mul24(rs8, s);
            grid_bstore<0x10>(rx, act && pub ? o : kBufOOB, r);
            grid_bstore<0>(rx, act && !pub ? o : kBufOOB, r);
        };
        static_assert(D >= 3 && D % 2 == 0, "the lookup runs two steps ahead; step parity = slot parity");
        Slot buf[D];
    #pragma unroll
        for (int i = 0; i < D; ++i) fetch(i, buf[i]);
        GridRec<K> rq[2] = {};   // DICT: rq[t & 1] = the record of step t
        if (DICT) {
            lookup(buf[0].idx, rq[0]);
            lookup(buf[1].idx, rq[1]);
        }
        double vn[K];
        wait_ext(0);
        request(0, buf[0], rq[0], vn);
        for (int s0 = 0; s0 < S; s0 += D) {   // D even: step s0 + i has the parity of i
    #pragma unroll
            for (int i = 0; i < D; ++i) {
                const int s = s0 + i;
                const double r = solve(s, buf[i], rq[i & 1], vn);
                __asm__ volatile("" ::: "memory");   // the ring write before the next step's reads
                wait_ext(s + 1);
                request(s + 1, buf[(i + 1) % D], rq[(i + 1) & 1], vn);
                store_x(s, r);
                __asm__ volatile("" ::: "memory");
                fetch(s + D, buf[i]);
                if (DICT) lookup(buf[(i + 2) % D].idx, rq[i & 1]);   // step s + 2's record
                // issued HERE: left to itself the machine scheduler sank the lookup into the next step,
                // next to the ring reads that need it (two LDS round trips on the chain)
                __builtin_amdgcn_sched_barrier(0);
            }
            if (j == 0)   // progress for the poller's ring capacity
                __hip_atomic_store(&ctl[1], u_lo + s0 + D - 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (j == 0) __hip_atomic_store(&ctl[1], INT64_MAX / 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (MK && !unit && rbad != 0 && j == 0) atomicOr(rflag, 1);
    #ifdef PSK_GRID_PROF
        if (j == 0 && band < 8192) {
            g_grid_prof[band * 8 + 0] = t_start;
            g_grid_prof[band * 8 + 1] = __builtin_amdgcn_s_memtime();
            g_grid_prof[band * 8 + 2] = n_wait;
            g_grid_prof[band * 8 + 3] = c_wait;
            g_grid_prof[band * 8 + 4] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;   // XCD
            g_grid_prof[band * 8 + 5] = blockIdx.x;
            g_grid_prof[band * 8 + 6] = rt_start;                                       // 100 MHz, device-wide
            g_grid_prof[band * 8 + 7] = __builtin_amdgcn_s_memrealtime();
        }
    #endif
    };
    for (;;) {
        __syncthreads();   // the previous band's waves are done with the ring (and the dictionary is in LDS)
        if (threadIdx.x == 0) s_band = sched_next_block(sched, nbands);
        __syncthreads();
        const int64_t band = s_band;
        if (band >= nbands) break;
        run_band(band);
    }
}

// ---- levels schedule (round 5): one workgroup, level-synchronous, x in LDS slots ---------------------------
// For factors with few rows per dependency level (the SA level-1 operator of -FD 8192^2: 131k rows, 1706
// levels of <= 109 rows): step s solves lane t's row of one level (a level wider than the workgroup takes
// several steps), reading its dependencies from LDS, then a barrier. A hop between levels is an LDS round
// trip plus a barrier instead of a device-scope publication seen by a polling load (sync-free, ~1 us per
// level). Each value lives in an LDS slot the host assigned it (interval allocation: a slot is reused only
// in a step after its last reader), so dependencies any number of levels back are fine as long as the
// values alive at once fit the LDS. Records are field-major per step, loaded D steps ahead into registers;
// the barrier waits for LDS only (lgkmcnt), so those loads stay in flight across it. Per-row arithmetic:
// fma over the stored entries in stored order from 0.0, padding entries (-0.0 x 0.0) add exactly nothing,
// then (b - acc) / d: the band and grid kernels' bits.
constexpr uint32_t kLevelIdle = 0xFFFFFFFFu;   // row field of an idle lane
constexpr int kLevelMaxK = 16, kLevelMaxW = 256, kLevelD = 4, kLevelPad = 8;   // D: steps loaded ahead (PSK_LEVELS_D=8: lab)
constexpr int64_t kLevelMaxSlots = 18432;     // live values + the zero and trash slots: <= 144 KiB of LDS
template <int KM, int D>
__global__ __launch_bounds__(256) void sptrsv_levels_kernel(int64_t nsteps, int R, int64_t n, int unit,
                                                            const uint64_t *__restrict__ rc,
                                                            const uint64_t *__restrict__ sl,
                                                            const double *__restrict__ cf,
                                                            const double *__restrict__ dg,
                                                            const double *__restrict__ bp, double *__restrict__ x) {
    static_assert(KM % 4 == 0, "slots are loaded four per 8-byte word, coefficients two per 16-byte load");
    extern __shared__ double lv_ring[];   // R + 2 slots: R live values, R = 0.0 (padding), R + 1 = trash
    const int t = threadIdx.x, W = blockDim.x;
    for (int i = t; i <= R + 1; i += W) lv_ring[i] = 0.0;
    __syncthreads();
    struct Rec {
        uint64_t rc;
        uint64_t sw[KM / 4];
        double c[KM];
        double d, b;
    };
    (void)R;
    // every load is unconditional, branch-free and independent of the others (an address computed from a
    // loaded count would make the wave wait for that load at once; a predicated load becomes a branch,
    // after which the compiler waits for ALL outstanding loads): entries past a row's count are stored
    // padding (slot R, coefficient -0.0), the diagonal is stored as 1.0 for a unit factor
    const __amdgpu_buffer_rsrc_t rrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(rc), (short)0,
                                                                         (int)(uint32_t)(nsteps * W * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t *>(sl), (short)0,
                                                                         (int)(uint32_t)(nsteps * W * (KM / 4) * 8),
                                                                         0x00020000);
    const __amdgpu_buffer_rsrc_t rcf = grid_rsrc(cf, nsteps * W * KM), rdg = grid_rsrc(dg, nsteps * W),
                                 rbp = grid_rsrc(bp, nsteps * W), rx = grid_rsrc(x, n);
    auto fetch = [&](int64_t s, Rec &r) {
        const uint32_t sc = (uint32_t)(s < nsteps ? s : nsteps - 1);   // past the end: the last step (unused)
        const uint32_t p = sc * (uint32_t)W + (uint32_t)t;
        r.rc = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rrc, p * 8, 0, 0));
        r.d = grid_bload(rdg, p * 8);
        r.b = grid_bload(rbp, p * 8);
#pragma unroll
        for (int k4 = 0; k4 < KM / 4; ++k4)
            r.sw[k4] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                                        rsl, ((sc * (KM / 4) + k4) * (uint32_t)W + (uint32_t)t) * 8, 0, 0));
#pragma unroll
        for (int k2 = 0; k2 < KM / 2; ++k2) {
            const auto v4 = __builtin_amdgcn_raw_buffer_load_b128(rcf, ((sc * (KM / 2) + k2) * (uint32_t)W + (uint32_t)t) * 16,
                                                                  0, 0);
            r.c[2 * k2] = __longlong_as_double((long long)((uint64_t)v4[0] | ((uint64_t)v4[1] << 32)));
            r.c[2 * k2 + 1] = __longlong_as_double((long long)((uint64_t)v4[2] | ((uint64_t)v4[3] << 32)));
        }
    };
    // The loop starts D steps early with zeroed records (idle: nothing stored), so that every record load
    // is issued inside the loop: loads issued before it (a prologue) would be merged into the loop
    // header's wait state and make the compiler wait for ALL loads at every iteration.
    Rec buf[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        buf[i].rc = (uint64_t)kLevelIdle | ((uint64_t)(R + 1) << 40);
#pragma unroll
        for (int k4 = 0; k4 < KM / 4; ++k4) buf[i].sw[k4] = 0;
#pragma unroll
        for (int k = 0; k < KM; ++k) buf[i].c[k] = 0.0;
        buf[i].d = 1.0;
        buf[i].b = 0.0;
    }
    for (int64_t s0 = -D; s0 < nsteps; s0 += D) {   // nsteps: a multiple of D (the host pads idle steps)
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int64_t s = s0 + i;
            double acc = 0.0;
            // every entry slot, padding included (-0.0 x 0.0 adds nothing): cutting the chain at the step's
            // widest row with a uniform branch per entry measured slower (0.93 vs 0.62 ms on AMG level 1:
            // the LDS reads no longer all go out before the first fma)
#pragma unroll
            for (int k = 0; k < KM; ++k) {
                const uint32_t slot = (uint32_t)(buf[i].sw[k >> 2] >> (16 * (k & 3))) & 0xFFFFu;
                acc = fma(buf[i].c[k], lv_ring[slot], acc);
            }
            double r = buf[i].b - acc;
            if (!unit) r = r / buf[i].d;   // (uniform)
            lv_ring[(uint32_t)(buf[i].rc >> 40) & 0xFFFFu] = r;
            const uint32_t row = (uint32_t)buf[i].rc;
            grid_bstore<0>(rx, row != kLevelIdle ? row * 8u : kBufOOB, r);   // idle lanes: out of range, dropped
            fetch(s + D, buf[i]);
            // the step's ring writes before the next step's reads (LDS-only fences: the prefetch loads stay
            // in flight across the barrier)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        }
    }
}

// right-hand side into step order: bp[p] = rhs[idx ? idx[row] : row] (0 on idle lanes)
__global__ void levels_gather_kernel(int64_t np, const uint64_t *__restrict__ rc, const double *__restrict__ rhs,
                                     const int32_t *__restrict__ idx, double *__restrict__ bp) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const uint32_t row = (uint32_t)rc[p];
    bp[p] = row == kLevelIdle ? 0.0 : rhs[idx ? idx[row] : row];
}

// x = sentinel on the rows the grid schedule publishes — lines y with y mod 64 >= 64 - maxyd, the ones
// the band below polls (every other row is read only after the launch): maxyd/64 of the vector instead
// of all of it. gate != nullptr: only when *gate is set (before the conditional re-solve).
__global__ void grid_fill_published_kernel(int64_t n, int64_t w, int64_t H, int64_t off, int maxyd, int upper,
                                           double *x, const int32_t *gate) {
    if (gate && __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    const int64_t total = ((H + kGridLanes - 1) / kGridLanes) * maxyd * w;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t li = t / w, xx = t - li * w;
        const int64_t y = (li / maxyd) * kGridLanes + (kGridLanes - maxyd) + li % maxyd, q = y * w + xx - off;
        if (y < H && q >= 0 && q < n) reinterpret_cast<uint64_t *>(x)[upper ? n - 1 - q : q] = kSentinel;
    }
}
__global__ void grid_flag_reset_kernel(int32_t *flag) { *flag = 0; }

static size_t grid_lds_bytes(int K, int ndict) {   // mirrored ring, ctl, dictionary records
    const size_t rec = K == 8 ? GridDict<8>::kBytes : K == 4 ? GridDict<4>::kBytes : GridDict<2>::kBytes;
    return 2 * (size_t)kGridMirror + 2 * sizeof(int64_t) + (ndict > 0 ? (size_t)ndict * rec : 0);
}

static size_t narrow_lds_bytes(int ring_words, int K) {
    return (size_t)ring_words * sizeof(double) +
           (size_t)kNarrowBufs * kNarrowChunk * ((2 * K + 2) * sizeof(double) + (K + 2) * sizeof(int32_t)) +
           (kNarrowBufs + 2) * sizeof(int32_t);
}

// out[i] = z[perm[i]] (perm == nullptr: copy)
__global__ void gather_perm_kernel(int64_t n, const double *__restrict__ z, const int32_t *__restrict__ perm,
                                   double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = perm ? z[perm[i]] : z[i];
}

// x[i] = x[i] + z[perm[i]]: the last gather fused with the smoother's x + dx (ClassicSmoothers.py:34),
// the same single rounding as gathering into a temporary and adding it (24 instead of 40 B/row)
__global__ void gather_add_kernel(int64_t n, const double *__restrict__ z, const int32_t *__restrict__ perm,
                                  double *__restrict__ x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] + (perm ? z[perm[i]] : z[i]);
}

static size_t band_lds_bytes(int ring_words, int K) {
    return (size_t)ring_words * sizeof(double) +
           2 * (size_t)kBandChunk * ((2 * K + 2) * sizeof(double) + (K + 2) * sizeof(int32_t));
}

static int coop_grid(const Context *c, const void *kern, size_t lds) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds) != hipSuccess) per_cu = 1;
    if (per_cu > 2) per_cu = 2;   // margin below the occupancy answer (MI355X_MICROARCH.md residency)
    if (per_cu < 1) per_cu = 1;
    return c->num_cus * per_cu;
}

// Sync-free grid: every resident slot the occupancy API reports minus one workgroup per CU (the
// hardware admits one fewer than the API at some SGPR counts, MI355X_MICROARCH.md "Residency"); all
// waves must be co-resident, since a row's wave may wait on any earlier position. The spin-waiting
// schedules (sync-free, band, partitioned) size their grids to fit and launch them plainly: a
// cooperative launch adds nothing they use (no grid barrier), and it left HIP holding per-process
// state whose teardown in exit() faulted under rocprofv3 (profiles/r4_exit_fault.txt). Every wait is
// bounded, so a workgroup that never became resident would surface as a reported error, not a hang.
int syncfree_grid(const Context *c) {
    static int per_cu = -1;
    if (per_cu < 0) {
        int api = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, reinterpret_cast<const void *>(&sptrsv_kernel), kBlock,
                                                         0) != hipSuccess)
            api = 2;
        per_cu = std::max(1, std::min(api, 8) - 1);
    }
    return c->num_cus * per_cu;
}

static unsigned grid_fill_blocks(const TriFactor &T) {
    const int64_t total = ((T.grid_H + kGridLanes - 1) / kGridLanes) * T.grid_maxyd * T.grid_w;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((total + kBlock - 1) / kBlock, 4096));
}

// the output of one factor before its solve: the sentinel where the schedule's waits read it (the grid
// schedule: only its published lines; every other schedule: every row)
static int fill_factor_output(const TriFactor &T, int64_t n, double *x, hipStream_t s) {
    if (T.schedule == kSchedLevel) return PSK_OK;   // nothing polls: one workgroup, dependencies through LDS
    if (T.schedule == kSchedGrid) {
        if (T.grid_pe == 0 || T.grid_maxyd == 0) return PSK_OK;   // no band waits on another
        hipLaunchKernelGGL(grid_fill_published_kernel, dim3(grid_fill_blocks(T)), dim3(kBlock), 0, s, n, T.grid_w,
                           T.grid_H, T.grid_off, T.grid_maxyd, T.upper ? 1 : 0, x, nullptr);
    } else {
        hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, x);
    }
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

// x = T^-1 rhs[rhs_idx] for one factor, with the factor's schedule
static int launch_factor(const Context *c, int64_t n, const TriFactor &T, const double *rhs, const int32_t *rhs_idx,
                         double *x, int32_t *err, hipStream_t s) {
    int64_t nn = n;
    const int32_t *rp = T.rowptr, *ci = T.colidx;
    const double *va = T.vals, *dg = T.diag;
    (void)rp;
    if (T.schedule == kSchedLds) {
        constexpr int depth = kLdsDepth;
        const void *k = depth <= 1   ? reinterpret_cast<const void *>(&sptrsv_lds_kernel<1>)
                        : depth == 2 ? reinterpret_cast<const void *>(&sptrsv_lds_kernel<2>)
                                     : reinterpret_cast<const void *>(&sptrsv_lds_kernel<3>);   // 4 spills
        const int32_t *ord = T.order;
        void *args[] = {&nn, &rp, &ci, &va, &dg, &rhs, &rhs_idx, &x, &err, &ord};
        PSK_HIP(hipLaunchKernel(k, dim3(1), dim3(kLdsThreads), args, (size_t)n * sizeof(double), s));
        return PSK_OK;
    }
    if (T.schedule == kSchedLevel) {
        int64_t ns = T.lv_steps;
        const int64_t np = ns * T.lv_W;
        hipLaunchKernelGGL(levels_gather_kernel, dim3((unsigned)((np + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, np,
                           T.lv_rc, rhs, rhs_idx, T.lv_b);
        PSK_HIP(hipGetLastError());
        constexpr bool d8 = false;   // 8 steps of prefetch: measured no faster than 4 (round 5)
        const void *k = d8 ? (T.lv_KM == 4    ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<4, 8>)
                              : T.lv_KM == 8  ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<8, 8>)
                              : T.lv_KM == 12 ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<12, 8>)
                                              : reinterpret_cast<const void *>(&sptrsv_levels_kernel<16, 8>))
                           : (T.lv_KM == 4    ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<4, kLevelD>)
                              : T.lv_KM == 8  ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<8, kLevelD>)
                              : T.lv_KM == 12 ? reinterpret_cast<const void *>(&sptrsv_levels_kernel<12, kLevelD>)
                                              : reinterpret_cast<const void *>(&sptrsv_levels_kernel<16, kLevelD>));
        int R = T.lv_R, unit = T.diag ? 0 : 1;
        const uint64_t *lrc = T.lv_rc;
        const uint64_t *lsl = T.lv_sl;
        const double *lcf = T.lv_cf, *ldg = T.lv_dg, *lb = T.lv_b;
        void *args[] = {&ns, &R, &nn, &unit, &lrc, &lsl, &lcf, &ldg, &lb, &x};
        PSK_HIP(hipLaunchKernel(k, dim3(1), dim3(T.lv_W), args, (size_t)(R + 2) * sizeof(double), s));
        return PSK_OK;
    }
    if (T.schedule == kSchedPart) {
        if (rhs_idx) return fail(PSK_ERR_ARG, "part schedule: gathered right-hand side (internal)");
        const void *k = dg ? reinterpret_cast<const void *>(&sptrsv_part_kernel<false>)
                           : reinterpret_cast<const void *>(&sptrsv_part_kernel<true>);
        const int64_t *sg = T.part_seg;
        const int32_t *prp = T.part_rp, *pc = T.part_code, *prow = T.part_row;
        const double *pv = T.part_va;
        void *args[] = {&sg, &prp, &pc, &pv, &dg, &rhs, &x, &err, &prow};
        PSK_HIP(hipLaunchKernel(k, dim3(T.part_P), dim3(kPartThreads), args, (unsigned)kPartLds, s));
        return PSK_OK;
    }
    if (T.schedule == kSchedGrid) {
        if (rhs_idx) return fail(PSK_ERR_ARG, "grid schedule: gathered right-hand side (internal)");
        const void *k = nullptr, *kf = nullptr;
#ifndef PSK_GRID_D
#define PSK_GRID_D 12
#endif
#ifndef PSK_GRID_DD   // prefetch depth with the record dictionary (a step's slot: index + rhs)
#define PSK_GRID_DD PSK_GRID_D
#endif
        const bool dict = T.grid_dict_n > 0;
#define PSK_GRID_K(KK, DN)                                                                                    \
    do {                                                                                                      \
        k = dict ? reinterpret_cast<const void *>(&sptrsv_grid_kernel<KK, PSK_GRID_DD, true, true>)            \
                 : reinterpret_cast<const void *>(&sptrsv_grid_kernel<KK, DN, false, false>);                  \
        kf = reinterpret_cast<const void *>(&sptrsv_grid_kernel<KK, PSK_GRID_DD, true, false>);                \
    } while (0)
        if (T.grid_K == 2) PSK_GRID_K(2, PSK_GRID_D);
        else if (T.grid_K == 4) PSK_GRID_K(4, (PSK_GRID_D > 8 ? 8 : PSK_GRID_D));
        else if (T.grid_K == 8) PSK_GRID_K(8, (PSK_GRID_D > 6 ? 6 : PSK_GRID_D));
#undef PSK_GRID_K
        if (!k) return fail(PSK_ERR_ARG, "grid schedule: bad record width");
        int64_t w = T.grid_w, H = T.grid_H, sg = T.grid_sigma, gph = T.grid_phase, goff = T.grid_off, sfull = T.grid_S;
        int upper = T.upper ? 1 : 0, pe_ = T.grid_pe, myd = T.grid_maxyd;
        int unit = T.diag ? 0 : 1;
        const double *gr = T.gd_coef;
        GridExt ext = T.grid_ext;
        const uint32_t *gi = T.gd_idx;
        const double *gdd = T.gd_dict;
        int nd = T.grid_dict_n;
        int32_t *flag = dict ? T.grid_flag : nullptr;
        const int32_t *nogate = nullptr;
        uint32_t *sch = T.sched;
        void *args[] = {&nn, &w, &H, &sg, &gph, &goff, &sfull, &upper, &pe_, &myd, &unit, &rhs, &x, &err, &gr, &ext, &gi,
                        &gdd, &nd, &flag, &nogate, &sch};
        // one workgroup per band, at most one per CU (a workgroup holds ~147 KiB of LDS); workgroups draw bands
        // until they run out, so fewer workgroups than bands still solve every band
        const unsigned nb = (unsigned)std::min<int64_t>((H + kGridLanes - 1) / kGridLanes, c->num_cus);
        const size_t lds = grid_lds_bytes(T.grid_K, T.grid_dict_n);
        PSK_HIP(hipLaunchKernel(k, dim3(nb), dim3(2 * kGridLanes), args, lds, s));
        if (dict) {   // conditional IEEE re-solve (div_markstein): no-ops unless a step was out of range
            const int32_t *gate = T.grid_flag;
            int32_t *noflag = nullptr;
            if (pe_ > 0 && myd > 0) {
                hipLaunchKernelGGL(grid_fill_published_kernel, dim3(grid_fill_blocks(T)), dim3(kBlock), 0, s, nn, w,
                                   H, goff, myd, upper, x, gate);
                PSK_HIP(hipGetLastError());
            }
            void *fargs[] = {&nn, &w, &H, &sg, &gph, &goff, &sfull, &upper, &pe_, &myd, &unit, &rhs, &x, &err, &gr, &ext,
                             &gi, &gdd, &nd, &noflag, &gate, &sch};
            // one workgroup: a no-op unless the gate is set (then it solves every band itself, a rare path), and
            // a launch that needs no more than one free CU to complete
            PSK_HIP(hipLaunchKernel(kf, dim3(1), dim3(2 * kGridLanes), fargs, lds, s));
            hipLaunchKernelGGL(grid_flag_reset_kernel, dim3(1), dim3(1), 0, s, T.grid_flag);
            PSK_HIP(hipGetLastError());
        }
        return PSK_OK;
    }
    if (T.schedule == kSchedBand && T.band_narrow) {
        const void *k = nullptr;
        switch (T.band_K) {
        case 1: k = reinterpret_cast<const void *>(&sptrsv_band_narrow_kernel<1>); break;
        case 2: k = reinterpret_cast<const void *>(&sptrsv_band_narrow_kernel<2>); break;
        case 4: k = reinterpret_cast<const void *>(&sptrsv_band_narrow_kernel<4>); break;
        case 8: k = reinterpret_cast<const void *>(&sptrsv_band_narrow_kernel<8>); break;
        default: return fail(PSK_ERR_ARG, "band schedule: bad record width");
        }
        const size_t lds = narrow_lds_bytes(T.ring_words, T.band_K);
        const int g = coop_grid(c, k, lds);
        int upper = T.upper ? 1 : 0;
        const int32_t *rr = T.rec_row, *re = T.rec_end, *rc = T.rec_c;
        const double *rv = T.rec_v, *rd = T.diag ? T.rec_d : nullptr;
        int64_t nb = T.band_nblocks, B = T.band_B;
        int mask = T.ring_words - 1;
        uint32_t *sch = T.sched;
        void *args[] = {&nn, &upper, &rhs, &rhs_idx, &x, &err, &rr, &re, &rc, &rv, &rd, &nb, &B, &mask, &sch};
        PSK_HIP(hipLaunchKernel(k, dim3(g), dim3(kBlock), args, (unsigned)lds, s));
        return PSK_OK;
    }
    if (T.schedule == kSchedBand) {
        const void *k = nullptr;
        switch (T.band_K) {
        case 1: k = reinterpret_cast<const void *>(&sptrsv_band_kernel<1>); break;
        case 2: k = reinterpret_cast<const void *>(&sptrsv_band_kernel<2>); break;
        case 4: k = reinterpret_cast<const void *>(&sptrsv_band_kernel<4>); break;
        case 8: k = reinterpret_cast<const void *>(&sptrsv_band_kernel<8>); break;
        default: return fail(PSK_ERR_ARG, "band schedule: bad record width");
        }
        const size_t lds = band_lds_bytes(T.ring_words, T.band_K);
        const int g = coop_grid(c, k, lds);
        int upper = T.upper ? 1 : 0;
        const int32_t *rr = T.rec_row, *re = T.rec_end, *rc = T.rec_c;
        const double *rv = T.rec_v, *rd = T.diag ? T.rec_d : nullptr;
        int64_t nb = T.band_nblocks, B = T.band_B;
        int mask = T.ring_words > 0 ? T.ring_words - 1 : -1;
        uint32_t *sch = T.sched;
        void *args[] = {&nn, &upper, &rhs, &rhs_idx, &x, &err, &rr, &re, &rc, &rv, &rd, &nb, &B, &mask, &sch};
        PSK_HIP(hipLaunchKernel(k, dim3(g), dim3(kBlock), args, (unsigned)lds, s));
        return PSK_OK;
    }
    const void *k = reinterpret_cast<const void *>(&sptrsv_kernel);
    const int g = syncfree_grid(c);
    const int32_t *ord = T.order;
    uint32_t *sch = T.sched;
    void *args[] = {&nn, &rp, &ci, &va, &dg, &rhs, &rhs_idx, &x, &err, &ord, &sch};
    PSK_HIP(hipLaunchKernel(k, dim3(g), dim3(kBlock), args, 0, s));
    return PSK_OK;
}

// out = (U^-1 L^-1 v[gather_in])[gather_out] for a triangular-solve chain (device pointers; out may
// not alias v)
// out = M^-1 v; add: out += M^-1 v (the Gauss-Seidel smoother's update, fused into the last gather)
static int ilu_apply_impl(const psk_prec *M, const double *v, double *out, bool add, hipStream_t s) {
    const int64_t n = M->n;
    if (n == 0) return PSK_OK;
    Context *c;
    PSK_TRY(ctx(&c));
    const unsigned fb = (unsigned)((n + kBlock - 1) / kBlock);
    double *y = M->work, *z = M->work + n;
    const int nbuf = (M->lo.present ? 1 : 0) + (M->up.present ? 1 : 0);
    // factors whose schedule fills (or needs) no sentinel of its own: the grid schedule's published lines only,
    // none for the levels schedule
    auto own_fill = [](const TriFactor &T) { return T.schedule == kSchedGrid || T.schedule == kSchedLevel; };
    const bool grid_any = (M->lo.present && own_fill(M->lo)) || (M->up.present && own_fill(M->up));
    if (nbuf > 0 && !grid_any) {
        hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((nbuf * n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           s, nbuf * n, y);   // y and z are contiguous
        PSK_HIP(hipGetLastError());
    } else if (nbuf > 0) {
        if (M->lo.present) PSK_TRY(fill_factor_output(M->lo, n, y, s));
        if (M->up.present) PSK_TRY(fill_factor_output(M->up, n, M->lo.present ? z : y, s));
    }
    const double *cur = v;                // current right-hand side
    const int32_t *cur_idx = M->gather_in;
    const TriFactor &first = M->lo.present ? M->lo : M->up;
    if (cur_idx && first.present && (first.schedule == kSchedGrid || first.schedule == kSchedPart)) {   // rhs[row]
        hipLaunchKernelGGL(gather_perm_kernel, dim3(fb), dim3(kBlock), 0, s, n, cur, cur_idx, M->work + 2 * n);
        PSK_HIP(hipGetLastError());
        cur = M->work + 2 * n;
        cur_idx = nullptr;
    }
    if (M->lo.present) {
        PSK_TRY(launch_factor(c, n, M->lo, cur, cur_idx, y, M->err, s));
        cur = y;
        cur_idx = nullptr;
    }
    if (M->up.present) {
        double *dst = M->lo.present ? z : y;
        PSK_TRY(launch_factor(c, n, M->up, cur, cur_idx, dst, M->err, s));
        cur = dst;
        cur_idx = nullptr;
    }
    if (cur_idx) {   // no factor at all: out = v[gather_in][gather_out]
        hipLaunchKernelGGL(gather_perm_kernel, dim3(fb), dim3(kBlock), 0, s, n, cur, cur_idx, y);
        PSK_HIP(hipGetLastError());
        cur = y;
    }
    if (add) hipLaunchKernelGGL(gather_add_kernel, dim3(fb), dim3(kBlock), 0, s, n, cur, M->gather_out, out);
    else hipLaunchKernelGGL(gather_perm_kernel, dim3(fb), dim3(kBlock), 0, s, n, cur, M->gather_out, out);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

int ilu_apply(const psk_prec *M, const double *v, double *out, hipStream_t s) {
    return ilu_apply_impl(M, v, out, false, s);
}

int ilu_apply_add(const psk_prec *M, const double *v, double *x, hipStream_t s) {
    return ilu_apply_impl(M, v, x, true, s);
}

int ilu_check_error(const psk_prec *M, hipStream_t s) {
    int32_t h = 0;
    PSK_HIP(hipMemcpyAsync(&h, M->err, 4, hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    if (h) {
        // a launch that stopped waiting may have left its scheduling words armed: re-zero them (and the
        // error word) so that the next apply starts clean
        for (const TriFactor *T : {&M->lo, &M->up})
            if (T->present && T->sched) (void)hipMemsetAsync(T->sched, 0, kSchedWords * sizeof(uint32_t), s);
        (void)hipMemsetAsync(M->err, 0, sizeof(int32_t), s);
        (void)hipStreamSynchronize(s);
        return fail(PSK_ERR_HIP, "triangular solve: dependency wait exceeded its bound, code " + std::to_string(h));
    }
    return PSK_OK;
}

}  // namespace psk

namespace psk {

void TriFactor::release() {
    void *ptrs[] = {rowptr, colidx, vals,   diag,    order,     rec_row,  rec_end,  rec_c,  rec_v,   rec_d,
                    gd_code, gd_coef, gd_diag, gd_idx, gd_dict, part_seg, part_rp, part_code, part_row, part_va,
                    grid_flag, sched, lv_rc,    lv_sl,    lv_cf,  lv_dg,   lv_b};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    *this = TriFactor();
}

// ---------------------------------------------------------------------------------------------
// host: schedules and their cost model
namespace {

constexpr int kGridDictMax = 64;

// Distinct records of the grid schedule's record blob (nsteps blocks of SB bytes: [64][K] codes at 0,
// [64][K] values at oc, [64] diagonals at od). With at most kGridDictMax of them: idx = each
// lane-step's record number in the kernel's access order (block-major, lane-minor), dict = [n][K]
// values, [n] diagonals, [n][K/2] code words packed two uint32 per double; ndict = n. Else ndict = 0.
void build_grid_dict(const unsigned char *gb, int64_t nsteps, int64_t SB, int K, int64_t oc, int64_t od,
                     std::vector<uint32_t> &idx, std::vector<double> &dict, int &ndict) {
    ndict = 0;
    const size_t rb = (size_t)K * 2 + (size_t)K * 8 + 8;   // key bytes: codes, values, diagonal
    std::vector<unsigned char> keys;                       // distinct records, rb bytes each
    std::unordered_map<uint64_t, std::vector<int>> by_hash;
    idx.assign((size_t)(nsteps * kGridLanes), 0);
    unsigned char key[2 * 8 + 8 * 8 + 8];
    for (int64_t t = 0; t < nsteps; ++t) {
        const unsigned char *blk = gb + t * SB;
        for (int l = 0; l < kGridLanes; ++l) {
            std::memcpy(key, blk + (size_t)l * K * 2, (size_t)K * 2);
            std::memcpy(key + K * 2, blk + oc + (size_t)l * K * 8, (size_t)K * 8);
            std::memcpy(key + K * 10, blk + od + (size_t)l * 8, 8);
            uint64_t h = 1469598103934665603ull;   // FNV-1a
            for (size_t i = 0; i < rb; ++i) h = (h ^ key[i]) * 1099511628211ull;
            int found = -1;
            auto &cand = by_hash[h];
            for (int c : cand)
                if (std::memcmp(keys.data() + (size_t)c * rb, key, rb) == 0) { found = c; break; }
            if (found < 0) {
                found = (int)(keys.size() / rb);
                if (found == kGridDictMax) {
                    idx.clear();
                    return;
                }
                keys.insert(keys.end(), key, key + rb);
                cand.push_back(found);
            }
            idx[(size_t)(t * kGridLanes + l)] = (uint32_t)found;
        }
    }
    const int nd = (int)(keys.size() / rb);
    const size_t ncw = (size_t)nd * K / 2;                  // code words
    dict.assign((size_t)nd * (K + 1) + (ncw + 1) / 2, 0.0);
    uint32_t *cw = reinterpret_cast<uint32_t *>(dict.data() + (size_t)nd * (K + 1));
    for (int r = 0; r < nd; ++r) {
        const unsigned char *k = keys.data() + (size_t)r * rb;
        std::memcpy(dict.data() + (size_t)r * K, k + K * 2, (size_t)K * 8);
        std::memcpy(dict.data() + (size_t)nd * K + r, k + K * 10, 8);
        std::memcpy(cw + (size_t)r * (K / 2), k, (size_t)K * 2);   // K uint16 codes = K/2 words, as in a record
    }
    ndict = nd;
}

// Cost model (us), fitted to measurements on MI355X (tools/bench_amg.py, tools/bench_gmres.py):
// sync-free: a row costs one agent-scope load round trip (~0.61) on its wave, plus a hand-off (~0.36)
// after its last dependency was published (FD m=1024 ILU with the DPP row total: 0.96 us per level,
// 12.1 ms for L + U); band: a local level
// costs ~0.9 us with the ring (it is paced by the one external load of the block's boundary row;
// FD 2048^2 Gauss-Seidel: 3.9 ms for ~4100 levels) and ~2.7 us without (AMG level 3 at 8192^2).
constexpr double kHopUs = 0.36, kRowUs = 0.61, kBandLevelRingUs = 1.0, kBandLevelMemUs = 2.7;
constexpr double kLdsLevelUs = 0.15, kLdsBytesPerUs = 40e3;   // LDS schedule (provisional)
// levels schedule: a step's barrier + LDS round trip, one CU's record stream (1708 steps, 31.5 MB: measured 0.615 ms)
constexpr double kLevelStepUs = 0.30, kLevelBytesPerUs = 200e3;   // fitted: AMG level 1 of -FD 8192^2, 0.615 ms
constexpr double kNarrowLevelUs = 0.8;    // narrow band local level (FD 8192^2 Gauss-Seidel: 12.6 ms / 16128 levels)

struct HostFactor {
    int64_t n = 0;
    bool upper = false;
    std::vector<int32_t> rp, ci;   // off-diagonal entries
    int64_t pos(int64_t i) const { return upper ? n - 1 - i : i; }
    int64_t row(int64_t p) const { return upper ? n - 1 - p : p; }
};

// global dependency levels -> counting-sort the rows by level (stable: solve order inside a level)
void level_order(const HostFactor &F, std::vector<int32_t> &order, std::vector<int32_t> &lev, int64_t &nlev) {
    const int64_t n = F.n;
    lev.assign(n, 0);
    int32_t maxl = -1;
    for (int64_t p = 0; p < n; ++p) {
        const int64_t i = F.row(p);
        int32_t l = 0;
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) l = std::max(l, lev[F.ci[j]] + 1);
        lev[i] = l;
        maxl = std::max(maxl, l);
    }
    nlev = maxl + 1;
    std::vector<int64_t> cnt((size_t)nlev + 1, 0);
    for (int64_t i = 0; i < n; ++i) cnt[lev[i] + 1]++;
    for (int64_t l = 0; l < nlev; ++l) cnt[l + 1] += cnt[l];
    order.assign(n, 0);
    for (int64_t p = 0; p < n; ++p) {
        const int64_t i = F.row(p);
        order[cnt[lev[i]]++] = (int32_t)i;
    }
}

// simulated time of the sync-free schedule: wave w processes order[w], order[w+W], ...
double simulate_syncfree(const HostFactor &F, const std::vector<int32_t> &order, int64_t waves) {
    std::vector<double> fin(F.n, 0.0), wave_free((size_t)std::max<int64_t>(waves, 1), 0.0);
    double tmax = 0.0;
    for (int64_t k = 0; k < F.n; ++k) {
        const int64_t i = order[k];
        double t = wave_free[k % waves];
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) t = std::max(t, fin[F.ci[j]] + kHopUs);
        t += kRowUs;
        fin[i] = t;
        wave_free[k % waves] = t;
        tmax = std::max(tmax, t);
    }
    return tmax;
}

struct Band {
    int64_t B = 0, nblocks = 0, G = 0;
    std::vector<int32_t> rows;
    std::vector<int64_t> lvl_ptr, blk_lvl;
    int32_t ring_words = 0;
    double est = 0.0;
};

// band schedule with block size B: local levels, ring check, simulated time with the workgroups that
// fit (per_cu_max per CU, fewer when the LDS ring + chunk buffers of record width K need it)
void build_band(const HostFactor &F, int64_t B, int num_cus, int per_cu_max, int K, Band &bd) {
    const int64_t n = F.n;
    bd.B = B;
    bd.nblocks = (n + B - 1) / B;
    std::vector<int32_t> llev(n, 0);   // local level by row
    int64_t max_dist = 0;
    for (int64_t p = 0; p < n; ++p) {
        const int64_t i = F.row(p), p_lo = (p / B) * B;
        int32_t l = 0;
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
            const int64_t pj = F.pos(F.ci[j]);
            if (pj >= p_lo) {
                l = std::max(l, llev[F.ci[j]] + 1);
                max_dist = std::max(max_dist, p - pj);
            }
        }
        llev[i] = l;
    }
    // rows of each block sorted by (local level, position)
    bd.rows.assign(n, 0);
    bd.blk_lvl.assign(bd.nblocks + 1, 0);
    bd.lvl_ptr.clear();
    std::vector<int64_t> cnt;
    for (int64_t b = 0; b < bd.nblocks; ++b) {
        const int64_t p_lo = b * B, p_hi = std::min(n, p_lo + B);
        int32_t maxl = 0;
        for (int64_t p = p_lo; p < p_hi; ++p) maxl = std::max(maxl, llev[F.row(p)]);
        cnt.assign((size_t)maxl + 2, 0);
        for (int64_t p = p_lo; p < p_hi; ++p) cnt[llev[F.row(p)] + 1]++;
        for (int32_t l = 0; l <= maxl; ++l) cnt[l + 1] += cnt[l];
        bd.blk_lvl[b] = (int64_t)bd.lvl_ptr.size();
        for (int32_t l = 0; l <= maxl; ++l) bd.lvl_ptr.push_back(p_lo + cnt[l]);
        std::vector<int64_t> fillp(cnt.begin(), cnt.end() - 1);
        for (int64_t p = p_lo; p < p_hi; ++p) {
            const int64_t i = F.row(p);
            bd.rows[p_lo + fillp[llev[i]]++] = (int32_t)i;
        }
    }
    bd.blk_lvl[bd.nblocks] = (int64_t)bd.lvl_ptr.size();
    bd.lvl_ptr.push_back(n);
    // LDS ring: W = pow2 >= max in-block dependency distance + 1; the slot of position p is next
    // written by position p+W, which must come at a later local level than p itself and than every
    // in-block reader of p
    bd.ring_words = 0;
    int64_t W = 1;
    while (W < max_dist + 1) W <<= 1;
    if (W <= kRingMaxWords) {
        std::vector<int32_t> maxcons(n, -1);   // by position
        for (int64_t p = 0; p < n; ++p) {
            const int64_t i = F.row(p), p_lo = (p / B) * B;
            for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
                const int64_t pj = F.pos(F.ci[j]);
                if (pj >= p_lo) maxcons[pj] = std::max(maxcons[pj], llev[i]);
            }
        }
        bool safe = true;
        for (int64_t p = 0; p < n && safe; ++p) {
            const int64_t q = p + W;
            if (q >= n || q / B != p / B) continue;
            const int32_t lq = llev[F.row(q)];
            if (lq <= llev[F.row(p)] || lq <= maxcons[p]) safe = false;
        }
        if (safe) bd.ring_words = (int32_t)W;
    }
    // simulated time: G resident workgroups take blocks round-robin, in order
    const size_t lds = band_lds_bytes(bd.ring_words, K);
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(per_cu_max, (int64_t)(160 * 1024 / std::max<size_t>(lds, 1))));
    const int64_t G = (int64_t)num_cus * per_cu;
    bd.G = G;
    const double cl = bd.ring_words ? kBandLevelRingUs : kBandLevelMemUs;
    std::vector<double> fin(n, 0.0), wg_free((size_t)std::max<int64_t>(G, 1), 0.0);
    double tmax = 0.0;
    for (int64_t b = 0; b < bd.nblocks; ++b) {
        const int64_t p_lo = b * B;
        double t = wg_free[b % G];
        for (int64_t L = bd.blk_lvl[b]; L < bd.blk_lvl[b + 1]; ++L) {
            double tl = t;
            for (int64_t q = bd.lvl_ptr[L]; q < bd.lvl_ptr[L + 1]; ++q) {
                const int64_t i = bd.rows[q];
                for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j)
                    if (F.pos(F.ci[j]) < p_lo) tl = std::max(tl, fin[F.ci[j]] + kHopUs);
            }
            const int64_t width = bd.lvl_ptr[L + 1] - bd.lvl_ptr[L];
            tl += cl * (double)((width + kBlock - 1) / kBlock);
            for (int64_t q = bd.lvl_ptr[L]; q < bd.lvl_ptr[L + 1]; ++q) fin[bd.rows[q]] = tl;
            t = tl;
        }
        wg_free[b % G] = t;
        tmax = std::max(tmax, t);
    }
    bd.est = tmax;
}

// Grid schedule plan (sptrsv_grid_kernel): width w = the most frequent solve-order distance >= 2
// (the line length of a 2-D stencil), every dependency as (yd lines, xd positions) back, the
// smallest skew making ud = xd + g(y) - g(y - yd) >= 1 for all of them — the integer skew sigma
// (g(y) = sigma*y), then sigma - 1/2 (g(y) = ((2 sigma - 1) y + phase) >> 1, either phase) when that
// also holds — and the ring depth. Rejected
// (ok = false) when the factor is not such a stencil: wide rows (> 8 entries), a dependency 64 or
// more lines back, a skew above 8, more than kGridMaxPE patterns reaching into the band above, a
// ring deeper than kGridMaxRing, or too few dependencies at distance w to call it a grid.
// fitted: FD 8192^2 Gauss-Seidel factor (8192 + 8191 steps) 5.0 ms, SA level 3 of it (2731 + 3*4095) 3.9 ms
constexpr double kGridStepUs = 0.26, kGridLagUs = 2.0;
constexpr int64_t kGridMaxYd = 8;   // lines of the band above held in the poller's LDS ring

struct GridPlan {
    bool ok = false;
    int64_t w = 0, H = 0, sigma2 = 0, phase = 0, off = 0;   // g(y) = (sigma2 * y + phase) >> 1
    int K = 0, pe = 0, maxyd = 0, ring = 0;
    GridExt ext{};
    double est = -1.0;
};

void plan_grid(const HostFactor &F, GridPlan &g) {
    const int64_t n = F.n;
    g = GridPlan();
    if (n < 4096) return;
    int32_t kmax = 0;
    std::unordered_map<int64_t, int64_t> hist;
    int64_t ndeps = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t len = F.rp[i + 1] - F.rp[i];
        kmax = std::max(kmax, len);
        ndeps += len;
        if (i % 7) continue;   // a sample is enough for the histogram
        const int64_t p = F.pos(i);
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
            const int64_t d = p - F.pos(F.ci[j]);
            if (d >= 2) hist[d]++;
        }
    }
    if (kmax == 0 || kmax > 8) return;
    // line-length candidates: the most frequent distances (a 9-point stencil ties w - 1, w and w + 1),
    // each holding at least ~1/8 of the rows; the first one that plans is taken
    std::vector<std::pair<int64_t, int64_t>> cand(hist.begin(), hist.end());   // (distance, count)
    std::sort(cand.begin(), cand.end(), [](const std::pair<int64_t, int64_t> &a, const std::pair<int64_t, int64_t> &b) {
        return a.second != b.second ? a.second > b.second : a.first < b.first;
    });
    int64_t w = 0;
    // patterns and skew, with grid position p + off: off = 0, or the offset that makes the solve order
    // START with a partial line (w - n mod w empty positions before it: an upper factor of a grid whose
    // last natural line is short, e.g. SA level 2 of -FD 8192^2, 1365 lines of 911 + one of 228)
    int64_t sigma2 = 0, phase = 0, maxyd = 0, maxud = 0, off = 0;
    std::vector<int32_t> ext_codes;
    // the dependency codes under g(y) = (s2 * y + ph) >> 1; false when a dependency is not >= 1 step back
    auto try_skew = [&](int64_t o, int64_t s2, int64_t ph) -> bool {
        maxud = 0;
        ext_codes.clear();
        for (int64_t i = 0; i < n; ++i) {
            const int64_t p = F.pos(i) + o, y = p / w, x = p % w;
            for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
                const int64_t pd = F.pos(F.ci[j]) + o, yd = y - pd / w, xd = x - pd % w;
                const int64_t ud = xd + grid_g(s2, ph, y) - grid_g(s2, ph, y - yd);
                if (ud < 1 || ud >= 1023) return false;
                maxud = std::max(maxud, ud);
                const int32_t code = (int32_t)(ud * 64 + yd);
                if (yd >= 1 && std::find(ext_codes.begin(), ext_codes.end(), code) == ext_codes.end()) {
                    if ((int)ext_codes.size() == kGridMaxPE) return false;
                    ext_codes.push_back(code);
                }
            }
        }
        off = o;
        sigma2 = s2;
        phase = ph;
        return true;
    };
    auto try_off = [&](int64_t o) -> bool {
        int64_t sigma = 0;
        maxyd = 0;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t p = F.pos(i) + o, y = p / w, x = p % w;
            for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
                const int64_t pd = F.pos(F.ci[j]) + o, yd = y - pd / w, xd = x - pd % w;
                if (yd > kGridMaxYd) return false;
                maxyd = std::max(maxyd, yd);
                if (yd >= 1 && xd < 1) sigma = std::max(sigma, (1 - xd + yd - 1) / yd);
            }
        }
        if (sigma > 8) return false;
        // half a step less skew when the dependencies that need sigma occur on every other line only
        // (round 4: AMG level 3 2.67 -> 2.20 ms, profiles/r4_half_skew_ab.txt)
        constexpr bool half = true;
        if (half && sigma >= 2 && (try_skew(o, 2 * sigma - 1, 0) || try_skew(o, 2 * sigma - 1, 1))) return true;
        return try_skew(o, 2 * sigma, 0);
    };
    bool planned = false;
    for (size_t ci = 0; ci < cand.size() && ci < 4 && !planned; ++ci) {
        w = cand[ci].first;
        if (w < 2 || cand[ci].second * 7 * 8 < n) break;
        planned = try_off(0) || (n % w != 0 && try_off(w - n % w));
    }
    if (!planned) return;
    // ring rows: the deepest dependency, and room for the poller to stay a 64-position chunk ahead
    int ring = ext_codes.empty() ? 1 : 2 * kGridLanes;
    while (ring < maxud + 1 + (ext_codes.empty() ? 0 : kGridLanes)) ring <<= 1;
    if (ring > kGridMaxRing) return;
    g.ok = true;
    g.w = w;
    g.off = off;
    g.H = (n + off + w - 1) / w;
    g.sigma2 = sigma2;
    g.phase = phase;
    g.K = kmax <= 2 ? 2 : (kmax <= 4 ? 4 : 8);
    g.pe = (int)ext_codes.size();
    g.maxyd = (int)maxyd;
    g.ring = ring;
    for (int e = 0; e < g.pe; ++e) {
        const int32_t yd = ext_codes[e] & 63;
        g.ext.delta[e] = ext_codes[e];
        g.ext.yd[e] = yd;
    }
    const int64_t nbands = (g.H + kGridLanes - 1) / kGridLanes;
    g.est = (double)((w - 1) + grid_g(sigma2, phase, g.H - 1) + 1) * kGridStepUs + (double)nbands * kGridLagUs;
    (void)ndeps;
}

}  // namespace

}  // namespace psk

using namespace psk;

// Partitioned schedule (sptrsv_part_kernel). Strip of row i: its natural index nat[i] cut into P
// equal ranges; strip s runs on workgroup (s % 8) * (P / 8) + s / 8, so neighbouring strips share an
// XCD (dispatch deals workgroups round-robin over the 8 XCDs). Two cost models (us): the PRIORITY
// model orders each strip's rows (ASAP finish times: a dependency inside the strip a, across strips
// b, a row c), the ESTIMATE model simulates the resulting schedule with constants fitted to MI355X
// measurements of the kernel (tools/ilu_probe.py, tools/part_micro.py: a wave's row costs ~0.5 us
// of issue and memory latency even when its dependencies are done; an LDS hand-off ~0.2 us
// including the row total and division; a published-value hand-off between CUs ~2 us under load).
// Strips longer than kPartMaxStrip rows measured slower than sync-free (FD 2896^2 ILUT: 32.8k rows
// per strip, 31.4 vs ~27 ms) and are not planned.
constexpr double kPartPrioLocalUs = 0.10, kPartPrioRemoteUs = 1.2, kPartPrioRowUs = 0.15;
constexpr double kPartEstLocalUs = 0.20, kPartEstRemoteUs = 2.0, kPartEstRowUs = 0.5;
constexpr int64_t kPartMaxStrip = 16384;

struct PartPlan {
    int P = 0;
    double est = -1.0;
    std::vector<int32_t> wg, lpos;   // workgroup and local position of every row
    std::vector<int64_t> seg;        // P + 1
};

void plan_part(const HostFactor &F, const std::vector<int32_t> &nat, int P, PartPlan &pp) {
    const int64_t n = F.n;
    pp.P = P;
    pp.wg.assign(n, 0);
    const int per = std::max(1, P / 8);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t s = (nat.empty() ? i : nat[i]) * P / n;
        pp.wg[i] = (P % 8 == 0) ? (int32_t)((s % 8) * per + s / 8) : (int32_t)s;
    }
    // ASAP finish times in solve order (a topological order)
    std::vector<double> fin(n, 0.0);
    for (int64_t p = 0; p < n; ++p) {
        const int64_t i = F.row(p);
        double t = 0.0;
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j)
            t = std::max(t, fin[F.ci[j]] + (pp.wg[F.ci[j]] == pp.wg[i] ? kPartPrioLocalUs : kPartPrioRemoteUs));
        fin[i] = t + kPartPrioRowUs;
    }
    // every workgroup's rows in ASAP order (ties: solve order)
    std::vector<int32_t> idx(n);
    for (int64_t i = 0; i < n; ++i) idx[i] = (int32_t)i;
    std::sort(idx.begin(), idx.end(), [&](int32_t u, int32_t v) {
        if (pp.wg[u] != pp.wg[v]) return pp.wg[u] < pp.wg[v];
        if (fin[u] != fin[v]) return fin[u] < fin[v];
        return F.pos(u) < F.pos(v);
    });
    pp.seg.assign((size_t)P + 1, 0);
    pp.lpos.assign(n, 0);
    for (int64_t k = 0; k < n; ++k) pp.seg[(size_t)pp.wg[idx[k]] + 1]++;
    for (int w = 0; w < P; ++w) pp.seg[w + 1] += pp.seg[w];
    for (int64_t k = 0; k < n; ++k) pp.lpos[idx[k]] = (int32_t)(k - pp.seg[pp.wg[idx[k]]]);
    // simulate: rows in global ASAP order, wave lpos % 16 of their workgroup
    std::sort(idx.begin(), idx.end(), [&](int32_t u, int32_t v) { return fin[u] != fin[v] ? fin[u] < fin[v] : F.pos(u) < F.pos(v); });
    std::vector<double> done(n, 0.0), wfree((size_t)P * kPartWaves, 0.0);
    double tmax = 0.0;
    for (int64_t k = 0; k < n; ++k) {
        const int32_t i = idx[k];
        double &wf = wfree[(size_t)pp.wg[i] * kPartWaves + pp.lpos[i] % kPartWaves];
        double t = wf;
        for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j) {
            const int32_t d = F.ci[j];
            const bool loc = pp.wg[d] == pp.wg[i] && pp.lpos[i] - pp.lpos[d] < kPartSlots;
            t = std::max(t, done[d] + (loc ? kPartEstLocalUs : kPartEstRemoteUs));
        }
        done[i] = wf = t + kPartEstRowUs;
        tmax = std::max(tmax, done[i]);
    }
    pp.est = tmax;
}

template <class T>
static int upload(T **d, const std::vector<T> &h) {
    if (h.empty()) {
        *d = nullptr;
        return PSK_OK;
    }
    if (hipMalloc(d, h.size() * sizeof(T)) != hipSuccess) return fail(PSK_ERR_ALLOC, "hipMalloc trisolve");
    if (hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return fail(PSK_ERR_HIP, "hipMemcpy trisolve");
    return PSK_OK;
}

// Split one host CSR factor into off-diagonal entries + diagonal. lower: entries must have c <= i.
static int split_factor(int64_t n, const int32_t *rp, const int32_t *ci, const double *va, bool lower, bool unit,
                        std::vector<int32_t> &orp, std::vector<int32_t> &oci, std::vector<double> &ova,
                        std::vector<double> &dg) {
    orp.assign(n + 1, 0);
    if (!unit) dg.assign(n, 0.0);
    const char *what = lower ? "lower factor" : "upper factor";
    if (rp[0] != 0) return fail(PSK_ERR_ARG, std::string(what) + ": rowptr[0] != 0");
    for (int64_t i = 0; i < n; ++i) {
        if (rp[i + 1] < rp[i]) return fail(PSK_ERR_ARG, std::string(what) + ": rowptr not monotone");
        bool has_diag = false;
        for (int32_t j = rp[i]; j < rp[i + 1]; ++j) {
            const int32_t c = ci[j];
            if (c < 0 || c >= n || (lower ? c > i : c < i))
                return fail(PSK_ERR_ARG, std::string(what) + ": entry on the wrong side of the diagonal");
            if (c == i) {
                if (!unit) dg[i] += va[j];
                has_diag = true;
                continue;
            }
            oci.push_back(c);
            ova.push_back(va[j]);
        }
        if (!unit && !has_diag) return fail(PSK_ERR_ARG, std::string(what) + ": missing diagonal entry");
        orp[i + 1] = (int32_t)oci.size();
    }
    return PSK_OK;
}

static int check_perm(int64_t n, const int32_t *p, const char *what) {
    std::vector<char> seen(n, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (p[i] < 0 || p[i] >= n || seen[p[i]]) return fail(PSK_ERR_ARG, std::string(what) + ": not a permutation");
        seen[p[i]] = 1;
    }
    return PSK_OK;
}

// The 5-point grid signature of an upper factor (TriFactor::fd5_*): triu of a 5-point operator on an m x H grid
// with one value per diagonal. amg.hip fuses two Gauss-Seidel sweeps of such a level into one launch.
static void detect_fd5(int64_t n, const std::vector<int32_t> &rp, const std::vector<int32_t> &ci,
                       const std::vector<double> &va, const std::vector<double> &dg, TriFactor &T) {
    T.fd5_m = 0;
    if (n < 4 || dg.empty() || rp[1] - rp[0] != 2) return;
    const int64_t m = std::max(ci[rp[0]], ci[rp[0] + 1]);
    if (m < 2 || n % m != 0 || n / m < 2) return;
    auto same = [](double a, double b) { return std::memcmp(&a, &b, sizeof(double)) == 0; };
    const double d = dg[0];
    double a1 = 0.0, am = 0.0;
    bool h1 = false, hm = false;
    int mfirst = -1;
    for (int64_t i = 0; i < n; ++i) {
        if (!same(dg[i], d)) return;
        const bool e1 = i % m != m - 1, em = i + m < n;
        const int32_t a = rp[i], e = rp[i + 1];
        if (e - a != (int)e1 + (int)em) return;
        bool s1 = false, sm = false;
        for (int32_t k = a; k < e; ++k) {
            const int64_t c = ci[k];
            if (e1 && !s1 && c == i + 1) {
                s1 = true;
                if (!h1) a1 = va[k], h1 = true;
                else if (!same(va[k], a1)) return;
            } else if (em && !sm && c == i + m) {
                sm = true;
                if (!hm) am = va[k], hm = true;
                else if (!same(va[k], am)) return;
            } else {
                return;
            }
        }
        if (e1 && em) {
            const int f = ci[a] == i + m;
            if (mfirst < 0) mfirst = f;
            else if (f != mfirst) return;
        }
    }
    if (!h1 || !hm || mfirst < 0) return;
    T.fd5_m = m;
    T.fd5_d = d;
    T.fd5_a1 = a1;
    T.fd5_am = am;
    T.fd5_mfirst = mfirst;
}

// Build, schedule and upload one factor.
static int make_factor(const Context *c, int64_t n, const int32_t *rp, const int32_t *ci, const double *va, bool upper,
                       bool unit, const std::vector<int32_t> &nat, TriFactor &T) {
    HostFactor F;
    F.n = n;
    F.upper = upper;
    std::vector<double> ova, dg;
    PSK_TRY(split_factor(n, rp, ci, va, !upper, unit, F.rp, F.ci, ova, dg));
    if (upper && !unit && nat.empty()) detect_fd5(n, F.rp, F.ci, ova, dg, T);
    std::vector<int32_t> order, lev;
    int64_t nlev = 0;
    level_order(F, order, lev, nlev);
    const int64_t waves = (int64_t)syncfree_grid(c) * kWaves;
    T.est_syncfree_us = simulate_syncfree(F, order, waves);
    // band candidates: one block per workgroup, and 2x / 4x / 8x more blocks. Eligible: at most 8
    // off-diagonal entries per row (record width K), levels at most one chunk wide, LDS fits a CU.
    int32_t kmax = 0;
    for (int64_t i = 0; i < n; ++i) kmax = std::max(kmax, F.rp[i + 1] - F.rp[i]);
    int K = 1;
    while (K < kmax) K <<= 1;
    Band best;
    best.est = -1.0;
    bool band_ok = false;
    std::vector<int64_t> cands = {(int64_t)c->num_cus, 2 * (int64_t)c->num_cus, 4 * (int64_t)c->num_cus,
                                  8 * (int64_t)c->num_cus};
    for (int64_t nb : cands) {
        if (n == 0 || kmax > 8) break;
        const int64_t B = std::max<int64_t>(64, (n + nb - 1) / nb);
        Band bd;
        build_band(F, B, c->num_cus, 2, K, bd);
        int64_t wmax = 0;
        for (size_t L = 0; L + 1 < bd.lvl_ptr.size(); ++L) wmax = std::max(wmax, bd.lvl_ptr[L + 1] - bd.lvl_ptr[L]);
        const bool ok = wmax <= kBandChunk && band_lds_bytes(bd.ring_words, K) <= 160 * 1024 - 64;   // + the static block ticket
        if (ok && (!band_ok || bd.est < best.est)) {
            best = std::move(bd);
            band_ok = true;
        }
        if (B == 64) break;
    }
    // narrow band (one solving wave, staging waves): every local level at most one wave wide, ring present
    bool narrow = false;
    if (band_ok && best.ring_words > 0 && narrow_lds_bytes(best.ring_words, K) <= 160 * 1024 - 64) {
        int64_t wmax = 0;
        for (size_t L = 0; L + 1 < best.lvl_ptr.size(); ++L) wmax = std::max(wmax, best.lvl_ptr[L + 1] - best.lvl_ptr[L]);
        const char *ne = std::getenv("PSK_BAND_NARROW");
        narrow = wmax <= kNarrowWidth && !(ne && std::atoi(ne) == 0);
        if (narrow) best.est *= kNarrowLevelUs / kBandLevelRingUs;   // levels dominate the simulated time
    }
    T.band_narrow = narrow;
    T.est_band_us = band_ok ? best.est : -1.0;
    T.schedule = (band_ok && best.est < T.est_syncfree_us) ? kSchedBand : kSchedSyncFree;
    // one workgroup with x in LDS: a level costs an LDS hand-off, the entries stream through one CU
    T.est_lds_us = -1.0;
    if (n > 0 && n <= kLdsMaxRows) {
        T.est_lds_us = (double)nlev * kLdsLevelUs + (double)F.ci.size() * 12.0 / kLdsBytesPerUs;
        const double other = T.schedule == kSchedBand ? T.est_band_us : T.est_syncfree_us;
        if (T.est_lds_us < other) T.schedule = kSchedLds;
    }
    // grid schedule (2-D stencil factors): records in solve order
    GridPlan gp;
    plan_grid(F, gp);
    if (n > kGridMaxRows) gp.ok = false;   // the grid kernel's 32-bit buffer offsets
    T.est_grid_us = gp.ok ? gp.est : -1.0;
    std::vector<uint16_t> gcode;
    std::vector<double> gcoef, gdiag, gdict;
    std::vector<uint32_t> gidx;
    if (gp.ok) {
        const double cur = T.schedule == kSchedBand ? T.est_band_us
                           : T.schedule == kSchedLds ? T.est_lds_us : T.est_syncfree_us;
        if (gp.est < cur) T.schedule = kSchedGrid;
        T.grid_K = gp.K;
        T.grid_pe = gp.pe;
        T.grid_maxyd = gp.maxyd;
        T.grid_ring = gp.ring;
        T.grid_w = gp.w;
        T.grid_H = gp.H;
        T.grid_sigma = gp.sigma2;
        T.grid_phase = gp.phase;
        T.grid_off = gp.off;
        T.grid_ext = gp.ext;
        // grid position p + off = (y*w + x): band b = y / 64, lane y % 64, step u - g(64b) with u = x + g(y);
        // one GridStep block per (band, step): codes (ud*64 + yd), values in stored order, diagonal.
        // Padding: value 0, code 0 (the lane's own column of the current row); empty lanes: diagonal 1
        // so the wave's unused results stay finite (padding entries read them times 0.0)
        // steps per band: g(y0 + 63) - g(y0) is the same for every band (sigma2 * y0 is even)
        T.grid_S = (gp.w - 1) + grid_g(gp.sigma2, gp.phase, kGridLanes - 1) - grid_g(gp.sigma2, gp.phase, 0) + 1;
        const int64_t SB = gp.K == 2 ? GridStep<2>::kBytes : gp.K == 4 ? GridStep<4>::kBytes : GridStep<8>::kBytes;
        const int64_t nb = (gp.H + kGridLanes - 1) / kGridLanes, nsteps = nb * T.grid_S;
        const int64_t oc = kGridLanes * 2 * gp.K, od = oc + kGridLanes * 8 * gp.K;
        gcoef.assign((size_t)(nsteps * SB / 8), 0.0);
        unsigned char *gb = reinterpret_cast<unsigned char *>(gcoef.data());
        for (int64_t t = 0; t < nsteps; ++t)
            for (int l = 0; l < kGridLanes; ++l) reinterpret_cast<double *>(gb + t * SB + od)[l] = 1.0;
        for (int64_t i = 0; i < n; ++i) {
            const int64_t p = F.pos(i) + gp.off, y = p / gp.w, x = p % gp.w, b = y / kGridLanes, l = y % kGridLanes;
            const int64_t st = x + grid_g(gp.sigma2, gp.phase, y) - grid_g(gp.sigma2, gp.phase, kGridLanes * b);
            unsigned char *blk = gb + (b * T.grid_S + st) * SB;
            uint16_t *codes = reinterpret_cast<uint16_t *>(blk) + l * gp.K;
            double *vals = reinterpret_cast<double *>(blk + oc) + l * gp.K;
            int k = 0;
            for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j, ++k) {
                const int64_t pd = F.pos(F.ci[j]) + gp.off, yd = y - pd / gp.w, xd = x - pd % gp.w;
                codes[k] = (uint16_t)((xd + grid_g(gp.sigma2, gp.phase, y) - grid_g(gp.sigma2, gp.phase, y - yd)) * 64 + yd);
                vals[k] = ova[j];
            }
            reinterpret_cast<double *>(blk + od)[l] = dg.empty() ? 1.0 : dg[i];
        }
        // record dictionary: when the lane-steps hold at most kGridDictMax distinct records (stencil
        // factors: the interior record, the boundary variants, the empty lanes), the kernel loads one
        // 32-bit index per lane-step instead of the record (PSK_TRISOLVE_GRID_DICT=0: never)
        const char *gde = std::getenv("PSK_TRISOLVE_GRID_DICT");
        if (!(gde && std::atoi(gde) == 0))
            build_grid_dict(gb, nsteps, SB, gp.K, oc, od, gidx, gdict, T.grid_dict_n);
        // the dictionary kernel divides by Markstein correction from RN(1/d) (div_markstein), which
        // equals IEEE r / d only while 1/d, the quotient and the remainder stay normal: keep the
        // dictionary only for diagonals with 2^-100 <= |d| <= 2^100 (the kernel itself falls back to
        // r / d for right-hand sides outside [2^-900, 2^900]); otherwise the per-step records
        for (int i = 0; i < T.grid_dict_n; ++i) {
            const double d = std::fabs(gdict[(size_t)T.grid_dict_n * gp.K + (size_t)i]);
            if (!(d >= 0x1p-100 && d <= 0x1p+100)) {
                T.grid_dict_n = 0;
                std::vector<double>().swap(gdict);
                std::vector<uint32_t>().swap(gidx);
                break;
            }
        }
        if (T.grid_dict_n > 0) std::vector<double>().swap(gcoef);   // the records are not uploaded
    }
    // levels schedule (sptrsv_levels_kernel): one workgroup of W = 64..256 lanes, one level (or a W-row
    // piece of one) per step, x in host-assigned LDS slots. Eligible: at most 16 entries per row, the values
    // alive at once (written, a reader still to come) within kLevelMaxSlots, records < 4 GB.
    // PSK_TRISOLVE_LEVELS=0 never plans it, =1 builds it and selects it whenever eligible.
    std::vector<uint64_t> lrc, lsl;
    std::vector<double> lcf, ldg;
    bool lv_forced = false;
    {
        const char *le = std::getenv("PSK_TRISOLVE_LEVELS");
        const bool force = le && std::atoi(le) == 1, off = le && std::atoi(le) == 0;
        if (!off && n > 0 && n < (int64_t)kLevelIdle && kmax <= kLevelMaxK) {
            std::vector<int64_t> lw((size_t)nlev, 0);
            for (int64_t i = 0; i < n; ++i) lw[(size_t)lev[(size_t)i]]++;
            int64_t wmax = 1;
            for (int64_t w : lw) wmax = std::max(wmax, w);
            const int W = (int)std::min<int64_t>(kLevelMaxW, (wmax + 63) / 64 * 64);
            // positions: level by level in `order`, each level padded to whole steps of W
            std::vector<int64_t> pos((size_t)n);
            int64_t steps = 0;
            {
                int64_t q = 0;
                for (int64_t L = 0; L < nlev; ++L) {
                    const int64_t cntL = lw[(size_t)L], st = (cntL + W - 1) / W;
                    for (int64_t j = 0; j < cntL; ++j) pos[(size_t)order[(size_t)(q + j)]] = steps * W + j;
                    q += cntL;
                    steps += st;
                }
            }
            steps = (steps + kLevelPad - 1) / kLevelPad * kLevelPad;   // the kernel's loop: whole groups of D steps
            // slot of every value: the step of its last reader, then greedy interval allocation in step order
            std::vector<int64_t> last((size_t)n, -1);
            for (int64_t i = 0; i < n; ++i)
                for (int32_t j = F.rp[(size_t)i]; j < F.rp[(size_t)i + 1]; ++j)
                    last[(size_t)F.ci[(size_t)j]] = std::max(last[(size_t)F.ci[(size_t)j]], pos[(size_t)i] / W);
            std::vector<int32_t> by_pos((size_t)steps * W, -1), slot((size_t)n, -1);
            for (int64_t i = 0; i < n; ++i) by_pos[(size_t)pos[(size_t)i]] = (int32_t)i;
            std::priority_queue<std::pair<int64_t, int32_t>, std::vector<std::pair<int64_t, int32_t>>,
                                std::greater<std::pair<int64_t, int32_t>>> live;   // (last reader step, slot)
            std::vector<int32_t> freed;
            int32_t nslots = 0;
            bool fits = true;
            for (int64_t st = 0; st < steps && fits; ++st) {
                while (!live.empty() && live.top().first < st) {   // its last reader ran in an earlier step
                    freed.push_back(live.top().second);
                    live.pop();
                }
                for (int64_t t = 0; t < W; ++t) {
                    const int32_t i = by_pos[(size_t)(st * W + t)];
                    if (i < 0 || last[(size_t)i] < 0) continue;   // idle lane / nobody reads it: the trash slot
                    int32_t sl;
                    if (!freed.empty()) {
                        sl = freed.back();
                        freed.pop_back();
                    } else {
                        sl = nslots++;
                    }
                    slot[(size_t)i] = sl;
                    live.push({last[(size_t)i], sl});
                }
                fits = nslots + 2 <= kLevelMaxSlots;
            }
            const int KM = kmax <= 4 ? 4 : kmax <= 8 ? 8 : kmax <= 12 ? 12 : 16;
            fits = fits && steps * W * KM * 8 < ((int64_t)1 << 32);
            if (fits) {
                const int64_t R = nslots, zero = R, trash = R + 1;
                T.est_level_us = (double)steps * kLevelStepUs +
                                 (double)steps * W * (24.0 + 10.0 * KM) / kLevelBytesPerUs;
                const double cur = T.schedule == kSchedBand ? T.est_band_us
                                   : T.schedule == kSchedLds  ? T.est_lds_us
                                   : T.schedule == kSchedGrid ? T.est_grid_us
                                                              : T.est_syncfree_us;
                if (force || T.est_level_us < cur) {
                    lv_forced = force;
                    T.schedule = kSchedLevel;
                    T.lv_steps = steps;
                    T.lv_W = W;
                    T.lv_R = (int)R;
                    T.lv_KM = KM;
                    const size_t NP = (size_t)steps * W;
                    lrc.assign(NP, (uint64_t)kLevelIdle | ((uint64_t)trash << 40));
                    lsl.assign(NP * (KM / 4), (uint64_t)zero * 0x0001000100010001ull);
                    lcf.assign(NP * KM, -0.0);
                    ldg.assign(NP, 1.0);
                    for (int64_t i = 0; i < n; ++i) {
                        const int64_t p = pos[(size_t)i], st = p / W, t = p % W;
                        const int32_t a = F.rp[(size_t)i], e = F.rp[(size_t)i + 1];
                        const uint64_t ws = slot[(size_t)i] >= 0 ? (uint64_t)slot[(size_t)i] : (uint64_t)trash;
                        lrc[(size_t)p] = (uint64_t)(uint32_t)i | (ws << 40);
                        for (int32_t j = a; j < e; ++j) {
                            const int k = j - a;
                            const uint64_t ds = (uint64_t)slot[(size_t)F.ci[(size_t)j]];   // read: it has a reader
                            uint64_t &w = lsl[((size_t)st * (KM / 4) + (size_t)(k / 4)) * W + (size_t)t];
                            w = (w & ~((uint64_t)0xFFFF << (16 * (k % 4)))) | (ds << (16 * (k % 4)));
                            // coefficient pairs (2k2, 2k2 + 1) of lane t: one 16-byte load
                            lcf[(((size_t)st * (KM / 2) + (size_t)(k / 2)) * W + (size_t)t) * 2 + (size_t)(k % 2)] = ova[(size_t)j];
                        }
                        if (!dg.empty()) ldg[(size_t)p] = dg[(size_t)i];
                    }
                }
            }
        }
    }
    // partitioned schedule: planned for factors too large for one CU and not solved by the grid
    // schedule (PSK_TRISOLVE_PART=0 disables it, =1 builds it and selects it whatever the estimate)
    std::vector<int64_t> pseg;
    std::vector<int32_t> prp, pcode, prow;
    std::vector<double> pva;
    {
        const char *pe = std::getenv("PSK_TRISOLVE_PART");
        const bool force = pe && std::atoi(pe) == 1, off = pe && std::atoi(pe) == 0;
        const int P = c->num_cus;   // one strip per CU (16-64 strips measured slower, round 5)
        const int64_t strip = (n + P - 1) / std::max(1, P);
        if (!off && !lv_forced && n > kLdsMaxRows && n >= (int64_t)P * kPartWaves &&
            (force || (T.schedule != kSchedGrid && strip <= kPartMaxStrip))) {
            PartPlan pp;
            plan_part(F, nat, P, pp);
            T.est_part_us = pp.est;
            const double cur = T.schedule == kSchedBand  ? T.est_band_us
                               : T.schedule == kSchedLds   ? T.est_lds_us
                               : T.schedule == kSchedGrid  ? T.est_grid_us
                               : T.schedule == kSchedLevel ? T.est_level_us
                                                           : T.est_syncfree_us;
            if (force || pp.est < cur) {
                T.schedule = kSchedPart;
                T.part_P = pp.P;
                pseg = pp.seg;
                prow.assign(n, 0);
                prp.assign((size_t)n + 1, 0);
                for (int64_t i = 0; i < n; ++i) {
                    const int64_t k = pp.seg[pp.wg[i]] + pp.lpos[i];
                    prow[k] = (int32_t)i;
                    prp[k + 1] = F.rp[i + 1] - F.rp[i];
                }
                for (int64_t k = 0; k < n; ++k) prp[k + 1] += prp[k];
                pcode.assign(F.ci.size() + kPartPadEntries, 0);   // padding: the kernel's unconditional loads
                pva.assign(F.ci.size() + kPartPadEntries, 0.0);
                for (int64_t k = 0; k < n; ++k) {
                    const int32_t i = prow[k];
                    int32_t o = prp[k];
                    for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j, ++o) {
                        const int32_t d = F.ci[j];
                        const bool loc = pp.wg[d] == pp.wg[i] && pp.lpos[i] - pp.lpos[d] < kPartSlots;
                        pcode[o] = loc ? ~pp.lpos[d] : d;   // ~q = -q-1 < 0: the strip's q-th row
                        pva[o] = ova[j];
                    }
                }
            }
        }
    }
    if (const char *ve = std::getenv("PSK_TRISOLVE_VERBOSE"))   // development: the cost model's view
        if (std::atoi(ve))
            std::fprintf(stderr, "psk trisolve %s n=%lld levels=%lld est_us syncfree=%.0f band=%.0f lds=%.0f grid=%.0f "
                                 "part=%.0f levels=%.0f -> schedule %d\n",
                         upper ? "U" : "L", (long long)n, (long long)nlev, T.est_syncfree_us, T.est_band_us,
                         T.est_lds_us, T.est_grid_us, T.est_part_us, T.est_level_us, T.schedule);
    T.present = true;
    T.upper = upper;
    T.nnz = (int64_t)F.ci.size();
    T.levels = nlev;
    T.band_B = best.B;
    T.band_nblocks = best.nblocks;
    T.band_levels = best.lvl_ptr.empty() ? 0 : (int64_t)best.lvl_ptr.size() - 1;
    T.ring_words = best.ring_words;
    std::vector<int32_t> rrow, rend, rc_;
    std::vector<double> rv, rd;
    if (band_ok) {
        T.band_K = K;
        rrow.assign(n, 0);
        rend.assign(n, 0);
        rc_.assign((size_t)K * n, -1);
        rv.assign((size_t)K * n, 0.0);
        if (!dg.empty()) rd.assign(n, 1.0);
        for (int64_t b = 0; b < best.nblocks; ++b) {
            const int64_t p_lo = b * best.B;
            for (int64_t L = best.blk_lvl[b]; L < best.blk_lvl[b + 1]; ++L)
                for (int64_t q = best.lvl_ptr[L]; q < best.lvl_ptr[L + 1]; ++q) {
                    const int32_t i = best.rows[q];
                    rrow[q] = i;
                    rend[q] = (int32_t)(best.lvl_ptr[L + 1] - p_lo);
                    int k = 0;
                    for (int32_t j = F.rp[i]; j < F.rp[i + 1]; ++j, ++k) {
                        rc_[(size_t)k * n + q] = F.ci[j];
                        rv[(size_t)k * n + q] = ova[j];
                    }
                    if (!dg.empty()) rd[q] = dg[i];
                }
        }
    }
    // the sync-free kernel's copy of the factor, in solve order (position k = row order[k])
    std::vector<int32_t> krp((size_t)n + 1, 0), kci(F.ci.size());
    std::vector<double> kva(ova.size());
    for (int64_t k = 0; k < n; ++k) {
        const int32_t i = order[(size_t)k], a = F.rp[(size_t)i], e = F.rp[(size_t)i + 1];
        std::copy(F.ci.begin() + a, F.ci.begin() + e, kci.begin() + krp[(size_t)k]);
        std::copy(ova.begin() + a, ova.begin() + e, kva.begin() + krp[(size_t)k]);
        krp[(size_t)k + 1] = krp[(size_t)k] + (e - a);
    }
    int rc = upload(&T.rowptr, krp);
    if (rc == PSK_OK) rc = upload(&T.colidx, kci);
    if (rc == PSK_OK) rc = upload(&T.vals, kva);
    if (rc == PSK_OK) rc = upload(&T.diag, dg);
    if (rc == PSK_OK) rc = upload(&T.order, order);
    if (rc == PSK_OK) rc = upload(&T.rec_row, rrow);
    if (rc == PSK_OK) rc = upload(&T.rec_end, rend);
    if (rc == PSK_OK) rc = upload(&T.rec_c, rc_);
    if (rc == PSK_OK) rc = upload(&T.rec_v, rv);
    if (rc == PSK_OK) rc = upload(&T.rec_d, rd);
    if (rc == PSK_OK) rc = upload(&T.gd_code, gcode);
    if (rc == PSK_OK) rc = upload(&T.gd_coef, gcoef);
    if (rc == PSK_OK) rc = upload(&T.gd_diag, gdiag);
    if (rc == PSK_OK) rc = upload(&T.gd_idx, gidx);
    if (rc == PSK_OK) rc = upload(&T.gd_dict, gdict);
    if (rc == PSK_OK) rc = upload(&T.grid_flag, std::vector<int32_t>(T.grid_dict_n > 0 ? 1 : 0, 0));
    if (rc == PSK_OK) rc = upload(&T.sched, std::vector<uint32_t>(kSchedWords, 0u));   // block tickets / enrolment
    if (rc == PSK_OK) rc = upload(&T.part_seg, pseg);
    if (rc == PSK_OK) rc = upload(&T.part_rp, prp);
    if (rc == PSK_OK) rc = upload(&T.part_code, pcode);
    if (rc == PSK_OK) rc = upload(&T.part_row, prow);
    if (rc == PSK_OK) rc = upload(&T.part_va, pva);
    if (rc == PSK_OK) rc = upload(&T.lv_rc, lrc);
    if (rc == PSK_OK) rc = upload(&T.lv_sl, lsl);
    if (rc == PSK_OK) rc = upload(&T.lv_cf, lcf);
    if (rc == PSK_OK) rc = upload(&T.lv_dg, ldg);
    if (rc == PSK_OK) rc = upload(&T.lv_b, std::vector<double>(lrc.size(), 0.0));
    return rc;
}

extern "C" int psk_prec_create_trisolve(int64_t n, const int32_t *l_rowptr, const int32_t *l_colidx,
                                        const double *l_vals, int32_t l_unit, const int32_t *u_rowptr,
                                        const int32_t *u_colidx, const double *u_vals, int32_t u_unit,
                                        const int32_t *gather_in, const int32_t *gather_out, psk_prec **out) {
    if (!out || n < 0) return fail(PSK_ERR_ARG, "psk_prec_create_trisolve: bad arguments");
    if (n >= INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "psk_prec_create_trisolve: n must fit int32");
    if (l_rowptr && l_rowptr[n] > 0 && (!l_colidx || !l_vals)) return fail(PSK_ERR_ARG, "lower factor: NULL arrays");
    if (u_rowptr && u_rowptr[n] > 0 && (!u_colidx || !u_vals)) return fail(PSK_ERR_ARG, "upper factor: NULL arrays");
    if (gather_in) PSK_TRY(check_perm(n, gather_in, "gather_in"));
    if (gather_out) PSK_TRY(check_perm(n, gather_out, "gather_out"));
    Context *c;
    PSK_TRY(ctx(&c));
    psk_prec *M = new psk_prec();
    M->kind = PSK_PREC_ILU;
    M->n = n;
    int rc = PSK_OK;
    // natural index of every factor row (the partitioned schedule's strips): L row r solves equation
    // gather_in[r]; U row gather_out[i] gives unknown i
    std::vector<int32_t> nat_l, nat_u;
    if (gather_in) nat_l.assign(gather_in, gather_in + n);
    if (gather_out) {
        nat_u.assign(n, 0);
        for (int64_t i = 0; i < n; ++i) nat_u[gather_out[i]] = (int32_t)i;
    }
    if (l_rowptr) rc = make_factor(c, n, l_rowptr, l_colidx, l_vals, false, l_unit != 0, nat_l, M->lo);
    if (rc == PSK_OK && u_rowptr) rc = make_factor(c, n, u_rowptr, u_colidx, u_vals, true, u_unit != 0, nat_u, M->up);
    std::vector<int32_t> gin, gout;
    if (gather_in) gin.assign(gather_in, gather_in + n);
    if (gather_out) gout.assign(gather_out, gather_out + n);
    if (rc == PSK_OK) rc = upload(&M->gather_in, gin);
    if (rc == PSK_OK) rc = upload(&M->gather_out, gout);
    if (rc == PSK_OK && n > 0 && hipMalloc(&M->work, (size_t)(3 * n) * sizeof(double)) != hipSuccess)
        rc = fail(PSK_ERR_ALLOC, "trisolve work");
    if (rc == PSK_OK && hipMalloc(&M->err, sizeof(int32_t)) != hipSuccess) rc = fail(PSK_ERR_ALLOC, "trisolve err");
    if (rc == PSK_OK && hipMemset(M->err, 0, sizeof(int32_t)) != hipSuccess) rc = fail(PSK_ERR_HIP, "trisolve err");
    if (rc != PSK_OK) {
        psk_prec_destroy(M);
        return rc;
    }
    *out = M;
    return PSK_OK;
}

// SuperLU ILU.solve: bb[perm_r[i]] = v[i]  <=>  bb[j] = v[pinv[j]];  out[i] = z[perm_c[i]]
extern "C" int psk_prec_create_ilu(int64_t n, const int32_t *l_rowptr, const int32_t *l_colidx, const double *l_vals,
                                   const int32_t *u_rowptr, const int32_t *u_colidx, const double *u_vals,
                                   const int32_t *perm_r, const int32_t *perm_c, psk_prec **out) {
    if (!out || n < 0 || !l_rowptr || !u_rowptr || !perm_r || !perm_c)
        return fail(PSK_ERR_ARG, "psk_prec_create_ilu: NULL argument");
    PSK_TRY(check_perm(n, perm_r, "ILU perm_r"));
    std::vector<int32_t> pinv(n);
    for (int64_t i = 0; i < n; ++i) pinv[perm_r[i]] = (int32_t)i;
    return psk_prec_create_trisolve(n, l_rowptr, l_colidx, l_vals, 1, u_rowptr, u_colidx, u_vals, 0, pinv.data(),
                                    perm_c, out);
}

extern "C" int psk_trisolve_grid_plan(int64_t n, const int32_t *rowptr, const int32_t *colidx, const double *vals,
                                      int32_t upper, int64_t *out) {
    if (n <= 0 || !rowptr || !colidx || !vals || !out) return fail(PSK_ERR_ARG, "psk_trisolve_grid_plan: bad arguments");
    HostFactor F;
    F.n = n;
    F.upper = upper != 0;
    std::vector<double> ova, dg;
    PSK_TRY(split_factor(n, rowptr, colidx, vals, upper == 0, false, F.rp, F.ci, ova, dg));
    GridPlan gp;
    plan_grid(F, gp);
    if (!gp.ok || n > kGridMaxRows)
        return fail(PSK_ERR_UNSUPPORTED, "psk_trisolve_grid_plan: factor is not a 2-D stencil (grid schedule)");
    const int64_t v[7] = {gp.w, gp.H, gp.sigma2, gp.phase, gp.off,
                          (gp.w - 1) + grid_g(gp.sigma2, gp.phase, kGridLanes - 1) - grid_g(gp.sigma2, gp.phase, 0) + 1,
                          (int64_t)gp.K};
    for (int i = 0; i < 7; ++i) out[i] = v[i];
    return PSK_OK;
}

extern "C" int psk_prec_trisolve_grid_info(const psk_prec *M, int32_t which, int64_t *out) {
    if (!M || M->kind != PSK_PREC_ILU || (which != 0 && which != 1) || !out)
        return fail(PSK_ERR_ARG, "psk_prec_trisolve_grid_info: not a triangular-solve chain / bad factor");
    const TriFactor &T = which == 0 ? M->lo : M->up;
    if (!T.present || T.grid_K == 0)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_grid_info: factor is not a 2-D stencil (grid schedule)");
    const int64_t v[7] = {T.grid_w, T.grid_H, T.grid_sigma, T.grid_phase, T.grid_off, T.grid_S, T.grid_dict_n};
    for (int i = 0; i < 7; ++i) out[i] = v[i];
    return PSK_OK;
}

extern "C" int psk_prec_trisolve_schedule(psk_prec *M, int32_t which, int32_t set, int32_t *schedule,
                                          int64_t *blocks, int32_t *ring_words, double *est_syncfree_us,
                                          double *est_band_us) {
    if (!M || M->kind != PSK_PREC_ILU || (which != 0 && which != 1))
        return fail(PSK_ERR_ARG, "psk_prec_trisolve_schedule: not a triangular-solve chain / bad factor");
    TriFactor &T = which == 0 ? M->lo : M->up;
    if (!T.present) return fail(PSK_ERR_ARG, "psk_prec_trisolve_schedule: factor absent");
    if (set == kSchedBand && T.band_K == 0)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_schedule: factor not eligible for the band schedule "
                                         "(more than 8 entries in a row or a level wider than a chunk)");
    if (set == kSchedLds && (M->n > kLdsMaxRows || M->n == 0))
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_schedule: factor too large for the LDS schedule");
    if (set == kSchedGrid && T.grid_K == 0)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_schedule: factor is not a 2-D stencil (grid schedule)");
    if (set == kSchedPart && T.part_P == 0)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_schedule: partitioned layout not built for this factor "
                                         "(built when chosen, or with PSK_TRISOLVE_PART=1 at creation)");
    if (set == kSchedLevel && T.lv_steps == 0)
        return fail(PSK_ERR_UNSUPPORTED, "psk_prec_trisolve_schedule: levels layout not built for this factor "
                                         "(built when chosen, or with PSK_TRISOLVE_LEVELS=1 at creation)");
    if (set >= kSchedSyncFree && set <= kSchedLevel) T.schedule = set;
    else if (set != -1) return fail(PSK_ERR_ARG, "psk_prec_trisolve_schedule: set must be -1 or 0..5");
    if (schedule) *schedule = T.schedule;
    if (blocks) *blocks = T.band_nblocks;
    if (ring_words) *ring_words = T.ring_words;
    if (est_syncfree_us) *est_syncfree_us = T.est_syncfree_us;
    if (est_band_us) *est_band_us = T.est_band_us;
    return PSK_OK;
}
