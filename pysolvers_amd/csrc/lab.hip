// lab.hip — libpsk_lab.so: test / lab entry points kept OUT of the product library (round 6).
// A separate shared library linked against libpsk.so (one instance of its state): a co-running kernel that holds
// CUs while a solve runs (the forward-progress tests, tests/test_gpu_progress.py), a dispatch probe and the
// enrolment count of the last sync-free triangular-solve launch. Declared in include/psk_lab.h; nothing in the
// product path calls them.
#include "psk_internal.hpp"
#include "../../include/psk_lab.h"

#include <chrono>
#include <string>

namespace psk {

// ---- lab: a co-running kernel that holds CUs while a solve runs (tests of the forward-progress rule) ----
// occupy_kernel: `wgs` workgroups of 1024 threads (16 waves each) with `lds` bytes of LDS each, on a
// stream of their own, every wave spinning until the flag is set on the solver's stream (occupy_end) or
// the time limit passes. A solve enqueued between begin and end can only use what the occupiers leave.
__global__ __launch_bounds__(1024) void occupy_kernel(uint32_t *flag, int64_t *started, uint64_t ticks,
                                                      int32_t *timed_out) {
    extern __shared__ unsigned char occ_lds[];
    if (threadIdx.x == 0) {
        occ_lds[0] = 1;
        __hip_atomic_fetch_add(started, (int64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // which XCD holds this occupier (HW_REG_XCC_ID, bits 3:0): psk_lab_occupy_xcc
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u;
        __hip_atomic_fetch_add(reinterpret_cast<uint32_t *>(timed_out) + 32 + xcc, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            if (threadIdx.x == 0) atomicOr(timed_out, 1);
            break;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}
__global__ void occupy_release_kernel(uint32_t *flag) {
    __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

namespace {
struct Occupier {
    hipStream_t s = nullptr;
    uint32_t *dw = nullptr;       // [0] release flag, [64] timed-out word
    int64_t *started = nullptr;   // host-mapped count of started occupier workgroups
    bool active = false;
};
Occupier g_occ;
}  // namespace

}  // namespace psk

extern "C" int psk_lab_occupy_begin(int32_t wgs, int32_t lds_bytes, double seconds) {
    using namespace psk;
    Context *c;
    PSK_TRY(ctx(&c));
    if (g_occ.active) return fail(PSK_ERR_ARG, "psk_lab_occupy_begin: already active");
    if (wgs < 1 || lds_bytes < 16 || lds_bytes > 160 * 1024 || seconds <= 0)
        return fail(PSK_ERR_ARG, "psk_lab_occupy_begin: bad arguments");
    if (!g_occ.s) {
        PSK_HIP(hipStreamCreateWithFlags(&g_occ.s, hipStreamNonBlocking));
        PSK_HIP(hipMalloc(&g_occ.dw, 128 * sizeof(uint32_t)));
        PSK_HIP(hipHostMalloc(&g_occ.started, 64, hipHostMallocCoherent));
    }
    PSK_HIP(hipMemsetAsync(g_occ.dw, 0, 128 * sizeof(uint32_t), g_occ.s));
    PSK_HIP(hipStreamSynchronize(g_occ.s));
    *reinterpret_cast<volatile int64_t *>(g_occ.started) = 0;
    const uint64_t ticks = (uint64_t)(seconds * 1e8);
    hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)wgs), dim3(1024), (size_t)lds_bytes, g_occ.s, g_occ.dw,
                       g_occ.started, ticks, reinterpret_cast<int32_t *>(g_occ.dw + 64));
    PSK_HIP(hipGetLastError());
    g_occ.active = true;
    // every occupier resident before the caller enqueues its solve (bounded: 5 s)
    const auto t0 = std::chrono::steady_clock::now();
    while (*reinterpret_cast<volatile int64_t *>(g_occ.started) < wgs &&
           std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5)) {
    }
    const int64_t got = *reinterpret_cast<volatile int64_t *>(g_occ.started);
    return got >= wgs ? PSK_OK : fail(PSK_ERR_HIP, "psk_lab_occupy_begin: only " + std::to_string(got) + " of " +
                                                       std::to_string(wgs) + " occupiers started");
}

// releases the occupiers behind everything enqueued on the solver's stream so far, waits for them;
// *timed_out = 1 when they hit their time limit first (the solve could not finish while they held CUs)
extern "C" int psk_lab_occupy_end(int32_t *timed_out) {
    using namespace psk;
    Context *c;
    PSK_TRY(ctx(&c));
    if (!g_occ.active) return fail(PSK_ERR_ARG, "psk_lab_occupy_end: not active");
    hipLaunchKernelGGL(occupy_release_kernel, dim3(1), dim3(1), 0, c->stream, g_occ.dw);
    PSK_HIP(hipGetLastError());
    PSK_HIP(hipStreamSynchronize(g_occ.s));
    int32_t h = 0;
    PSK_HIP(hipMemcpy(&h, g_occ.dw + 64, sizeof(int32_t), hipMemcpyDeviceToHost));
    g_occ.active = false;
    if (timed_out) *timed_out = h;
    return PSK_OK;
}

// lab: `nwg` workgroups of 128 threads holding `lds_bytes` of LDS each, each spinning `usec` and recording
// (start, end, XCD) in s_memrealtime ticks — is a launch that needs its workgroups recycled dispatched
// beside the occupiers? (the grid schedule's progress test)
__global__ void dispatch_probe_kernel(uint64_t ticks, int64_t *rec) {
    extern __shared__ unsigned char dp_lds[];
    if (threadIdx.x == 0) {
        dp_lds[0] = 1;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t t = t0;
        while (t - t0 < ticks) {
            __builtin_amdgcn_s_sleep(4);
            t = __builtin_amdgcn_s_memrealtime();
        }
        rec[3 * blockIdx.x + 0] = (int64_t)t0;
        rec[3 * blockIdx.x + 1] = (int64_t)t;
        rec[3 * blockIdx.x + 2] = (int64_t)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u);
    }
}

extern "C" int psk_lab_dispatch_probe(int32_t nwg, int32_t lds_bytes, double usec, int64_t *rec_out) {
    using namespace psk;
    if (nwg < 1 || lds_bytes < 16 || lds_bytes > 160 * 1024 || usec < 0 || !rec_out)
        return fail(PSK_ERR_ARG, "psk_lab_dispatch_probe: bad arguments");
    Context *c;
    PSK_TRY(ctx(&c));
    int64_t *rec = nullptr;
    PSK_HIP(hipMalloc(&rec, (size_t)nwg * 3 * sizeof(int64_t)));
    hipLaunchKernelGGL(dispatch_probe_kernel, dim3((unsigned)nwg), dim3(128), (size_t)lds_bytes, c->stream,
                       (uint64_t)(usec * 100.0), rec);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(rec_out, rec, (size_t)nwg * 3 * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(rec);   // (after the launch completed: the caller releases the occupiers afterwards)
    return e == hipSuccess ? PSK_OK : fail(PSK_ERR_HIP, hipGetErrorString(e));
}

// occupiers per XCD of the last psk_lab_occupy_begin (counts[8]; after psk_lab_occupy_end)
extern "C" int psk_lab_occupy_xcc(int32_t *counts) {
    using namespace psk;
    if (!counts || !g_occ.dw) return fail(PSK_ERR_ARG, "psk_lab_occupy_xcc: no occupiers yet");
    PSK_HIP(hipMemcpy(counts, g_occ.dw + 96, 8 * sizeof(int32_t), hipMemcpyDeviceToHost));
    return PSK_OK;
}

// workers (waves / 4) the last sync-free launch of a factor enrolled, and the grid it was launched with
extern "C" int psk_lab_trisolve_workers(const psk_prec *M, int32_t which, int32_t *enrolled, int32_t *grid) {
    using namespace psk;
    if (!M || M->kind != PSK_PREC_ILU) return fail(PSK_ERR_ARG, "psk_lab_trisolve_workers: not a triangular-solve chain");
    const TriFactor &T = which == 0 ? M->lo : M->up;
    if (!T.present || !T.sched) return fail(PSK_ERR_ARG, "psk_lab_trisolve_workers: factor absent");
    Context *c;
    PSK_TRY(ctx(&c));
    uint32_t v = 0;
    PSK_HIP(hipStreamSynchronize(c->stream));
    PSK_HIP(hipMemcpy(&v, T.sched + kSchedLast, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (enrolled) *enrolled = (int32_t)v;
    if (grid) *grid = syncfree_grid(c);
    return PSK_OK;
}

extern "C" int psk_lab_amg_gs_pair(psk_prec *M, int32_t set, int32_t *levels_on, int32_t *levels_eligible) {
    using namespace psk;
    if (set < -1 || set > 1) return fail(PSK_ERR_ARG, "psk_lab_amg_gs_pair: set must be -1, 0 or 1");
    Context *c;
    PSK_TRY(ctx(&c));
    PSK_HIP(hipStreamSynchronize(c->stream));   // queued applies keep the setting they were enqueued with
    int on = 0, el = 0;
    PSK_TRY(amg_gs_pair(M, set, &on, &el));
    if (levels_on) *levels_on = on;
    if (levels_eligible) *levels_eligible = el;
    return PSK_OK;
}

// the probe's writer: dst = src with 16-B accesses (the shape of K3 writing p_{k+1}, which the next SpMV gathers)
__global__ __launch_bounds__(256) void lab_copy_kernel(int64_t n, const double *__restrict__ src, double *__restrict__ dst) {
    const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (i + 1 < n) {
        const double2 v = *reinterpret_cast<const double2 *>(src + i);
        *reinterpret_cast<double2 *>(dst + i) = v;
    } else if (i < n) {
        dst[i] = src[i];
    }
}

extern "C" int psk_lab_spmv_rotate(const psk_csr *A, const double *const *xs, double *const *ys, int32_t nbuf,
                                   int32_t reps, int32_t dot, double *avg_ms) {
    using namespace psk;
    if (!A || !xs || !ys || nbuf < 1 || reps < 1 || !avg_ms) return fail(PSK_ERR_ARG, "psk_lab_spmv_rotate: bad arguments");
    if (A->comm) return fail(PSK_ERR_UNSUPPORTED, "psk_lab_spmv_rotate: sharded matrix");
    for (int32_t i = 0; i < nbuf; ++i)
        if (!xs[i] || !ys[i]) return fail(PSK_ERR_ARG, "psk_lab_spmv_rotate: NULL buffer");
    Context *c;
    PSK_TRY(ctx(&c));
    hipEvent_t e0, e1;
    PSK_HIP(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
    PSK_HIP(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    const int mode = dot ? kSpmvDot : kSpmvPlain;
    DevBuf part;
    int rc = part.ensure(64);
    double *pp = dot ? part.as<double>() : nullptr;
    for (int32_t i = 0; i < nbuf && rc == PSK_OK; ++i)   // warm: every pair once
        rc = launch_spmv(A, mode, xs[i], ys[i], nullptr, nullptr, pp, nullptr, c->stream);
    if (rc == PSK_OK && hipEventRecord(e0, c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "event record");
    for (int32_t r = 0; r < reps && rc == PSK_OK; ++r)
        rc = launch_spmv(A, mode, xs[r % nbuf], ys[r % nbuf], nullptr, nullptr, pp, nullptr, c->stream);
    if (rc == PSK_OK && hipEventRecord(e1, c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "event record");
    float ms = 0.f;
    if (rc == PSK_OK && hipEventSynchronize(e1) != hipSuccess) rc = fail(PSK_ERR_HIP, "event sync");
    if (rc == PSK_OK && hipEventElapsedTime(&ms, e0, e1) != hipSuccess) rc = fail(PSK_ERR_HIP, "event time");
    (void)hipStreamSynchronize(c->stream);   // before `part` is freed
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    part.release();
    if (rc == PSK_OK) *avg_ms = (double)ms / reps;
    return rc;
}

extern "C" int psk_lab_spmv_after_write(const psk_csr *A, double *x, double *y, const double *src, double *scratch,
                                        int32_t target, int32_t reps, int32_t dot, double *avg_ms) {
    using namespace psk;
    if (!A || !x || !y || !src || !scratch || reps < 1 || reps > 256 || !avg_ms)
        return fail(PSK_ERR_ARG, "psk_lab_spmv_after_write: bad arguments");
    if (A->comm || A->ncols != A->n) return fail(PSK_ERR_UNSUPPORTED, "psk_lab_spmv_after_write: square unsharded only");
    Context *c;
    PSK_TRY(ctx(&c));
    std::vector<hipEvent_t> ea((size_t)reps), eb((size_t)reps);
    for (int32_t r = 0; r < reps; ++r) {
        PSK_HIP(hipEventCreateWithFlags(&ea[(size_t)r], hipEventDisableSystemFence));
        PSK_HIP(hipEventCreateWithFlags(&eb[(size_t)r], hipEventDisableSystemFence));
    }
    const int mode = dot ? kSpmvDot : kSpmvPlain;
    DevBuf part;
    int rc = part.ensure(64);
    double *pp = dot ? part.as<double>() : nullptr;
    const int64_t n = A->n;
    const unsigned g = (unsigned)((n + 511) / 512);
    double *dst = target == 1 ? x : scratch;   // 1: the writer writes the SpMV's x (as K3 writes p); 2: another buffer
    rc = launch_spmv(A, mode, x, y, nullptr, nullptr, pp, nullptr, c->stream);   // warm
    for (int32_t r = 0; r < reps && rc == PSK_OK; ++r) {
        if (target > 0) {
            hipLaunchKernelGGL(lab_copy_kernel, dim3(g), dim3(256), 0, c->stream, n, src, dst);
            if (hipGetLastError() != hipSuccess) rc = fail(PSK_ERR_HIP, "lab copy");
        }
        if (rc == PSK_OK)
            rc = launch_spmv(A, mode, x, y, nullptr, nullptr, pp, nullptr, c->stream, ea[(size_t)r], eb[(size_t)r]);
    }
    double tot = 0.0;
    if (rc == PSK_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "sync");
    for (int32_t r = 0; r < reps && rc == PSK_OK; ++r) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ea[(size_t)r], eb[(size_t)r]) != hipSuccess) rc = fail(PSK_ERR_HIP, "event time");
        tot += ms;
    }
    (void)hipStreamSynchronize(c->stream);
    for (int32_t r = 0; r < reps; ++r) {
        (void)hipEventDestroy(ea[(size_t)r]);
        (void)hipEventDestroy(eb[(size_t)r]);
    }
    part.release();
    if (rc == PSK_OK) *avg_ms = tot / reps;
    return rc;
}
