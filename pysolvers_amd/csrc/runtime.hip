// runtime.hip — error plumbing, per-device context, device-memory entry points.
#include "psk_internal.hpp"

#include <mutex>
#include <atomic>

namespace psk {

static thread_local std::string g_last_error;

void set_error(int code, const std::string &msg) {
    g_last_error = "psk error " + std::to_string(code) + ": " + msg;
}

int fail(int code, const std::string &msg) {
    set_error(code, msg);
    return code;
}

static std::mutex g_ctx_mu;
static Context g_ctx[64];
// set FIRST by psk_shutdown_ex (before anything is torn down), read without a lock by every entry point
static std::atomic<bool> g_shut{false};

bool lib_shut_down() { return g_shut.load(std::memory_order_acquire); }
static std::atomic<int> g_live_rccl{0};   // RCCL communicators alive (psk_comm_init .. psk_comm_destroy)
void rccl_comm_count(int delta) { g_live_rccl += delta; }

int solve_kit(Context *c, bool timed, SolveKit **out) {
    SolveKit &k = c->kit;
    if (!k.ready) {
        PSK_HIP(hipHostMalloc(&k.hmap, 64 * sizeof(int64_t), hipHostMallocCoherent));
        std::memset(k.hmap, 0, 64 * sizeof(int64_t));
        PSK_HIP(hipHostMalloc(&k.hstage, kStageBytes, hipHostMallocDefault));
        PSK_HIP(hipEventCreate(&k.ev0));
        PSK_HIP(hipEventCreate(&k.ev1));
        for (auto &e : k.fev) PSK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        PSK_HIP(hipEventCreateWithFlags(&k.ev_a, hipEventDisableTiming));
        PSK_HIP(hipEventCreateWithFlags(&k.ev_b, hipEventDisableTiming));
        k.ready = true;
    }
    if (timed && !k.timed_ready) {
        for (int i = 0; i < kTimedSlots; ++i) {
            // timing only: no system-scope fence at record (its L2 writeback of the SpMV's freshly
            // written y landed inside the bracket: +4-6 us per sampled launch at N = 10M against the
            // profiler's kernel time, profiles/r4_headline_regions_rocprof.json)
            PSK_HIP(hipEventCreateWithFlags(&k.ta[i], hipEventDisableSystemFence));
            PSK_HIP(hipEventCreateWithFlags(&k.tb[i], hipEventDisableSystemFence));
            for (hipEvent_t *e : {&k.ga[i], &k.gb[i], &k.ha[i], &k.hb[i]})
                PSK_HIP(hipEventCreateWithFlags(e, hipEventDisableSystemFence));
        }
        k.timed_ready = true;
    }
    *out = &k;
    return PSK_OK;
}

int comm_stream(Context *c, hipStream_t *out) {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (c->comm_stream == nullptr) PSK_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    *out = c->comm_stream;
    return PSK_OK;
}

int ctx(Context **out) {
    if (g_shut) return fail(PSK_ERR_ARG, "libpsk was shut down (psk_shutdown)");
    int dev = 0;
    PSK_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(PSK_ERR_ARG, "device index out of range");
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (g_shut) return fail(PSK_ERR_ARG, "libpsk was shut down (psk_shutdown)");
    Context &c = g_ctx[dev];
    if (c.stream == nullptr) {
        PSK_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        hipDeviceProp_t prop;
        PSK_HIP(hipGetDeviceProperties(&prop, dev));
        c.device = dev;
        c.num_cus = prop.multiProcessorCount;
        // 4 streaming 256-thread workgroups per CU (spmv_lab: 1024 workgroups beat 2048 for both the
        // SpMV and the 16-B/lane vector streams); partial arrays are sized for kMaxGrid
        int cap = c.num_cus * 4;
        c.grid_cap = cap < kMaxGrid ? cap : kMaxGrid;
        // keep the grid a multiple of 8 (XCD-aware tile mapping) when it is capped
        c.grid_cap -= c.grid_cap % 8;
        if (c.grid_cap < 8) c.grid_cap = 8;
    }
    *out = &c;
    return PSK_OK;
}

int DevBuf::ensure(size_t need) {
    if (need <= bytes && p != nullptr) return PSK_OK;
    if (p) {
        hipError_t e = hipFree(p);
        p = nullptr;
        bytes = 0;
        if (e != hipSuccess) return fail(PSK_ERR_HIP, std::string("hipFree: ") + hipGetErrorString(e));
    }
    if (need == 0) return PSK_OK;
    hipError_t e = hipMalloc(&p, need);
    if (e != hipSuccess) {
        p = nullptr;
        return fail(PSK_ERR_ALLOC, "hipMalloc(" + std::to_string(need) + "): " + hipGetErrorString(e));
    }
    bytes = need;
    return PSK_OK;
}

void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

__global__ void gridsum_arm_kernel(uint64_t *slots, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) slots[i] = kGridSumSentinel;
}

static int gridsum_arm(uint64_t **p, int64_t count, hipStream_t s) {
    PSK_HIP(hipMalloc(p, (size_t)count * sizeof(uint64_t)));
    hipLaunchKernelGGL(gridsum_arm_kernel, dim3((unsigned)((count + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, *p,
                       count);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

int gridsum_prepare(Context *c, int64_t nt, int W, double *out, GridSum *gs) {
    if (W < 1 || W > kGridSumMaxW || nt < 1)
        return fail(PSK_ERR_ARG, "gridsum_prepare: bad geometry");
    if (!c->gs_err) {
        PSK_HIP(hipMalloc(&c->gs_err, sizeof(int32_t)));
        PSK_HIP(hipMemsetAsync(c->gs_err, 0, sizeof(int32_t), c->stream));
        const size_t cb = (size_t)(kGridSumMaxGroups + 1) * kGridSumCntStride * sizeof(uint32_t);
        PSK_HIP(hipMalloc(&c->gs_cnt, cb));
        PSK_HIP(hipMemsetAsync(c->gs_cnt, 0, cb, c->stream));
        PSK_TRY(gridsum_arm(&c->gs_gslots, (int64_t)kGridSumMaxGroups * kGridSumMaxW, c->stream));
    }
    gs->out = out;
    gs->nt = nt;
    gs->grp_log2 = gridsum_grp_log2(nt);
    gs->ngroups = gridsum_ngroups(nt, gs->grp_log2);
    if (gs->ngroups > kGridSumMaxGroups) return fail(PSK_ERR_ARG, "gridsum_prepare: too many groups");
    gs->err = c->gs_err;
    gs->mb = nullptr;
    gs->mb_q = 0;
    gs->mb_P = 0;
    gs->gslots = c->gs_gslots;
    gs->cnt = c->gs_cnt;
    gs->slots = nullptr;
    if (gs->grp_log2 < 0) return PSK_OK;
    const int64_t need = (gs->ngroups << gs->grp_log2) * W;   // group-major slots (gridsum_slot)
    if (need > c->gs_cap) {
        int64_t cap = c->gs_cap > 0 ? c->gs_cap : (int64_t)1 << 20;
        while (cap < need) cap *= 2;
        uint64_t *p = nullptr;
        PSK_TRY(gridsum_arm(&p, cap, c->stream));
        if (c->gs_slots) c->gs_retired.push_back(c->gs_slots);
        c->gs_slots = p;
        c->gs_cap = cap;
    }
    gs->slots = c->gs_slots;
    return PSK_OK;
}

// Every ticket counter must be back at zero between launches: a launch that left one non-zero (a
// grid that differs from gs.nt, a tile that drew but never published, an aborted launch) would make
// every later reduction of that group skip its reducer silently. One workgroup scans the
// kGridSumMaxGroups + 1 counters and flags a non-zero one in gs_err (bit 4); cheap enough to run at
// the end of every solve.
__global__ __launch_bounds__(kBlock) void gridsum_counter_check_kernel(const uint32_t *cnt, int32_t *err) {
    uint32_t any = 0;
    for (int g = threadIdx.x; g <= kGridSumMaxGroups; g += kBlock) any |= cnt[(int64_t)g * kGridSumCntStride];
    if (__syncthreads_or(any != 0) && threadIdx.x == 0) atomicOr(err, 4);
}

int gridsum_check_enqueue(Context *c, int32_t *host_word) {
    if (!c->gs_err) {
        *host_word = 0;
        return PSK_OK;
    }
    hipLaunchKernelGGL(gridsum_counter_check_kernel, dim3(1), dim3(kBlock), 0, c->stream, c->gs_cnt, c->gs_err);
    PSK_HIP(hipGetLastError());
    PSK_HIP(hipMemcpyAsync(host_word, c->gs_err, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    return PSK_OK;
}

int gridsum_check_result(Context *c, int32_t h) {
    if (h == 0) return PSK_OK;
    PSK_HIP(hipMemsetAsync(c->gs_err, 0, sizeof(int32_t), c->stream));
    if (h & 4) {   // re-arm the counters so that later solves reduce again
        const size_t cb = (size_t)(kGridSumMaxGroups + 1) * kGridSumCntStride * sizeof(uint32_t);
        PSK_HIP(hipMemsetAsync(c->gs_cnt, 0, cb, c->stream));
    }
    PSK_HIP(hipStreamSynchronize(c->stream));
    if (h & 8) return fail(PSK_ERR_RCCL, "mailbox exchange: a rank's value did not arrive (2 s wait expired)");
    if (h & 2) return fail(PSK_ERR_HIP, "grid reduction: a launch's grid differs from the tiles it was prepared for");
    if (h & 4) return fail(PSK_ERR_HIP, "grid reduction: a ticket counter was left non-zero by a launch");
    return fail(PSK_ERR_HIP, "grid reduction: an issued partial-sum store never landed (1.3 s wait expired)");
}

int gridsum_check(Context *c) {
    if (!c->gs_err) return PSK_OK;
    SolveKit *k;
    PSK_TRY(solve_kit(c, false, &k));
    int32_t *h = reinterpret_cast<int32_t *>(static_cast<char *>(k->hstage) + kStageBytes - 64);
    PSK_TRY(gridsum_check_enqueue(c, h));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return gridsum_check_result(c, *h);
}

int to_device_vec(const double *src, int32_t loc, int64_t n, double *dst, hipStream_t s) {
    if (n <= 0) return PSK_OK;
    PSK_HIP(hipMemcpyAsync(dst, src, (size_t)n * sizeof(double),
                           loc == PSK_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice, s));
    return PSK_OK;
}

int from_device_vec(const double *src, int32_t loc, int64_t n, double *dst, hipStream_t s) {
    if (n <= 0) return PSK_OK;
    PSK_HIP(hipMemcpyAsync(dst, src, (size_t)n * sizeof(double),
                           loc == PSK_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice, s));
    return PSK_OK;
}

}  // namespace psk

using namespace psk;

extern "C" {

int psk_abi_version(void) { return PSK_ABI_VERSION; }

const char *psk_last_error(void) { return g_last_error.c_str(); }

int psk_device_count(int32_t *n) {
    if (!n) return fail(PSK_ERR_ARG, "n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *n = c;
    return PSK_OK;
}

int psk_set_device(int32_t dev) {
    PSK_HIP(hipSetDevice(dev));
    return PSK_OK;
}

int psk_synchronize(void) {
    Context *c;
    PSK_TRY(ctx(&c));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

int psk_dmalloc(int64_t bytes, void **dptr) {
    if (!dptr || bytes < 0) return fail(PSK_ERR_ARG, "psk_dmalloc: bad arguments");
    *dptr = nullptr;
    if (bytes == 0) return PSK_OK;
    hipError_t e = hipMalloc(dptr, (size_t)bytes);
    if (e != hipSuccess) return fail(PSK_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    return PSK_OK;
}

int psk_dfree(void *dptr) {
    if (g_shut) return PSK_OK;   // process exit: the runtime reclaims it
    if (dptr) PSK_HIP(hipFree(dptr));
    return PSK_OK;
}

// Drains every device's stream and releases what the library holds for the process lifetime (the
// SolveKit's host-mapped words, pinned staging and events, the gridsum arrays, the streams), while the
// HIP runtime is still fully alive. Python registers it with atexit (pysolvers_amd/_native.py) so that
// nothing of libpsk is left for the runtime's own static destructors at exit(); afterwards every
// entry point that needs a device fails with PSK_ERR_ARG and the destroy entry points are no-ops
// (objects still alive then are reclaimed with the process).
int psk_shutdown(void) { return psk_shutdown_ex(0); }

int psk_shutdown_ex(int32_t flags) {
    {
        // refuse new work first: ctx() (which tests the flag under the same lock) fails from here on, so no
        // context is created and no solve starts on one being torn down. The lock is not held below: a
        // running solve holds its context's solve_mu and may take g_ctx_mu (comm_stream).
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        if (g_shut.exchange(true, std::memory_order_acq_rel)) return PSK_OK;
    }
    int rc = PSK_OK;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int d = 0; d < 64; ++d) {
        Context &c = g_ctx[d];
        if (c.stream == nullptr) continue;
        if (hipSetDevice(d) != hipSuccess) continue;
        // a solve already running on this device (another thread) finishes before its streams, events and
        // staging go away
        std::lock_guard<std::mutex> solve_lk(c.solve_mu);
        if (hipStreamSynchronize(c.stream) != hipSuccess && rc == PSK_OK) rc = fail(PSK_ERR_HIP, "psk_shutdown: sync");
        if (c.comm_stream) (void)hipStreamSynchronize(c.comm_stream);
        SolveKit &k = c.kit;
        if (k.ready) {
            (void)hipEventDestroy(k.ev0);
            (void)hipEventDestroy(k.ev1);
            for (auto e : k.fev) (void)hipEventDestroy(e);
            (void)hipEventDestroy(k.ev_a);
            (void)hipEventDestroy(k.ev_b);
            (void)hipHostFree(k.hmap);
            (void)hipHostFree(k.hstage);
        }
        if (k.timed_ready)
            for (int i = 0; i < kTimedSlots; ++i) {
                (void)hipEventDestroy(k.ta[i]);
                (void)hipEventDestroy(k.tb[i]);
                for (hipEvent_t e : {k.ga[i], k.gb[i], k.ha[i], k.hb[i]}) (void)hipEventDestroy(e);
            }
        k = SolveKit{};
        for (uint64_t *p : c.gs_retired) (void)hipFree(p);
        c.gs_retired.clear();
        void *bufs[] = {c.gs_slots, c.gs_gslots, c.gs_cnt, c.gs_err};
        for (void *p : bufs)
            if (p) (void)hipFree(p);
        c.gs_slots = nullptr;
        c.gs_gslots = nullptr;
        c.gs_cnt = nullptr;
        c.gs_err = nullptr;
        c.gs_cap = 0;
        if (c.comm_stream) (void)hipStreamDestroy(c.comm_stream);
        (void)hipStreamDestroy(c.stream);
        c.comm_stream = nullptr;
        c.stream = nullptr;
        // hipDeviceReset only when the caller asks for it (PSK_SHUTDOWN_RESET_DEVICE; the Python binding
        // passes it only with PSK_SHUTDOWN_RESET=1): it destroys every allocation of the device, other HIP
        // users' in the process included. It is not what fixed the exit fault under rocprofv3 — dropping the
        // cooperative launches was (profiles/r4_exit_fault.txt:35: the reset changed nothing).
        if ((flags & PSK_SHUTDOWN_RESET_DEVICE) && g_live_rccl.load() == 0) (void)hipDeviceReset();
    }
    (void)hipSetDevice(cur);
    return rc;
}

int psk_h2d(void *dst, const void *src, int64_t bytes) {
    Context *c;
    PSK_TRY(ctx(&c));
    if (bytes <= 0) return PSK_OK;
    PSK_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

int psk_d2h(void *dst, const void *src, int64_t bytes) {
    Context *c;
    PSK_TRY(ctx(&c));
    if (bytes <= 0) return PSK_OK;
    PSK_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

int psk_dmemset0(void *dst, int64_t bytes) {
    Context *c;
    PSK_TRY(ctx(&c));
    if (bytes <= 0) return PSK_OK;
    PSK_HIP(hipMemsetAsync(dst, 0, (size_t)bytes, c->stream));
    PSK_HIP(hipStreamSynchronize(c->stream));
    return PSK_OK;
}

}  // extern "C"
