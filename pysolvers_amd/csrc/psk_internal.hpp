// psk_internal.hpp — shared types, error plumbing and device helpers of libpsk.so (gfx950).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/psk.h"

namespace psk {

// ---------------------------------------------------------------------------------------------
// launch geometry (CDNA4: 64-wide waves, 256 CUs in 8 XCDs)
constexpr int kBlock = 256;            // threads per workgroup = 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kChunk = 1280;           // SpMV LDS-staged products per chunk (10 KiB of f64) = 256 FD rows
constexpr int kMaxGrid = 2048;         // 256 CUs x 8 resident workgroups; partial arrays sized for it
constexpr int kVecTile = 2 * kBlock;   // elementwise tile: 2 doubles (16 B) per lane
// largest nnz of a device CSR: the CSR SpMV kernel forms entry indices e0 + k*kBlock + tid and the
// next chunk start in int32, which must stay below INT32_MAX in every tile
constexpr int64_t kMaxNnz = (int64_t)INT32_MAX - kChunk - kBlock;

// ---------------------------------------------------------------------------------------------
// errors
void set_error(int code, const std::string &msg);
int fail(int code, const std::string &msg);
const char *hip_err_str(hipError_t e);

#define PSK_HIP(call)                                                                         \
    do {                                                                                      \
        hipError_t _e = (call);                                                               \
        if (_e != hipSuccess)                                                                 \
            return ::psk::fail(PSK_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define PSK_RCCL(call)                                                                           \
    do {                                                                                         \
        ncclResult_t _r = (call);                                                                \
        if (_r != ncclSuccess)                                                                   \
            return ::psk::fail(PSK_ERR_RCCL, std::string(#call) + ": " + ncclGetErrorString(_r)); \
    } while (0)

#define PSK_TRY(call)              \
    do {                           \
        int _rc = (call);          \
        if (_rc != PSK_OK) return _rc; \
    } while (0)

// ---------------------------------------------------------------------------------------------
// per-process device context: one non-blocking stream per device
constexpr int kPollSlots = 4;     // solve-loop poll events (lag L = 2 chunks, L + 2 in flight)
constexpr int kTimedSlots = 64;   // sampled SpMV timing event pairs of one solve
// Host-side resources every solve reuses, created on a device's first solve and released only by
// psk_shutdown (round 4): before, each psk_pcg/psk_gmres call paid hipHostMalloc + hipHostFree (which
// synchronises the device) and up to 2 x 64 + 6 event creations, ~0.5 ms per call at N = 10M
// (VERDICT r3 weak #3). One solve at a time per device: `solve_mu` is held by psk_pcg/psk_gmres.
struct SolveKit {
    bool ready = false;
    uint64_t solve_gen = 0;       // PCG solves started (tags the done stamps, pcg.hip set_done)
    int64_t *hmap = nullptr;      // host-mapped coherent words the kernels write (PCG done stamp at [0])
    void *hstage = nullptr;       // pinned staging for the end-of-solve state / error-word copies (4 KiB)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;   // loop_ms (timing)
    hipEvent_t fev[kPollSlots] = {};           // poll chunks (no timing)
    hipEvent_t ev_a = nullptr, ev_b = nullptr; // halo overlap hand-offs (no timing)
    bool timed_ready = false;
    hipEvent_t ta[kTimedSlots] = {}, tb[kTimedSlots] = {};   // sampled SpMV intervals (timing)
    // sharded solves (ABI 4): the sampled iterations' p.Ap gather and halo exchange (timing)
    hipEvent_t ga[kTimedSlots] = {}, gb[kTimedSlots] = {}, ha[kTimedSlots] = {}, hb[kTimedSlots] = {};
};
constexpr size_t kStageBytes = 4096;
struct Context {
    int device = -1;
    hipStream_t stream = nullptr;
    int num_cus = 256;
    int grid_cap = kMaxGrid;
    // gridsum slots (below): one armed array per stream, grow-only; outgrown arrays are kept until
    // exit because queued launches may still use them
    uint64_t *gs_slots = nullptr;
    int64_t gs_cap = 0;
    uint64_t *gs_gslots = nullptr;   // kGridSumMaxGroups * kGridSumMaxW
    uint32_t *gs_cnt = nullptr;      // gridsum ticket counters (zero between launches)
    std::vector<uint64_t *> gs_retired;
    int32_t *gs_err = nullptr;
    hipStream_t comm_stream = nullptr;   // halo exchanges overlapped with compute (created lazily)
    SolveKit kit;
    std::mutex solve_mu;
};
int ctx(Context **out);   // current device's context (created lazily)
int comm_stream(Context *c, hipStream_t *out);
// the context's SolveKit, created on first use (with the SpMV timing events when `timed`)
int solve_kit(Context *c, bool timed, SolveKit **out);
// true once psk_shutdown ran: destroy entry points become no-ops (the process is exiting)
bool lib_shut_down();
void rccl_comm_count(int delta);   // live RCCL communicators (psk_shutdown_ex resets the device only at 0)

// ---------------------------------------------------------------------------------------------
// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need);
    void release();
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// halo exchange plan of a row-block sharded matrix: local vector layout [owned | halo]
struct HaloPeer {
    int rank;
    int64_t send_count;   // owned entries we send to this peer
    int64_t recv_count;   // halo entries we receive from it
    int64_t recv_offset;  // offset inside the halo region
    int32_t *send_idx;    // device: owned local indices to pack (nullptr when contiguous); points
                          // into psk_csr::pack_idx (not owned)
    int64_t send_begin;   // contiguous owned range start when send_idx == nullptr
    int64_t pack_off;     // offset of this peer's packed segment in pack_idx / sendbuf
};

struct ShmComm;
struct DenseInverse;
// largest dense coarse inverse (psk_prec_create_dense_inverse): 32768^2 doubles = 8.6 GB
constexpr int64_t kDenseMaxN = 32768;

// Device-side exchange of the solvers' per-rank scalars through a host-shared mailbox (dist.hip,
// psk_comm_mailbox; round 5): the kernel that finishes a rank's grid sums stores them straight into
// every rank's slot of the exchange (system-scope stores to pinned host memory mapped by all ranks of
// the node), and a one-wave kernel on each rank waits for the P values of its own slot, copies them to
// the gathered array the solver sums in rank order and re-arms the slot. Slot index (reader q, ring
// position e mod kMbRing of exchange e, writer r, component c): ((q*kMbRing + e%kMbRing)*P + r)*kMbW + c.
constexpr int kMbRing = 4;
constexpr int kMbW = 2;
struct Mailbox {
    std::string name;
    char *host = nullptr;     // the mapped segment (4 KiB header, then the slots)
    size_t bytes = 0;
    uint64_t *dev = nullptr;  // device address of the slots
    int P = 1, rank = 0;
    uint64_t seq = 0;         // exchanges issued on this communicator (identical on every rank)
};
}  // namespace psk

struct psk_comm {
    int nranks = 1;
    int rank = 0;
    int device = 0;
    ncclComm_t nccl = nullptr;
    bool dry = false;     // psk_comm_init_dry: builds shards, no collectives (single-GPU validation)
    psk::ShmComm *shm = nullptr;   // psk_comm_init_host: shared-memory transport (shmcomm.hip)
    psk::Mailbox *mb = nullptr;    // psk_comm_mailbox: device-side scalar exchange (dist.hip)
};

namespace psk {
// shared-memory transport (shmcomm.hip): stream-ordered like the RCCL calls they stand in for
int shm_allgather(psk_comm *c, const double *send, double *recv, int64_t count, hipStream_t s);
int shm_exchange(psk_comm *c, int npeers, const int *peers, const double *const *sends, const int64_t *send_counts,
                 double *const *recvs, const int64_t *recv_counts, hipStream_t s);
int shm_allgather_host(psk_comm *c, const void *mine, void *all, size_t bytes);
int shm_exchange_host(psk_comm *c, int npeers, const int *peers, const void *const *sends, const size_t *send_bytes,
                      void *const *recvs, const size_t *recv_bytes);
int shm_error(const psk_comm *c);
void shm_close(psk_comm *c);
}  // namespace psk

struct psk_csr {
    int64_t n = 0;        // local (owned) rows
    int64_t ncols = 0;    // local columns = n + halo
    int64_t nnz = 0;
    int tile_rows = 256;  // SpMV rows per tile (psk::tile_rows_for)
    int32_t *rowptr = nullptr;
    int32_t *colidx = nullptr;
    double *vals = nullptr;
    int device = 0;
    // sliced copy of the same entries (spmv.hip, "sliced layout"): slices of kSlice rows, slot-major
    // inside a slice (values in slot pairs, or byte indices into sl_dict), per slice either packed
    // int16 column-delta pairs (sl_fmt[t] = 1) or int32 columns (sl_col); sl_col and sl_val are
    // addressed from the slice's slot offset sl_off[t], the word stream sl_pcol (packed columns,
    // then value indices) from sl_woff[t]. Present when the SpMV uses it (psk_csr_layout); the CSR
    // arrays above are always kept.
    int64_t *sl_off = nullptr;   // [nslices + 1] slot offsets
    int64_t *sl_woff = nullptr;  // [nslices + 1] word offsets into sl_pcol (packed columns, value indices)
    int8_t *sl_fmt = nullptr;    // [nslices] 1 = packed (int16 deltas)
    int32_t *sl_col = nullptr;   // nullptr when every slice is packed
    int32_t *sl_pcol = nullptr;  // word stream: 2 int16 deltas per word, then 4 value indices per word
    double *sl_val = nullptr;    // values (nullptr with a dictionary)
    double *sl_dict = nullptr;   // value dictionary (<= 8 distinct values, padded to 8), nullptr = none
    int32_t sl_dict_n = 0;
    int32_t sl_uniform_w = 0;    // > 0: every slice this wide and packed (offsets computed, not loaded)
    int32_t sl_compact = 0;      // uniform, odd width, <= 2 dictionary values: the value-index bits sit in
                                 // the last delta word's free half (no index words; spmv_uniform_kernel CMP)
    int64_t sl_slots = 0, sl_packed_slots = 0, sl_stream_bytes = 0;
    // diagonal layout (spmv.hip, "diagonal layout"; round 5): every row's entries lie, in stored order, on
    // a subsequence of dg_K <= 8 diagonals c = row + dg_d[j] (columns outside [0, n) of a row-block shard
    // mapped to its halo by dg_lo / dg_hi) with ONE value dg_v[j] per diagonal; per row a presence mask
    // byte (dg_mask, padded to whole 256-row slices). Present instead of the sliced copy when it applies.
    uint8_t *dg_mask = nullptr;
    int32_t dg_K = 0, dg_jd = -1;     // jd: the diagonal d = 0 (-1: none)
    int32_t dg_d[8] = {};
    double dg_v[8] = {};
    int64_t dg_lo = 0, dg_hi = 0;
    // distributed
    psk_comm *comm = nullptr;
    int64_t n_global = 0, row_begin = 0, row_end = 0;
    std::vector<psk::HaloPeer> peers;
    psk::DevBuf sendbuf;  // packed halo sends
    int32_t *pack_idx = nullptr;   // device: the packed peers' send indices, concatenated
    int64_t pack_count = 0;
    std::vector<int64_t> halo_cols;   // global index of each halo column, in local order
    // per-matrix solver workspace (grow-only)
    psk::DevBuf ws;
    psk::DevBuf ws_small;
};

namespace psk {
struct AmgHierarchy;

// One sparse triangular factor on the device: off-diagonal entries in stored order (lower or
// upper implied by the solve direction), diagonal (nullptr = unit), and two schedules built on
// the host at creation (ilu.hip):
//  * sync-free: rows dealt to waves in dependency-level order (`order`, `levels` global levels);
//  * band: solve order cut into `band_nblocks` contiguous blocks of `band_B` rows, one workgroup
//    per block walking the block's LOCAL levels (dependencies inside the block) with a barrier
//    between levels; dependencies on earlier blocks are waited on through the published values;
//    an LDS ring of `ring_words` doubles (0 = none) serves the in-block dependencies.
//  * LDS: small factors (x fits LDS) solved by one workgroup, sync-free inside it with x in LDS.
//  * grid: factors whose dependencies form a 2-D stencil in solve order (grid_w positions per line,
//    every dependency (lines back, positions back) within 63 lines and skewable):
//    one wave per band of 64 lines, all 64 lines advancing together along the skewed coordinate
//    u = x + g(y), g(y) = (grid_sigma * y + grid_phase) >> 1 (grid_sigma is TWICE the skew, so a
//    half-integer skew is an odd grid_sigma), in-band dependencies through an LDS ring of the last
//    grid_ring steps, only
//    the band above through published values (sptrsv_grid_kernel).
//  * part: rows cut into strips of their natural index, one workgroup per strip (per CU), the
//    strip's own dependencies through an LDS cache, the others through published values
//    (sptrsv_part_kernel).
// `schedule` picks one (kSchedSyncFree / kSchedBand / kSchedLds / kSchedGrid / kSchedPart), chosen by host
// cost models.
enum TriSchedule : int { kSchedSyncFree = 0, kSchedBand = 1, kSchedLds = 2, kSchedGrid = 3, kSchedPart = 4,
                         kSchedLevel = 5 };
constexpr int kGridMaxPE = 8;   // distinct dependency patterns reaching into the band above
struct GridExt {
    int32_t delta[kGridMaxPE];  // pattern code: ud * 64 + yd (steps back, lines back)
    int32_t yd[kGridMaxPE];     // lines back
};
// words of a factor's scheduling array (TriFactor::sched, ilu.hip): block tickets, publication counters, the
// exit count and the workers the last sync-free launch enrolled, each on its own 256-B line
constexpr int kSchedTicket = 0, kSchedPub = 64, kSchedExit = 128, kSchedLast = 192, kSchedWords = 256;
// the grid of a sync-free triangular-solve launch (ilu.hip)
int syncfree_grid(const Context *c);
struct TriFactor {
    bool present = false, upper = false;
    int64_t nnz = 0;
    int32_t *rowptr = nullptr, *colidx = nullptr;
    double *vals = nullptr, *diag = nullptr;
    int32_t *order = nullptr;
    int64_t levels = 0;
    int schedule = kSchedSyncFree;
    // band record stream (n records, block by block in local-level order; SoA, K entries each)
    int32_t *rec_row = nullptr, *rec_end = nullptr, *rec_c = nullptr;
    double *rec_v = nullptr, *rec_d = nullptr;
    int band_K = 0;
    int64_t band_B = 0, band_nblocks = 0, band_levels = 0;
    int32_t ring_words = 0;
    bool band_narrow = false;   // band run by sptrsv_band_narrow_kernel (local levels <= one wave wide)
    // grid records in solve order q: K pattern codes (uint16, 0xFFFF = padding) and K values per row
    // (row-major, stored entry order), diagonal (nullptr = unit)
    uint16_t *gd_code = nullptr;
    double *gd_coef = nullptr, *gd_diag = nullptr;
    // record dictionary (grid_dict_n > 0): every lane-step's record is one of grid_dict_n distinct
    // (codes, values, diagonal) records, gd_dict = [n][K] values, [n] diagonals, then [n][K/2] code
    // words; gd_idx = the record index of each lane-step in the solver's access order
    uint32_t *gd_idx = nullptr;
    double *gd_dict = nullptr;
    int grid_dict_n = 0;
    int32_t *grid_flag = nullptr;   // dictionary kernel: a step's quotient needed the IEEE re-solve (zeroed after it)
    uint32_t *sched = nullptr;      // block tickets / worker enrolment of the spin-waiting schedules (ilu.hip)
    int grid_K = 0, grid_pe = 0, grid_maxyd = 0, grid_ring = 0;
    int64_t grid_w = 0, grid_H = 0, grid_S = 0;   // grid_S: steps per band (slot stride)
    int64_t grid_sigma = 0, grid_phase = 0;      // g(y) = (grid_sigma * y + grid_phase) >> 1 (twice the skew)
    int64_t grid_off = 0;   // empty grid positions before the first row (a partial first line)
    GridExt grid_ext{};
    // part layout: position k = part_seg[w] + q (workgroup w's q-th row); rows, entries (codes) in it
    int64_t *part_seg = nullptr;
    int32_t *part_rp = nullptr, *part_code = nullptr, *part_row = nullptr;
    double *part_va = nullptr;
    int part_P = 0;
    // levels layout (round 5, sptrsv_levels_kernel): ONE workgroup of lv_W lanes, a dependency level (or a
    // lv_W-row piece of one) per step behind a barrier, x in lv_R LDS slots the host assigns (a value's slot
    // is free again after the step of its last reader; slot lv_R holds 0.0, slot lv_R + 1 takes the values
    // nobody reads). Per step s and lane t (field-major, coalesced): lv_rc = row | (write slot << 40)
    // (row 0xFFFFFFFF: idle lane), lv_sl = slots of the entries, four uint16 per word (padding: slot lv_R),
    // lv_cf = coefficients in stored order (padding -0.0), two per 16 bytes, lv_dg = diagonal (1.0 for a
    // unit factor), lv_b = the right-hand side gathered into step order before each solve
    uint64_t *lv_rc = nullptr;
    uint64_t *lv_sl = nullptr;
    double *lv_cf = nullptr, *lv_dg = nullptr, *lv_b = nullptr;
    int64_t lv_steps = 0;
    int lv_W = 0, lv_R = 0, lv_KM = 0;
    double est_syncfree_us = 0.0, est_band_us = 0.0, est_lds_us = -1.0, est_grid_us = -1.0, est_part_us = -1.0;
    double est_level_us = -1.0;
    // 5-point grid signature of an upper factor (make_factor; amg.hip's paired Gauss-Seidel sweeps): n = fd5_m * H,
    // row i's off-diagonal entries exactly columns i + 1 (i % m < m - 1) and i + m (i + m < n), values fd5_a1 / fd5_am,
    // every diagonal fd5_d, fd5_mfirst = the +m entry stored before the +1 entry. fd5_m = 0: no such signature.
    int64_t fd5_m = 0;
    double fd5_d = 0.0, fd5_a1 = 0.0, fd5_am = 0.0;
    int fd5_mfirst = 0;
    void release();
};
}  // namespace psk

struct psk_prec {
    int kind = PSK_PREC_IDENTITY;
    int64_t n = 0;
    double *dinv = nullptr;   // JACOBI
    bool dinv_uniform = false;   // every DInv entry the same bits (constant diagonal): PCG reads dinv_value
    double dinv_value = 0.0;
    // PSK_PREC_ILU = triangular-solve chain: out = (U^-1 L^-1 v[gather_in])[gather_out]
    psk::TriFactor lo, up;
    int32_t *gather_in = nullptr, *gather_out = nullptr;
    double *work = nullptr;   // 2n: y, z
    int32_t *err = nullptr;
    psk::AmgHierarchy *amg = nullptr;   // PSK_PREC_AMG
    psk::DenseInverse *dense = nullptr; // PSK_PREC_DENSE (dense.hip)
};

namespace psk {

// ---------------------------------------------------------------------------------------------
// device-side reduction helpers (deterministic: fixed order for a fixed grid)

__device__ __forceinline__ double wave_sum(double v) {
    // butterfly: every lane ends with the same bits (IEEE add is commutative)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// One DPP step on a double (both halves moved by the same lane pattern CTRL)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Wave total without LDS traffic: DPP inside each 16-lane row (pairs, quads, then row_ror 4 and 8,
// after which lane 0 of a row holds ((Q0+Q3)+(Q2+Q1)) of its four quad sums), then the four row
// totals read from lanes 0/16/32/48 and added in that order. Fixed order; the result is uniform
// (scalar) across the wave. Used where only one lane publishes the sum (the SpMV dot epilogue): a
// butterfly of ds_bpermute shuffles holds each wave longer at the end of its slice.
__device__ __forceinline__ double wave_total(double v) {
    v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_f64<0x124>(v);   // row_ror:4
    v += dpp_f64<0x128>(v);   // row_ror:8
    auto lane = [](double x, int l) {
        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                                __builtin_amdgcn_readlane(__double2loint(x), l));
    };
    return ((lane(v, 0) + lane(v, 16)) + lane(v, 32)) + lane(v, 48);
}

// Block-wide sum; all threads get the same value. `sh` must hold kWaves doubles.
__device__ __forceinline__ double block_sum(double v, double *sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    double r = sh[0];
#pragma unroll
    for (int i = 1; i < kWaves; ++i) r += sh[i];
    return r;
}

// block_sum of two values at once: each gets exactly block_sum's butterflies and wave-order sum (the same bits as
// two calls), with one barrier pair instead of two and the two butterflies interleaved. `sh` holds 2 * kWaves doubles.
__device__ __forceinline__ void block_sum2(double &a, double &b, double *sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        sh[2 * w] = a;
        sh[2 * w + 1] = b;
    }
    __syncthreads();
    double ra = sh[0], rb = sh[1];
#pragma unroll
    for (int i = 1; i < kWaves; ++i) {
        ra += sh[2 * i];
        rb += sh[2 * i + 1];
    }
    a = ra;
    b = rb;
}

// Sum over the ranks of a gathered [nparts][W] array, component c, in rank order: every rank of a
// sharded solve gets the same bits from its allgather'd copy (nparts == 1: the value itself).
__device__ __forceinline__ double rank_sum(const double *g, int nparts, int W, int c) {
    double s = g[c];
    for (int q = 1; q < nparts; ++q) s += g[q * W + c];
    return s;
}

// Sum of np partials laid out with `stride` (identical bits in every workgroup).
__device__ __forceinline__ double reduce_partials(const double *part, int np, int stride, double *sh) {
    double v = 0.0;
    for (int i = threadIdx.x; i < np; i += kBlock) v += part[(int64_t)i * stride];
    return block_sum(v, sh);
}

// ---------------------------------------------------------------------------------------------
// One-shot launches and their deterministic grid reduction ("gridsum").
//
// The streaming kernels (SpMV, PCG K2/K3) run ONE TILE PER WORKGROUP, grid = tiles: no workgroup
// carries loop state and the chip sweeps a compact window of every stream (tools/spmv_lab.hip /
// tools/stream_lab.hip at n = 268M: SpMV +5%, the K2 access shape +7% over persistent grids; SpMV
// +7-10% at n = 10-17M). Their dot products are finished inside the same launch, deterministically,
// without data atomics, and no workgroup ever waits for one that has not started — so the protocol
// holds whatever the dispatch order, the workgroup->XCD placement or the co-resident kernels (HIP
// promises none of them, MI355X_MICROARCH.md "Contract [G]"):
//  1. a tile's workgroup draws a TICKET when it starts: one returning agent-scope atomic add by
//     lane 0 of wave 0 on its group's counter, issued once the tile's stream loads are in flight
//     (the return hides behind them; it is read at the end). Groups interleave tiles — group l of
//     a superblock holds tiles l, l+256, l+512, ... — so the tickets drawn at any moment spread
//     over 256 counters, each on its own 256-B line (one word takes ~88 atomics/us; the SpMV at
//     16384^2 starts ~580 tiles/us).
//  2. at its end every SLOT of the tile — the workgroup, or each of its waves for the *_wave
//     variant (no workgroup barrier) — publishes its W partials with agent-scope (sc1) 8-byte
//     stores into slots armed with a signalling-NaN sentinel (value-is-flag; MI355X_MICROARCH.md
//     handoff granule).
//  3. the tile holding its group's LAST ticket (its wave 0) sums the group's slots in order: every
//     other member tile drew its ticket earlier, so all its waves are resident (a workgroup's waves
//     are created together) and running, and producers never wait, so every slot it polls is
//     written by a store that will land. It re-arms the slots, resets the counter, publishes the
//     group sum the same way, then draws a ticket on the final counter.
//  4. the group reducer holding the final counter's last ticket sums the group sums in group order
//     into out[0..W) (again only already-issued stores are awaited) and resets that counter.
// Launches of at most kBlock tiles skip the group stage: every slot publishes into the group-sum
// slots and draws the final ticket at its end. The summation order depends on the tile and slot
// indices only: sums are bitwise reproducible run to run, and equal across kernels that publish
// over the same tiles and slots (the SpMV layouts).
constexpr int kGridSumLLog = 8;
constexpr int64_t kGridSumL = (int64_t)1 << kGridSumLLog;   // groups interleaved per superblock
// counters one per 256-B line: atomics to one line serialise at its memory channel (64 counters
// packed in 256 B, one ticket per wave, put the SpMV at ~800 tickets/us: in-loop SpMV 1.8 -> 6.8 ms
// at 16384^2)
constexpr int kGridSumCntStride = 64;
constexpr uint64_t kGridSumSentinel = 0x7FF0000000000001ull;   // sNaN: arithmetic never produces it
constexpr int kGridSumMaxW = 4;
constexpr int64_t kGridSumMaxGroups = kMaxGrid;
// a wait on an already-issued store that has not landed after ~1.3 s (s_memrealtime, 100 MHz) is
// reported (gridsum_check) instead of hanging the launch: never expected
constexpr uint64_t kGridSumWaitTicks = (uint64_t)1 << 27;

struct GridSum {
    uint64_t *slots;    // W partials per tile, group-major (two-level launches)
    uint64_t *gslots;   // ngroups*W group sums (one-level: the slots themselves)
    uint32_t *cnt;      // counter g at cnt[g * kGridSumCntStride] (g < kGridSumMaxGroups), the final one at
                        // g = kGridSumMaxGroups; zero between launches
    double *out;        // the W grid sums
    int64_t nt;         // tiles (workgroups) of the launch
    int64_t ngroups;    // groups of tiles (one-level: nt)
    int32_t grp_log2;   // tiles of a full group = 2^grp_log2; -1 = one level (nt <= kBlock)
    int32_t *err;       // set when a wait expires (reported by gridsum_check)
    uint64_t *mb;       // sharded solves: the W grid sums also go to mb[q * mb_q + c] for every rank q < mb_P
    int64_t mb_q;       // (this rank's writer slot of one exchange in each reader's mailbox; nullptr: none)
    int32_t mb_P;
};

// the finished W sums into every rank's mailbox slot (system scope: pinned host memory other ranks poll)
template <int W>
__device__ __forceinline__ void gridsum_mail(const GridSum &gs, const double *r) {
    if (!gs.mb) return;
    for (int q = 0; q < gs.mb_P; ++q)
#pragma unroll
        for (int c = 0; c < W; ++c)
            __hip_atomic_store(gs.mb + q * gs.mb_q + c, (uint64_t)__double_as_longlong(r[c]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
}

// tiles of a full group ~ sqrt(nt) (both reductions stay short), and ngroups <= kGridSumMaxGroups
inline int32_t gridsum_grp_log2(int64_t nt) {
    if (nt <= kBlock) return -1;
    int32_t l = 0;
    while (((int64_t)1 << (2 * l)) < nt) ++l;
    auto ng = [&](int32_t g) { return ((nt + (kGridSumL << g) - 1) >> (kGridSumLLog + g)) * kGridSumL; };
    while (ng(l) > kGridSumMaxGroups) ++l;
    return l;
}
inline int64_t gridsum_ngroups(int64_t nt, int32_t gl) {
    if (gl < 0) return nt;
    const int64_t S = kGridSumL << gl, full = nt / S, tail = nt - full * S;
    return full * kGridSumL + (tail < kGridSumL ? tail : kGridSumL);
}

__device__ __forceinline__ int64_t gridsum_group_of(int64_t t, int32_t gl) {
    return ((t >> (kGridSumLLog + gl)) << kGridSumLLog) | (t & (kGridSumL - 1));
}
// member tiles of group g (base, base + 256, ...): count
__device__ __forceinline__ int64_t gridsum_members(const GridSum &gs, int64_t g, int64_t &base) {
    const int32_t gl = gs.grp_log2;
    const int64_t sb = g >> kGridSumLLog, l = g & (kGridSumL - 1), S = kGridSumL << gl;
    base = sb * S + l;
    const int64_t t = gs.nt - sb * S;
    return t >= S ? ((int64_t)1 << gl) : (t - l + kGridSumL - 1) >> kGridSumLLog;
}

__device__ __forceinline__ void gridsum_put(uint64_t *sl, double v) {
    __hip_atomic_store(sl, (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gridsum_draw(uint32_t *c) {
    return __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gridsum_reset(uint32_t *c) {
    __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t *gridsum_counter(const GridSum &gs, int64_t g) {
    return gs.cnt + g * kGridSumCntStride;
}
// a published value whose store has been issued (see above); poisoned and reported if it never lands
__device__ __forceinline__ uint64_t gridsum_wait(const uint64_t *sl, int32_t *err) {
    uint64_t bits = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (bits != kGridSumSentinel) return bits;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((bits = __hip_atomic_load(sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == kGridSumSentinel) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kGridSumWaitTicks) {
            atomicOr(err, 1);
            return 0x7FF8000000000000ull;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return bits;
}

// sum of src[(start + m)*W + c] over m in [0, cnt), lane-strided over NT lanes (lane t sums m = t,
// t + NT, ... in order), then the lanes' fixed-order total; every slot is re-armed. NT = kBlock:
// whole workgroup (block_sum); NT = 64: one wave (wave_total). A group's slots are contiguous
// (gridsum_slot), so is the group-sum array.
template <int W, int NT>
__device__ __forceinline__ void gridsum_take(uint64_t *src, int64_t start, int64_t cnt, int32_t *err, double *sh,
                                             double *res) {
    // B loads per lane in flight at once: the reductions of the launch's last tiles are its tail
    // (every group reducer and then the final one), one memory round trip per batch. 32-bit
    // offsets from one base (a group holds < 2^26 slots) keep the batch in few registers.
    constexpr int B = NT == 64 ? 8 : 4;
    const uint32_t lane = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
    const uint32_t n = (uint32_t)cnt;
    uint64_t *p = src + start * W;
#pragma unroll
    for (int c = 0; c < W; ++c) {
        // optimistic pass: a batch of independent loads, summed in member order; a sentinel seen
        // anywhere (rare: a store still in flight) redoes the lane's sum in the same order with waits
        double a = 0.0;
        bool ok = true;
        for (uint32_t m0 = lane; m0 < n; m0 += NT * B) {
            // unpredicated loads (index clamped with a min); members past the end then add -0.0,
            // which leaves every sum (+0.0 included) unchanged
            uint64_t v[B];
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const uint32_t m = __builtin_elementwise_min(m0 + (uint32_t)(i * NT), n - 1);
                v[i] = __hip_atomic_load(p + (m * W + c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int i = 0; i < B; ++i) {
                const uint64_t x = m0 + (uint32_t)(i * NT) < n ? v[i] : 0x8000000000000000ull;
                ok = ok && x != kGridSumSentinel;
                a += __longlong_as_double((long long)x);
            }
        }
        if (!ok) {
            a = 0.0;
            for (uint32_t m = lane; m < n; m += NT)
                a += __longlong_as_double((long long)gridsum_wait(p + (m * W + c), err));
        }
        for (uint32_t m = lane; m < n; m += NT)
            p[m * W + c] = kGridSumSentinel;   // re-arm; ordered before the next launch by the boundary
        res[c] = NT == 64 ? wave_total(a) : block_sum(a, sh);
    }
}

// slot of tile t in the two-level layout: group-major, so a group's slots (member tiles in order)
// are contiguous
__device__ __forceinline__ int64_t gridsum_slot(const GridSum &gs, int64_t t) {
    const int32_t gl = gs.grp_log2;
    const int64_t g = gridsum_group_of(t, gl), j = (t & ((kGridSumL << gl) - 1)) >> kGridSumLLog;
    return (g << gl) + j;
}

// ---- workgroup slots (every thread of every workgroup calls these; barriers inside) ---------
// The ticket (meaningful in thread 0 only; read at publish time). Call once the workgroup is known
// to publish (after any launch-uniform early exit), best after its first stream loads are issued.
// `tile`: the gridsum tile this workgroup publishes (default: its block index); a launch that maps
// blocks to tiles by any bijection (XCD bands) publishes by tile, so the sums do not depend on it.
__device__ __forceinline__ uint32_t gridsum_ticket(const GridSum &gs, int64_t tile) {
    uint32_t t = 0;
    if (threadIdx.x == 0 && gridDim.x != gs.nt) atomicOr(gs.err, 2);   // prepared for another grid
    if (gs.grp_log2 >= 0 && threadIdx.x == 0) t = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tile, gs.grp_log2)));
    return t;
}
__device__ __forceinline__ uint32_t gridsum_ticket(const GridSum &gs) { return gridsum_ticket(gs, blockIdx.x); }

// no-op finisher (below)
struct GridSumNoFin {
    __device__ void operator()(const double *) const {}
};

// final stage: after this workgroup's group sum (or one-level partial) was stored. `fin(r)` runs in
// thread 0 of the workgroup that computed the W grid sums, right after it stored them to out[]: a
// launch's own epilogue on the finished sums (e.g. the PCG init's normB / breakdown tests) without a
// second launch.
template <int W, class F = GridSumNoFin>
__device__ __forceinline__ void gridsum_final(const GridSum &gs, double *sh, const F &fin = F()) {
    __shared__ uint32_t tk;
    if (threadIdx.x == 0) tk = gridsum_draw(gridsum_counter(gs, kGridSumMaxGroups));
    __syncthreads();
    const bool last = tk == (uint32_t)(gs.ngroups - 1);
    __syncthreads();
    if (!last) return;
    double r[W];
    gridsum_take<W, kBlock>(gs.gslots, 0, gs.ngroups, gs.err, sh, r);
    if (threadIdx.x == 0) {
        gridsum_reset(gridsum_counter(gs, kGridSumMaxGroups));
#pragma unroll
        for (int c = 0; c < W; ++c) gs.out[c] = r[c];
        gridsum_mail<W>(gs, r);
        fin(r);
    }
}

// Called with the workgroup's W sums (identical in all threads, e.g. from block_sum) and the raw
// ticket from gridsum_ticket. Kernel-uniform control flow. fin: see gridsum_final.
template <int W, class F = GridSumNoFin>
__device__ __forceinline__ void gridsum_publish_tile(const GridSum &gs, const double *v, double *sh, uint32_t ticket,
                                                     int64_t b, const F &fin = F()) {
    if (gs.grp_log2 < 0) {
        if (threadIdx.x == 0)
#pragma unroll
            for (int c = 0; c < W; ++c) gridsum_put(gs.gslots + b * W + c, v[c]);
        gridsum_final<W>(gs, sh, fin);
        return;
    }
    __shared__ uint32_t tk;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int c = 0; c < W; ++c) gridsum_put(gs.slots + gridsum_slot(gs, b) * W + c, v[c]);
        tk = ticket;
    }
    __syncthreads();
    const int64_t g = gridsum_group_of(b, gs.grp_log2);
    int64_t base;
    const int64_t cnt = gridsum_members(gs, g, base);
    const bool last = tk == (uint32_t)(cnt - 1);
    __syncthreads();
    if (!last) return;
    double r[W];
    gridsum_take<W, kBlock>(gs.slots, g << gs.grp_log2, cnt, gs.err, sh, r);
    if (threadIdx.x == 0) {
        gridsum_reset(gridsum_counter(gs, g));
#pragma unroll
        for (int c = 0; c < W; ++c) gridsum_put(gs.gslots + g * W + c, r[c]);
    }
    gridsum_final<W>(gs, sh, fin);
}
template <int W, class F = GridSumNoFin>
__device__ __forceinline__ void gridsum_publish(const GridSum &gs, const double *v, double *sh, uint32_t ticket,
                                                const F &fin = F()) {
    gridsum_publish_tile<W>(gs, v, sh, ticket, blockIdx.x, fin);
}

// ---- per-wave partials combined in LDS (the SpMV's dot epilogue) ------------------------------
// Each wave of a tile writes its wave total (DPP, no shuffle traffic) to LDS and counts itself in
// with an LDS atomic; the wave that counts last adds the kWaves totals in wave order and publishes
// the tile's ONE slot, then plays the tile's part in the ticket protocol: one write-through store
// per tile instead of one per wave (~2 us less at N = 10M; what the remaining ~6 us of the dot
// epilogue is — it is not per store — is recorded in profiles/r3_gridsum_lab.txt and, for the pair-row kernel,
// profiles/r6_diagp_epilogue_ab.txt (round-3/6 probe builds, removed from the product since)). No workgroup barrier at the end; the one barrier (arming the
// LDS counter) sits where every wave waits for its stream loads anyway.
template <int W>
struct GridSumTile {
    uint32_t cnt;
    uint32_t ticket;
    double part[kWaves * W];
};
// every thread, once the tile's stream loads are issued and it is known to publish (after any
// launch-uniform early exit); returns the raw ticket (thread 0), read at publish time
template <int W>
__device__ __forceinline__ uint32_t gridsum_tile_begin(const GridSum &gs, GridSumTile<W> &L, int64_t tile) {
    if (threadIdx.x == 0) {
        L.cnt = 0;
        if (gridDim.x != gs.nt) atomicOr(gs.err, 2);   // prepared for another grid
    }
    __syncthreads();
    uint32_t t = 0;
    if (gs.grp_log2 >= 0 && threadIdx.x == 0) t = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tile, gs.grp_log2)));
    return t;
}

// fin: see gridsum_final (run by lane 0 of the wave that finished the W sums)
template <int W, class F = GridSumNoFin>
__device__ __forceinline__ void gridsum_final_wave(const GridSum &gs, const F &fin = F()) {
    const bool lane0 = (threadIdx.x & 63) == 0;
    uint32_t f = 0;
    if (lane0) f = gridsum_draw(gridsum_counter(gs, kGridSumMaxGroups));
    f = __builtin_amdgcn_readfirstlane(f);
    if (f != (uint32_t)(gs.ngroups - 1)) return;
    double r[W];
    gridsum_take<W, 64>(gs.gslots, 0, gs.ngroups, gs.err, nullptr, r);
    if (lane0) {
        gridsum_reset(gridsum_counter(gs, kGridSumMaxGroups));
#pragma unroll
        for (int c = 0; c < W; ++c) gs.out[c] = r[c];
        gridsum_mail<W>(gs, r);
        fin(r);
    }
}

// every lane of every wave, with the wave's W totals (uniform) and the raw ticket; no barrier
template <int W>
__device__ __forceinline__ void gridsum_tile_publish(const GridSum &gs, GridSumTile<W> &L, const double *v,
                                                     uint32_t ticket, int64_t tile) {
    const bool lane0 = (threadIdx.x & 63) == 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t old = 0;
    if (lane0) {
#pragma unroll
        for (int c = 0; c < W; ++c) L.part[wave * W + c] = v[c];
        if (threadIdx.x == 0) L.ticket = ticket;
        // this wave's LDS writes land before its count (release, LDS only)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        old = atomicAdd(&L.cnt, 1u);
    }
    if (__builtin_amdgcn_readfirstlane(old) != kWaves - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    double s[W];
#pragma unroll
    for (int c = 0; c < W; ++c) {
        s[c] = L.part[c];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) s[c] += L.part[w * W + c];   // wave order
    }
    const uint32_t tk = L.ticket;
    if (gs.grp_log2 < 0) {
        if (lane0)
#pragma unroll
            for (int c = 0; c < W; ++c) gridsum_put(gs.gslots + tile * W + c, s[c]);
        gridsum_final_wave<W>(gs);
        return;
    }
    if (lane0)
#pragma unroll
        for (int c = 0; c < W; ++c) gridsum_put(gs.slots + gridsum_slot(gs, tile) * W + c, s[c]);
    const int64_t g = gridsum_group_of(tile, gs.grp_log2);
    int64_t base;
    const int64_t cnt = gridsum_members(gs, g, base);
    if (tk != (uint32_t)(cnt - 1)) return;
    double r[W];
    gridsum_take<W, 64>(gs.slots, g << gs.grp_log2, cnt, gs.err, nullptr, r);
    if (lane0) {
        gridsum_reset(gridsum_counter(gs, g));
#pragma unroll
        for (int c = 0; c < W; ++c) gridsum_put(gs.gslots + g * W + c, r[c]);
    }
    gridsum_final_wave<W>(gs);
}

// The tile epilogue of a workgroup holding TPW gridsum tiles with W sums each (the W = 1 form is the SpMV's
// spmv_publish_multi): each wave's totals (DPP) combined in LDS in wave order per tile, every tile's slot
// stored first, then a wave holding a group's last ticket reduces that group; fin: see gridsum_final.
// Every thread, after the tiles' LDS counters were zeroed behind a barrier; tv[q] uniform.
template <int TPW, int W, class F = GridSumNoFin>
__device__ __forceinline__ void gridsum_tiles_publish(const GridSum &gs, GridSumTile<W> *L, const double (*acc)[W],
                                                      const uint32_t *ticket, const int64_t *tl, const bool *tv,
                                                      const F &fin = F()) {
    const bool lane0 = (threadIdx.x & 63) == 0;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    bool mine[TPW];
    uint32_t tk[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        mine[q] = false;
        tk[q] = 0;
        if (!tv[q]) continue;
        double ws[W];
#pragma unroll
        for (int c = 0; c < W; ++c) ws[c] = wave_total(acc[q][c]);
        uint32_t old = 0;
        if (lane0) {
#pragma unroll
            for (int c = 0; c < W; ++c) L[q].part[wave * W + c] = ws[c];
            if (threadIdx.x == 0) L[q].ticket = ticket[q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            old = atomicAdd(&L[q].cnt, 1u);
        }
        if (__builtin_amdgcn_readfirstlane(old) != kWaves - 1) continue;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        double sum[W];
#pragma unroll
        for (int c = 0; c < W; ++c) {
            sum[c] = L[q].part[c];
#pragma unroll
            for (int w = 1; w < kWaves; ++w) sum[c] += L[q].part[w * W + c];   // wave order
        }
        tk[q] = L[q].ticket;
        if (lane0)
#pragma unroll
            for (int c = 0; c < W; ++c)
                gridsum_put(gs.grp_log2 < 0 ? gs.gslots + tl[q] * W + c : gs.slots + gridsum_slot(gs, tl[q]) * W + c, sum[c]);
        mine[q] = true;
    }
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        if (!mine[q]) continue;
        if (gs.grp_log2 < 0) {
            gridsum_final_wave<W>(gs, fin);
            continue;
        }
        const int64_t g = gridsum_group_of(tl[q], gs.grp_log2);
        int64_t base;
        const int64_t cnt = gridsum_members(gs, g, base);
        if (tk[q] != (uint32_t)(cnt - 1)) continue;
        double r[W];
        gridsum_take<W, 64>(gs.slots, g << gs.grp_log2, cnt, gs.err, nullptr, r);
        if (lane0) {
            gridsum_reset(gridsum_counter(gs, g));
#pragma unroll
            for (int c = 0; c < W; ++c) gridsum_put(gs.gslots + g * W + c, r[c]);
        }
        gridsum_final_wave<W>(gs, fin);
    }
}

// host: a GridSum for a one-shot launch of nt tiles (workgroups) with W (<= kGridSumMaxW) sums
// written to out[0..W)
int gridsum_prepare(Context *c, int64_t nt, int W, double *out, GridSum *gs);
// reports (and clears) an expired gridsum wait, a launch whose grid was not the prepared one and a
// ticket counter left non-zero; syncs the stream
int gridsum_check(Context *c);
// the same split in two, so a solve folds it into its final synchronisation: enqueue the counter
// scan and the copy of the error word into *host_word (pinned), then, after the stream sync, decode
int gridsum_check_enqueue(Context *c, int32_t *host_word);
int gridsum_check_result(Context *c, int32_t host_word);

// ---------------------------------------------------------------------------------------------
// XCD-banded tile order (speed only, never correctness): workgroups are dealt round-robin over the
// 8 XCDs (observed; MI355X_MICROARCH.md), so blocks b and b + 8 share an XCD and its L2. Tile
// (slice) t = s_k + b/8 for block b, k = b mod 8, hands XCD k the CONTIGUOUS tiles [s_k, s_k + c_k):
// a stencil row's x neighbours one grid line away (m rows = m/256 tiles: 12.4 at N = 10M, where
// round-robin puts them on other XCDs and x is fetched ~3 times) are then read through the same L2.
// TileMap{0, 0} is the identity. Bijective for any tile count.
struct TileMap {
    int64_t a;     // tiles / 8 (0 = identity)
    int32_t r;     // tiles mod 8: classes k < r hold one more tile
    int32_t rev;   // 1: each XCD walks its band from the end (the lines its predecessor wrote last first)
    int64_t c;     // > 0 (with a == 0): CHUNKED — XCD k takes chunks k, k + 8, ... of c consecutive tiles (round 6,
                   // the CSR tile kernel); the tiles past the last whole 8c in block order
};
inline TileMap tile_map_for(int64_t ntiles, bool banded, bool rev = false) {
    return banded && ntiles >= 64 ? TileMap{ntiles >> 3, (int32_t)(ntiles & 7), rev ? 1 : 0, 0} : TileMap{0, 0, 0, 0};
}
inline TileMap tile_map_chunked(int64_t ntiles, int64_t c) {
    return c > 0 && ntiles >= 8 * c ? TileMap{0, 0, 0, c} : TileMap{0, 0, 0, 0};
}
__device__ __forceinline__ int64_t tile_of_block(TileMap tm) {
    const int64_t b = blockIdx.x;
    if (tm.c > 0) {   // b = 8 j + k on XCD k (round-robin dealing): its j-th tile is in chunk (j / c) * 8 + k
        const int64_t k = b & 7, j = b >> 3;
        const int64_t t = ((j / tm.c) * 8 + k) * tm.c + j % tm.c;
        const int64_t full = (int64_t)(gridDim.x / (8 * tm.c)) * 8 * tm.c;
        return b < full ? t : b;
    }
    if (tm.a == 0) return b;
    const int64_t k = b & 7, j = b >> 3;
    const int64_t start = k * tm.a + (k < tm.r ? k : tm.r);
    return tm.rev ? start + (tm.a + (k < tm.r ? 1 : 0)) - 1 - j : start + j;
}

// 16-byte vector accesses; *_nt = non-temporal (streamed data that is not re-read soon)
typedef double dv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dv2 ld2(const double *p) { return *reinterpret_cast<const dv2 *>(p); }
__device__ __forceinline__ dv2 ld2nt(const double *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const dv2 *>(p));
}
__device__ __forceinline__ void st2(double *p, dv2 v) { *reinterpret_cast<dv2 *>(p) = v; }
__device__ __forceinline__ void st2nt(double *p, dv2 v) { __builtin_nontemporal_store(v, reinterpret_cast<dv2 *>(p)); }

// contiguous share [b0,b1) of `ntiles` tiles for workgroup `b` of `g`
__device__ __forceinline__ void block_range(int64_t ntiles, int64_t &t0, int64_t &t1) {
    const int64_t g = gridDim.x, b = blockIdx.x;
    t0 = ntiles * b / g;
    t1 = ntiles * (b + 1) / g;
}

inline int grid_for_rows(const Context *c, int64_t rows, int per_tile) {
    int64_t tiles = (rows + per_tile - 1) / per_tile;
    if (tiles < 1) tiles = 1;
    return (int)(tiles < c->grid_cap ? tiles : c->grid_cap);
}

// ---------------------------------------------------------------------------------------------
// host helpers shared by the solver TUs
int to_device_vec(const double *src, int32_t loc, int64_t n, double *dst, hipStream_t s);
int from_device_vec(const double *src, int32_t loc, int64_t n, double *dst, hipStream_t s);
int halo_exchange(psk_csr *A, double *x_local, hipStream_t s);
// the exchange on stream cs after the work enqueued on s (ev_a), completion recorded in ev_b
int halo_exchange_async(psk_csr *A, double *x, hipStream_t s, hipStream_t cs, hipEvent_t ev_a, hipEvent_t ev_b,
                        hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// rows sent to peers confined to the first lo / the tiles from hi on (of nv tiles of `tile` rows)
bool halo_split(const psk_csr *A, int64_t tile, int64_t nv, int64_t &lo, int64_t &hi);
// recv[q*count + i] = rank q's send[i]: no arithmetic, so every rank holds the same bits and
// reduces them in rank order itself (RCCL's reduction order is algorithm- and rank-dependent)
int allgather(psk_csr *A, const double *send, double *recv, int64_t count, hipStream_t s);
// mailbox exchanges (psk_comm::mb): the next exchange's writer slots into gs (producer launch), and the
// gather of that exchange into recv[q*W + c] on s (skipped on the device when *done is set: the producer
// did not run either); returns the exchange number
uint64_t mbox_next(psk_comm *c, GridSum *gs);
int mbox_gather(psk_comm *c, uint64_t seq, int W, double *recv, const int32_t *done, hipStream_t s,
                hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

// SpMV launch (defined in spmv.hip); modes below
enum SpmvMode : int {
    kSpmvPlain = 0,     // y = A x
    kSpmvDot = 1,       // y = A x, partial[b] = sum_i x_i y_i        (PCG: p.Ap)
    kSpmvJacobiDot = 2, // y = A (d .* x), partial[b] = sum_i q_i y_i (GMRES: A M^-1 q_k, q_0.u)
    kSpmvPlainDot = 3,  // y = A x, partial[b] = sum_i q_i y_i        (GMRES identity)
    kSpmvResid = 4,     // y = b - A x, partial[b] = sum_i y_i^2      (true residual; partial nullable)
    kSpmvAdd = 5,       // y = q + A x                                (AMG prolongation x + P x2)
};
int fd2d_fill(psk_csr *A, int64_t m, double a, double b, int64_t row_begin, int64_t row_end,
              int64_t halo_lo_start, hipStream_t s);
// generic preconditioner apply (device pointers, out must not alias v): identity copy, Jacobi, ILU
int prec_apply_dev(const psk_prec *M, int64_t n, const double *v, double *out, hipStream_t s);
int ilu_apply(const psk_prec *M, const double *v, double *out, hipStream_t s);
int ilu_apply_add(const psk_prec *M, const double *v, double *x, hipStream_t s);
// AMG paired Gauss-Seidel sweeps (amg.hip; the lab library's switch): set -1 / 0 / 1, counts out
int amg_gs_pair(psk_prec *M, int set, int *on, int *eligible);   // x += M^-1 v
int ilu_check_error(const psk_prec *M, hipStream_t s);
int amg_apply(const psk_prec *M, const double *v, double *out, hipStream_t s);
void amg_free(AmgHierarchy *h);
int dense_apply(const psk_prec *M, const double *v, double *out, hipStream_t s);
int dense_check_error(const psk_prec *M, hipStream_t s);
void dense_free(DenseInverse *d);
// preconditioners whose apply is not a single elementwise op (triangular solves, AMG): the
// Krylov drivers take their general path for these
inline bool prec_is_general(const psk_prec *M) {
    return M && (M->kind == PSK_PREC_ILU || M->kind == PSK_PREC_AMG || M->kind == PSK_PREC_DENSE);
}
// reports a bounded-spin timeout of any triangular solve inside M (syncs the stream)
int prec_check_error(const psk_prec *M, hipStream_t s);
int tile_rows_for(int64_t n, int64_t nnz);
// SpMV layout of a freshly created matrix: the sliced copy when it streams no more bytes than the
// CSR arrays (PSK_SPMV_LAYOUT=csr|sliced overrides); called at the end of every creation path
int csr_choose_layout(psk_csr *A, hipStream_t s);
void sliced_free(psk_csr *A);
// one-shot SpMV (grid = tiles of A->tile_rows rows); dot modes write their grid sum to partial[0].
// ev0/ev1 (optional): HIP events the dispatch itself records at the kernel's start and end
// (hipExtLaunchKernel), so their interval is the kernel alone, without the launch gaps around it
// mail: the dot sum also goes to the communicator's next mailbox exchange (*mail_seq = its number)
int launch_spmv(const psk_csr *A, int mode, const double *x, double *y, const double *aux_d,
                const double *aux_q, double *partial, const int32_t *done_flag, hipStream_t s,
                hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int rev = 0, uint64_t *mail_seq = nullptr);

}  // namespace psk
