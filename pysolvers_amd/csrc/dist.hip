// dist.hip — row-block sharding across the GPUs of one node (one process per GPU, RCCL over xGMI).
//
// No reference counterpart: PySolvers is single-process. The sharded PCG is the same loop as
// pcg.hip; per iteration it adds (1) a halo exchange of the search direction p with the two
// neighbouring ranks (grouped ncclSend/ncclRecv of one grid line each way for the 5-point FD
// matrix: m doubles per side), and (2) two ncclAllGather of the ranks' dot products (p.Ap; then
// r.r and u.r fused). Every rank then sums the gathered values in rank order itself, so all ranks
// hold bit-identical scalars and stop on the same iteration without further communication (an
// all-reduce would leave the order of the rank sum to RCCL's algorithm choice).
#include "psk_internal.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>

namespace psk {

// sendbuf[k] = x[idx[k]]: the owned entries the peers need, packed peer by peer
__global__ void halo_pack_kernel(int64_t count, const int32_t *__restrict__ idx, const double *__restrict__ x,
                                 double *__restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < count) out[k] = x[idx[k]];
}

int halo_exchange(psk_csr *A, double *x, hipStream_t s) {
    if (!A->comm || A->peers.empty()) return PSK_OK;
    if (A->comm->dry) return PSK_OK;   // the caller supplied the halo entries
    ncclComm_t nc = A->comm->nccl;
    double *sb = A->sendbuf.as<double>();
    if (A->pack_count > 0) {
        hipLaunchKernelGGL(halo_pack_kernel, dim3((unsigned)((A->pack_count + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           s, A->pack_count, A->pack_idx, x, sb);
        PSK_HIP(hipGetLastError());
    }
    if (A->comm->shm) {
        std::vector<int> pr;
        std::vector<const double *> sd;
        std::vector<double *> rv;
        std::vector<int64_t> sc, rc;
        for (const HaloPeer &p : A->peers) {
            pr.push_back(p.rank);
            sd.push_back(p.send_idx ? sb + p.pack_off : x + p.send_begin);
            sc.push_back(p.send_count);
            rv.push_back(x + A->n + p.recv_offset);
            rc.push_back(p.recv_count);
        }
        return shm_exchange(A->comm, (int)pr.size(), pr.data(), sd.data(), sc.data(), rv.data(), rc.data(), s);
    }
    PSK_RCCL(ncclGroupStart());
    for (const HaloPeer &p : A->peers) {
        if (p.send_count > 0) {
            const double *src = p.send_idx ? sb + p.pack_off : x + p.send_begin;
            PSK_RCCL(ncclSend(src, (size_t)p.send_count, ncclDouble, p.rank, nc, s));
        }
        if (p.recv_count > 0)
            PSK_RCCL(ncclRecv(x + A->n + p.recv_offset, (size_t)p.recv_count, ncclDouble, p.rank, nc, s));
    }
    PSK_RCCL(ncclGroupEnd());
    return PSK_OK;
}

// The halo exchange on the second stream `cs`, after the work already enqueued on `s` (event ev_a);
// ev_b marks its completion for the consumer (the next SpMV waits on it).
// t0 / t1 (optional, timing): recorded on `cs` around the exchange itself
int halo_exchange_async(psk_csr *A, double *x, hipStream_t s, hipStream_t cs, hipEvent_t ev_a, hipEvent_t ev_b,
                        hipEvent_t t0, hipEvent_t t1) {
    PSK_HIP(hipEventRecord(ev_a, s));
    PSK_HIP(hipStreamWaitEvent(cs, ev_a, 0));
    if (t0) PSK_HIP(hipEventRecord(t0, cs));
    PSK_TRY(halo_exchange(A, x, cs));
    if (t1) PSK_HIP(hipEventRecord(t1, cs));
    PSK_HIP(hipEventRecord(ev_b, cs));
    return PSK_OK;
}

// Overlap plan: true when every row sent to a peer lies in a prefix [0, lo*tile) or a suffix
// [hi*tile, n) of the owned rows (contiguous sends: row blocks of banded matrices) and the middle
// [lo, hi) is at least a quarter of the `nv` tiles, so that K3 can run the send tiles first.
bool halo_split(const psk_csr *A, int64_t tile, int64_t nv, int64_t &lo, int64_t &hi) {
    if (!A->comm || A->peers.empty() || A->comm->dry) return false;
    int64_t pre = 0, suf = A->n;
    for (const HaloPeer &p : A->peers) {
        if (p.send_count == 0) continue;
        if (p.send_idx) return false;
        const int64_t b = p.send_begin, e = p.send_begin + p.send_count;
        if (b == 0) pre = std::max(pre, e);
        else if (e == A->n) suf = std::min(suf, b);
        else return false;
    }
    lo = (pre + tile - 1) / tile;
    hi = suf / tile;
    return hi > lo && (hi - lo) * 4 >= nv;
}

int allgather(psk_csr *A, const double *send, double *recv, int64_t count, hipStream_t s) {
    if (!A->comm) return fail(PSK_ERR_ARG, "allgather on an unsharded matrix");
    if (A->comm->dry) return fail(PSK_ERR_UNSUPPORTED, "collective on a dry (RCCL-less) communicator");
    if (A->comm->shm) return shm_allgather(A->comm, send, recv, count, s);
    PSK_RCCL(ncclAllGather(send, recv, (size_t)count, ncclDouble, A->comm->nccl, s));
    return PSK_OK;
}

// ---- device-side scalar exchange through a host-shared mailbox (round 5; psk_internal.hpp Mailbox) ----
// An RCCL all-gather of a few bytes costs a collective kernel launch and its protocol on the solver's
// stream (tens of us at P = 8 by DESIGN.md's budget), twice per PCG iteration, on the critical path. Here
// the kernel that finishes a rank's grid sums (gridsum_mail) stores them directly into every rank's slot,
// and each rank's one-wave gather kernel polls its own slot: one posted system-scope store per value and
// one host-memory round trip per poll. Value-is-flag: a slot holds a signalling-NaN sentinel until its
// value lands; the reader re-arms it after copying. Ring of kMbRing exchanges: exchange e + kMbRing is
// written by a rank only after it consumed exchange e + kMbRing - 1 from every rank, and every rank
// consumed e before producing e + 1 (each exchange's values come from a kernel that follows the gather
// of the previous one), so a slot is never overwritten before its reader re-armed it.
constexpr size_t kMbHeader = 4096;
constexpr uint64_t kMbSentinel = 0x7FF0DEAD5EED0001ull;   // sNaN payload: never an arithmetic result
constexpr uint64_t kMbWaitTicks = (uint64_t)2 << 27;       // s_memrealtime (100 MHz): ~2.7 s

static inline size_t mb_index(const Mailbox &m, int q, int64_t slot, int r, int c) {
    return (((size_t)q * kMbRing + (size_t)slot) * (size_t)m.P + (size_t)r) * kMbW + (size_t)c;
}

uint64_t mbox_next(psk_comm *c, GridSum *gs) {
    Mailbox &m = *c->mb;
    const uint64_t e = m.seq++;
    gs->mb = m.dev + mb_index(m, 0, (int64_t)(e % kMbRing), m.rank, 0);
    gs->mb_q = (int64_t)kMbRing * m.P * kMbW;
    gs->mb_P = m.P;
    return e;
}

// lane q < P: writer q's W values of this rank's slot -> recv[q*W + c], then re-armed
__global__ void mbox_gather_kernel(uint64_t *mine, int P, int W, double *__restrict__ recv, const int32_t *done,
                                   int32_t *err) {
    if (done && __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;   // uniform
    const int q = threadIdx.x;
    if (q >= P) return;
    for (int c = 0; c < W; ++c) {
        uint64_t *p = mine + (size_t)q * kMbW + c;
        uint64_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == kMbSentinel) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while ((v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) == kMbSentinel) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > kMbWaitTicks) {
                    atomicOr(err, 8);
                    v = 0x7FF8000000000000ull;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        recv[q * W + c] = __longlong_as_double((long long)v);
        __hip_atomic_store(p, kMbSentinel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // the re-arms are visible system-wide before this rank's next mailbox stores (a later kernel's), whatever the
    // other ranks' progress: exchange e + 4 reuses this slot
    __threadfence_system();
}

int mbox_gather(psk_comm *c, uint64_t seq, int W, double *recv, const int32_t *done, hipStream_t s, hipEvent_t ev0,
                hipEvent_t ev1) {
    Context *cx;
    PSK_TRY(ctx(&cx));
    if (!cx->gs_err) {   // the error word gridsum_check reports (allocated with the first grid sum)
        GridSum tmp;
        PSK_TRY(gridsum_prepare(cx, 1, 1, recv, &tmp));
    }
    Mailbox &m = *c->mb;
    if (W < 1 || W > kMbW) return fail(PSK_ERR_ARG, "mbox_gather: bad width");
    // ev0 / ev1 (optional, timing): recorded by the dispatch itself around the kernel (its wait for the ranks)
    hipExtLaunchKernelGGL(mbox_gather_kernel, dim3(1), dim3(64), 0, s, ev0, ev1, 0,
                          m.dev + mb_index(m, m.rank, (int64_t)(seq % kMbRing), 0, 0), m.P, W, recv, done, cx->gs_err);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

static void mbox_close(psk_comm *c) {
    Mailbox *m = c->mb;
    if (!m) return;
    if (m->host) {
        (void)hipHostUnregister(m->host);
        munmap(m->host, m->bytes);
    }
    if (m->rank == 0) shm_unlink(m->name.c_str());
    delete m;
    c->mb = nullptr;
}

// Row-block plan of the m x m 5-point matrix over P ranks: whole grid lines per rank; local column
// layout [owned | halo_lo (previous rank's last line) | halo_hi (next rank's first line)].
struct FdPlan {
    int64_t rb, re, nloc, ncols, halo_lo, halo_hi;
};

static int fd2d_plan(int64_t m, int P, int r, FdPlan &p) {
    if (m < 1 || P < 1 || r < 0 || r >= P) return fail(PSK_ERR_ARG, "fd2d plan: bad arguments");
    if (P > m) return fail(PSK_ERR_ARG, "fd2d_dist: more ranks than grid lines");
    const int64_t l0 = m * r / P, l1 = m * (r + 1) / P;
    p.rb = l0 * m;
    p.re = l1 * m;
    p.nloc = p.re - p.rb;
    p.halo_lo = l0 > 0 ? m : 0;
    p.halo_hi = l1 < m ? m : 0;
    p.ncols = p.nloc + p.halo_lo + p.halo_hi;
    return PSK_OK;
}


// ---- general row-block sharding (psk_csr_create_dist) --------------------------------------
// Host plan of rank r's block, rows [rs[r], rs[r+1]) of a global CSR:
//  * local columns: owned c -> c - rb; every other referenced column -> nloc + its position in the
//    ascending list of distinct off-block columns (the halo), which is therefore grouped by owner
//    rank in rank order: the segment received from rank q is contiguous;
//  * send to q: the owned rows that have an entry in q's block, ascending. For a structurally
//    symmetric pattern that is exactly the list q receives from us (A[j][c] != 0 <=> A[c][j] != 0),
//    so it is built without communication; under RCCL the lists are exchanged once at creation and
//    compared (dist_verify), and every rank refuses a pattern that is not symmetric across ranks.
struct DistPlan {
    int64_t rb = 0, re = 0, nloc = 0;
    std::vector<int32_t> lcol;                    // local column of every local entry
    std::vector<int64_t> halo;                    // global ids of the halo columns (ascending)
    std::vector<int64_t> recv_off, recv_cnt;      // per rank: halo segment it owns
    std::vector<std::vector<int32_t>> send_rows;  // per rank: owned local rows it needs
};

static int owner_of(const int64_t *rs, int P, int64_t c) {
    return (int)(std::upper_bound(rs, rs + P + 1, c) - rs) - 1;   // largest q with rs[q] <= c
}

static int dist_plan(int64_t n_global, const int64_t *rs, int P, int r, const int64_t *rowptr, const int32_t *colidx,
                     DistPlan &pl) {
    pl.rb = rs[r];
    pl.re = rs[r + 1];
    pl.nloc = pl.re - pl.rb;
    const int64_t e0 = rowptr[0], nnz = rowptr[pl.nloc] - e0;
    std::vector<int64_t> off;
    for (int64_t j = 0; j < nnz; ++j) {
        const int64_t c = colidx[j];
        if (c < 0 || c >= n_global) return fail(PSK_ERR_ARG, "psk_csr_create_dist: column index out of range");
        if (c < pl.rb || c >= pl.re) off.push_back(c);
    }
    std::sort(off.begin(), off.end());
    off.erase(std::unique(off.begin(), off.end()), off.end());
    pl.halo.swap(off);
    if (pl.nloc + (int64_t)pl.halo.size() >= INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "local columns exceed int32");
    pl.lcol.resize((size_t)nnz);
    pl.recv_off.assign((size_t)P, 0);
    pl.recv_cnt.assign((size_t)P, 0);
    pl.send_rows.assign((size_t)P, {});
    for (size_t k = 0; k < pl.halo.size(); ++k) {
        const int q = owner_of(rs, P, pl.halo[k]);
        if (pl.recv_cnt[(size_t)q] == 0) pl.recv_off[(size_t)q] = (int64_t)k;
        ++pl.recv_cnt[(size_t)q];
    }
    for (int64_t i = 0; i < pl.nloc; ++i)
        for (int64_t j = rowptr[i] - e0; j < rowptr[i + 1] - e0; ++j) {
            const int64_t c = colidx[j];
            if (c >= pl.rb && c < pl.re) {
                pl.lcol[(size_t)j] = (int32_t)(c - pl.rb);
                continue;
            }
            const int64_t k = std::lower_bound(pl.halo.begin(), pl.halo.end(), c) - pl.halo.begin();
            pl.lcol[(size_t)j] = (int32_t)(pl.nloc + k);
            std::vector<int32_t> &sr = pl.send_rows[(size_t)owner_of(rs, P, c)];
            if (sr.empty() || sr.back() != (int32_t)i) sr.push_back((int32_t)i);
        }
    return PSK_OK;
}

// Synchronous host-buffer collectives for creation-time checks, over the communicator's transport
// (RCCL: staged through device memory on libpsk's stream; shared memory: shmcomm.hip).
static int host_allgather(psk_comm *cm, const void *mine, void *all, size_t bytes) {
    if (cm->shm) return shm_allgather_host(cm, mine, all, bytes);
    Context *c;
    PSK_TRY(ctx(&c));
    hipStream_t s = c->stream;
    DevBuf d;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{d};
    PSK_TRY(d.ensure(bytes * (size_t)(cm->nranks + 1) + 64));
    char *dm = d.as<char>(), *da = dm + bytes;
    PSK_HIP(hipMemcpy(dm, mine, bytes, hipMemcpyHostToDevice));
    PSK_RCCL(ncclAllGather(dm, da, bytes, ncclUint8, cm->nccl, s));
    PSK_HIP(hipMemcpyAsync(all, da, bytes * (size_t)cm->nranks, hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    return PSK_OK;
}

static int host_exchange(psk_comm *cm, const std::vector<int> &peers, const std::vector<const void *> &sends,
                         const std::vector<size_t> &sb, const std::vector<void *> &recvs, const std::vector<size_t> &rb) {
    const int np = (int)peers.size();
    if (cm->shm) return shm_exchange_host(cm, np, peers.data(), sends.data(), sb.data(), recvs.data(), rb.data());
    Context *c;
    PSK_TRY(ctx(&c));
    hipStream_t s = c->stream;
    size_t tot = 0;
    for (int k = 0; k < np; ++k) tot += sb[(size_t)k] + rb[(size_t)k];
    DevBuf d;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{d};
    PSK_TRY(d.ensure(tot + 64));
    char *p = d.as<char>();
    std::vector<char *> dr((size_t)np);
    PSK_RCCL(ncclGroupStart());
    for (int k = 0; k < np; ++k) {
        if (sb[(size_t)k]) {
            PSK_HIP(hipMemcpy(p, sends[(size_t)k], sb[(size_t)k], hipMemcpyHostToDevice));
            PSK_RCCL(ncclSend(p, sb[(size_t)k], ncclUint8, peers[(size_t)k], cm->nccl, s));
            p += sb[(size_t)k];
        }
        dr[(size_t)k] = p;
        if (rb[(size_t)k]) {
            PSK_RCCL(ncclRecv(p, rb[(size_t)k], ncclUint8, peers[(size_t)k], cm->nccl, s));
            p += rb[(size_t)k];
        }
    }
    PSK_RCCL(ncclGroupEnd());
    for (int k = 0; k < np; ++k)
        if (rb[(size_t)k]) PSK_HIP(hipMemcpyAsync(recvs[(size_t)k], dr[(size_t)k], rb[(size_t)k], hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    return PSK_OK;
}

// Creation-time check (collective over all ranks, same verdict everywhere): the send and receive
// counts agree pairwise, then each rank's send list equals what its peer expects to receive.
static int dist_verify(psk_comm *cm, const DistPlan &pl) {
    const int P = cm->nranks;
    std::vector<int64_t> mine((size_t)2 * P), all((size_t)2 * P * P);
    for (int q = 0; q < P; ++q) {
        mine[(size_t)q] = (int64_t)pl.send_rows[(size_t)q].size();
        mine[(size_t)(P + q)] = pl.recv_cnt[(size_t)q];
    }
    PSK_TRY(host_allgather(cm, mine.data(), all.data(), mine.size() * 8));
    for (int a = 0; a < P; ++a)
        for (int b = 0; b < P; ++b)
            if (a != b && all[(size_t)(2 * P * a + b)] != all[(size_t)(2 * P * b + P + a)])
                return fail(PSK_ERR_ARG, "psk_csr_create_dist: halo counts disagree across ranks (pattern not "
                                         "structurally symmetric)");
    // send each owner the global ids we receive from it; receive the ids each peer receives from us
    std::vector<int> peers;
    std::vector<const void *> sends;
    std::vector<void *> recvs;
    std::vector<size_t> sb, rb;
    std::vector<std::vector<int64_t>> got((size_t)P);
    for (int q = 0; q < P; ++q) {
        const size_t ns = pl.send_rows[(size_t)q].size(), nr = (size_t)pl.recv_cnt[(size_t)q];
        if (ns == 0 && nr == 0) continue;
        got[(size_t)q].resize(ns);
        peers.push_back(q);
        sends.push_back(pl.halo.data() + (nr ? pl.recv_off[(size_t)q] : 0));
        sb.push_back(nr * 8);
        recvs.push_back(got[(size_t)q].data());
        rb.push_back(ns * 8);
    }
    PSK_TRY(host_exchange(cm, peers, sends, sb, recvs, rb));
    int32_t ok = 1;
    for (int q = 0; q < P && ok; ++q)
        for (size_t k = 0; k < pl.send_rows[(size_t)q].size(); ++k)
            if (got[(size_t)q][k] != pl.rb + pl.send_rows[(size_t)q][k]) {
                ok = 0;
                break;
            }
    std::vector<int32_t> oks((size_t)P);
    PSK_TRY(host_allgather(cm, &ok, oks.data(), 4));
    for (int q = 0; q < P; ++q)
        if (!oks[(size_t)q])
            return fail(PSK_ERR_ARG, "psk_csr_create_dist: halo lists disagree across ranks (pattern not "
                                     "structurally symmetric)");
    return PSK_OK;
}

}  // namespace psk

using namespace psk;

extern "C" {

int psk_fd2d_dist_plan(int64_t m, int32_t nranks, int32_t rank, int64_t *row_begin, int64_t *row_end,
                       int64_t *ncols, int64_t *halo_lo, int64_t *halo_hi) {
    FdPlan p;
    PSK_TRY(fd2d_plan(m, nranks, rank, p));
    if (row_begin) *row_begin = p.rb;
    if (row_end) *row_end = p.re;
    if (ncols) *ncols = p.ncols;
    if (halo_lo) *halo_lo = p.halo_lo;
    if (halo_hi) *halo_hi = p.halo_hi;
    return PSK_OK;
}

int psk_comm_unique_id(uint8_t *id) {
    if (!id) return fail(PSK_ERR_ARG, "NULL id");
    static_assert(sizeof(ncclUniqueId) <= PSK_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId uid;
    PSK_RCCL(ncclGetUniqueId(&uid));
    std::memset(id, 0, PSK_UNIQUE_ID_BYTES);
    std::memcpy(id, &uid, sizeof(uid));
    return PSK_OK;
}

int psk_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, psk_comm **out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(PSK_ERR_ARG, "psk_comm_init: bad arguments");
    psk_comm *c = new psk_comm();
    c->nranks = nranks;
    c->rank = rank;
    hipError_t e = hipGetDevice(&c->device);
    if (e != hipSuccess) {
        delete c;
        return fail(PSK_ERR_HIP, "hipGetDevice");
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(PSK_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    rccl_comm_count(1);
    *out = c;
    return PSK_OK;
}

int psk_comm_init_dry(int32_t nranks, int32_t rank, psk_comm **out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) return fail(PSK_ERR_ARG, "psk_comm_init_dry: bad arguments");
    psk_comm *c = new psk_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->dry = true;
    if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
    *out = c;
    return PSK_OK;
}

// Attach the host-shared mailbox `name` to the communicator (collective: every rank of c, one node).
// Each rank maps the segment, arms its own reader slots, then waits until all P have attached.
int psk_comm_mailbox(psk_comm *c, const char *name) {
    if (!c || !name || name[0] != '/' || std::strlen(name) > 200)
        return fail(PSK_ERR_ARG, "psk_comm_mailbox: bad arguments (name must start with '/')");
    if (c->dry) return fail(PSK_ERR_UNSUPPORTED, "psk_comm_mailbox: dry communicator");
    if (c->mb) return fail(PSK_ERR_ARG, "psk_comm_mailbox: already attached");
    Mailbox *m = new Mailbox();
    m->name = name;
    m->P = c->nranks;
    m->rank = c->rank;
    m->bytes = kMbHeader + (size_t)m->P * kMbRing * m->P * kMbW * sizeof(uint64_t);
    auto bail = [&](int code, const std::string &msg) {
        c->mb = m;
        mbox_close(c);
        return fail(code, "psk_comm_mailbox: " + msg);
    };
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        delete m;
        return fail(PSK_ERR_ARG, std::string("psk_comm_mailbox: shm_open ") + name);
    }
    struct stat st;
    if (fstat(fd, &st) == 0 && (size_t)st.st_size < m->bytes && ftruncate(fd, (off_t)m->bytes) != 0) {
        close(fd);
        delete m;
        return fail(PSK_ERR_ALLOC, "psk_comm_mailbox: ftruncate");
    }
    void *p = mmap(nullptr, m->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        delete m;
        return fail(PSK_ERR_ALLOC, "psk_comm_mailbox: mmap");
    }
    m->host = static_cast<char *>(p);
    // mapped for the kernels (fine-grained: system-scope stores and loads are coherent across devices)
    if (hipHostRegister(m->host, m->bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
        (void)hipGetLastError();
        munmap(m->host, m->bytes);
        m->host = nullptr;
        return bail(PSK_ERR_HIP, "hipHostRegister of the shared segment");
    }
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, m->host, 0) != hipSuccess) return bail(PSK_ERR_HIP, "hipHostGetDevicePointer");
    m->dev = reinterpret_cast<uint64_t *>(static_cast<char *>(dp) + kMbHeader);
    uint64_t *slots = reinterpret_cast<uint64_t *>(m->host + kMbHeader);
    for (int64_t e = 0; e < kMbRing; ++e)   // this rank's reader slots: only it reads and re-arms them
        for (int r = 0; r < m->P; ++r)
            for (int k = 0; k < kMbW; ++k) slots[mb_index(*m, m->rank, e, r, k)] = kMbSentinel;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    auto *attached = reinterpret_cast<std::atomic<int32_t> *>(m->host);
    attached->fetch_add(1);
    const auto t0 = std::chrono::steady_clock::now();
    while (attached->load() < m->P) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return bail(PSK_ERR_RCCL, "peers did not attach");
        std::this_thread::yield();
    }
    c->mb = m;
    return PSK_OK;
}

// mailbox self-check: each rank stores (rank*4096 + r, -(rank*4096 + r)) into exchange r the way a
// solver's grid-sum finisher does, gathers the P pairs and verifies them (bounded waits: a value that
// never arrives is reported, not waited for). Collective: every rank of c, the same rounds.
__global__ void mbox_check_put_kernel(GridSum gs, double v) {
    if (threadIdx.x == 0) {
        const double r[2] = {v, -v};
        gridsum_mail<2>(gs, r);
    }
}

extern "C" int psk_comm_mailbox_check(psk_comm *c, int32_t rounds) {
    if (!c || !c->mb || rounds < 1) return fail(PSK_ERR_ARG, "psk_comm_mailbox_check: no mailbox attached");
    Context *cx;
    PSK_TRY(ctx(&cx));
    const int P = c->nranks;
    DevBuf rb;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } rel{rb};
    PSK_TRY(rb.ensure((size_t)P * 2 * sizeof(double)));
    std::vector<double> h((size_t)P * 2);
    for (int r = 0; r < rounds; ++r) {
        GridSum gs{};
        const uint64_t seq = mbox_next(c, &gs);
        hipLaunchKernelGGL(mbox_check_put_kernel, dim3(1), dim3(64), 0, cx->stream, gs, (double)(c->rank * 4096 + r));
        PSK_HIP(hipGetLastError());
        PSK_TRY(mbox_gather(c, seq, 2, rb.as<double>(), nullptr, cx->stream));
        PSK_HIP(hipMemcpyAsync(h.data(), rb.p, h.size() * sizeof(double), hipMemcpyDeviceToHost, cx->stream));
        PSK_HIP(hipStreamSynchronize(cx->stream));
        PSK_TRY(gridsum_check(cx));   // a wait that expired (bit 8)
        for (int q = 0; q < P; ++q)
            if (h[2 * q] != (double)(q * 4096 + r) || h[2 * q + 1] != -(double)(q * 4096 + r))
                return fail(PSK_ERR_RCCL, "psk_comm_mailbox_check: rank " + std::to_string(q) + "'s value of exchange " +
                                              std::to_string(r) + " is wrong");
    }
    return PSK_OK;
}

int psk_comm_destroy(psk_comm *c) {
    if (!c) return PSK_OK;
    mbox_close(c);
    if (c->nccl) {
        (void)ncclCommDestroy(c->nccl);
        rccl_comm_count(-1);
    }
    shm_close(c);
    delete c;
    return PSK_OK;
}

int psk_csr_create_fd2d_dist(double a, double b, int64_t m, psk_comm *cm, psk_csr **out,
                             int64_t *row_begin, int64_t *row_end) {
    if (!cm || !out || m < 1) return fail(PSK_ERR_ARG, "psk_csr_create_fd2d_dist: bad arguments");
    const int r = cm->rank;
    if ((m == 1 ? 1 : 5 * m * m - 4 * m) > kMaxNnz) return fail(PSK_ERR_UNSUPPORTED, "nnz > int32");
    FdPlan plan;
    PSK_TRY(fd2d_plan(m, cm->nranks, r, plan));
    Context *c;
    PSK_TRY(ctx(&c));
    const int64_t rb = plan.rb, re = plan.re, nloc = plan.nloc;
    const bool lo = plan.halo_lo > 0, hi = plan.halo_hi > 0;
    psk_csr *A = new psk_csr();
    A->n = nloc;
    A->ncols = plan.ncols;
    A->n_global = m * m;
    A->row_begin = rb;
    A->row_end = re;
    A->comm = cm;
    A->device = c->device;
    // nnz of the local rows from the closed-form rowptr
    auto fdrp = [m](int64_t k) -> int64_t {
        int64_t mk = k < m ? k : m, top = k - m * (m - 1);
        if (top < 0) top = 0;
        return 5 * k - mk - top - (k + m - 1) / m - k / m;
    };
    A->nnz = fdrp(re) - fdrp(rb);
    A->tile_rows = tile_rows_for(nloc, A->nnz);
    int rc = PSK_OK;
    if (hipMalloc(&A->rowptr, (size_t)(nloc + 1) * 4) != hipSuccess ||
        hipMalloc(&A->colidx, (size_t)A->nnz * 4) != hipSuccess ||
        hipMalloc(&A->vals, (size_t)A->nnz * 8) != hipSuccess)
        rc = fail(PSK_ERR_ALLOC, "fd2d_dist alloc");
    if (rc == PSK_OK) rc = fd2d_fill(A, m, a, b, rb, re, lo ? rb - m : rb, c->stream);
    if (rc == PSK_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(PSK_ERR_HIP, "fd2d_dist sync");
    if (rc == PSK_OK) rc = csr_choose_layout(A, c->stream);
    if (rc != PSK_OK) {
        psk_csr_destroy(A);
        return rc;
    }
    if (lo) {
        HaloPeer p{};
        p.rank = r - 1;
        p.send_count = m;        // our first grid line
        p.send_begin = 0;
        p.recv_count = m;        // their last grid line -> halo_lo
        p.recv_offset = 0;
        p.send_idx = nullptr;
        A->peers.push_back(p);
    }
    if (hi) {
        HaloPeer p{};
        p.rank = r + 1;
        p.send_count = m;        // our last grid line
        p.send_begin = nloc - m;
        p.recv_count = m;        // their first grid line -> halo_hi
        p.recv_offset = lo ? m : 0;
        p.send_idx = nullptr;
        A->peers.push_back(p);
    }
    if (lo)
        for (int64_t j = rb - m; j < rb; ++j) A->halo_cols.push_back(j);
    if (hi)
        for (int64_t j = re; j < re + m; ++j) A->halo_cols.push_back(j);
    *out = A;
    if (row_begin) *row_begin = rb;
    if (row_end) *row_end = re;
    return PSK_OK;
}

int psk_csr_create_dist(int64_t n_global, const int64_t *row_starts, const int64_t *rowptr, const int32_t *colidx,
                        const double *vals, psk_comm *cm, psk_csr **out) {
    if (!cm || !out || !row_starts || !rowptr || n_global < 0)
        return fail(PSK_ERR_ARG, "psk_csr_create_dist: bad arguments");
    const int P = cm->nranks, r = cm->rank;
    if (row_starts[0] != 0 || row_starts[P] != n_global)
        return fail(PSK_ERR_ARG, "psk_csr_create_dist: row_starts must run from 0 to n_global");
    for (int q = 0; q < P; ++q)
        if (row_starts[q + 1] < row_starts[q]) return fail(PSK_ERR_ARG, "psk_csr_create_dist: row_starts not monotone");
    if (n_global >= INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "psk_csr_create_dist: int32 columns required");
    const int64_t nloc = row_starts[r + 1] - row_starts[r];
    for (int64_t i = 0; i < nloc; ++i)
        if (rowptr[i + 1] < rowptr[i]) return fail(PSK_ERR_ARG, "psk_csr_create_dist: rowptr not monotone");
    const int64_t nnz = rowptr[nloc] - rowptr[0];
    if (nnz > kMaxNnz) return fail(PSK_ERR_UNSUPPORTED, "psk_csr_create_dist: local nnz exceeds int32");
    if (nnz > 0 && (!colidx || !vals)) return fail(PSK_ERR_ARG, "psk_csr_create_dist: NULL entries");
    DistPlan pl;
    PSK_TRY(dist_plan(n_global, row_starts, P, r, rowptr, colidx, pl));
    if (!cm->dry) PSK_TRY(dist_verify(cm, pl));
    Context *c;
    PSK_TRY(ctx(&c));
    psk_csr *A = new psk_csr();
    A->n = nloc;
    A->ncols = nloc + (int64_t)pl.halo.size();
    A->nnz = nnz;
    A->tile_rows = tile_rows_for(nloc, nnz);
    A->n_global = n_global;
    A->row_begin = pl.rb;
    A->row_end = pl.re;
    A->comm = cm;
    A->device = c->device;
    A->halo_cols = pl.halo;
    std::vector<int32_t> rp32((size_t)nloc + 1);
    for (int64_t i = 0; i <= nloc; ++i) rp32[(size_t)i] = (int32_t)(rowptr[i] - rowptr[0]);
    std::vector<int32_t> pack;
    for (int q = 0; q < P; ++q) {
        const std::vector<int32_t> &sr = pl.send_rows[(size_t)q];
        if (pl.recv_cnt[(size_t)q] == 0 && sr.empty()) continue;
        HaloPeer p{};
        p.rank = q;
        p.recv_count = pl.recv_cnt[(size_t)q];
        p.recv_offset = pl.recv_off[(size_t)q];
        p.send_count = (int64_t)sr.size();
        p.send_idx = nullptr;
        p.send_begin = sr.empty() ? 0 : sr[0];
        p.pack_off = 0;
        const bool contiguous = sr.empty() || (int64_t)sr.back() - sr.front() + 1 == (int64_t)sr.size();
        if (!contiguous) {
            p.pack_off = (int64_t)pack.size();
            pack.insert(pack.end(), sr.begin(), sr.end());
            p.send_idx = reinterpret_cast<int32_t *>(1);   // resolved after the upload below
        }
        A->peers.push_back(p);
    }
    int rc = PSK_OK;
    const size_t mn = nnz > 0 ? (size_t)nnz : 1;
    if (hipMalloc(&A->rowptr, (size_t)(nloc + 1) * 4) != hipSuccess || hipMalloc(&A->colidx, mn * 4) != hipSuccess ||
        hipMalloc(&A->vals, mn * 8) != hipSuccess)
        rc = fail(PSK_ERR_ALLOC, "psk_csr_create_dist: alloc");
    if (rc == PSK_OK && !pack.empty()) {
        A->pack_count = (int64_t)pack.size();
        if (hipMalloc(&A->pack_idx, pack.size() * 4) != hipSuccess) rc = fail(PSK_ERR_ALLOC, "halo pack alloc");
        else if (hipMemcpy(A->pack_idx, pack.data(), pack.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            rc = fail(PSK_ERR_HIP, "halo pack upload");
        if (rc == PSK_OK) rc = A->sendbuf.ensure(pack.size() * 8);
        for (HaloPeer &p : A->peers)
            if (p.send_idx) p.send_idx = A->pack_idx + p.pack_off;
    } else {
        for (HaloPeer &p : A->peers) p.send_idx = nullptr;
    }
    if (rc == PSK_OK && (hipMemcpy(A->rowptr, rp32.data(), rp32.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
                         (nnz > 0 && hipMemcpy(A->colidx, pl.lcol.data(), (size_t)nnz * 4, hipMemcpyHostToDevice) !=
                                         hipSuccess) ||
                         (nnz > 0 && hipMemcpy(A->vals, vals, (size_t)nnz * 8, hipMemcpyHostToDevice) != hipSuccess) ||
                         (nnz == 0 && (hipMemset(A->colidx, 0, 4) != hipSuccess || hipMemset(A->vals, 0, 8) != hipSuccess))))
        rc = fail(PSK_ERR_HIP, "psk_csr_create_dist: upload");
    if (rc == PSK_OK) rc = csr_choose_layout(A, c->stream);
    if (rc != PSK_OK) {
        psk_csr_destroy(A);
        return rc;
    }
    *out = A;
    return PSK_OK;
}

int psk_csr_halo_peers(const psk_csr *A, int32_t *ranks, int64_t *send_counts, int64_t *recv_counts,
                       int64_t *recv_offsets, int32_t *npeers) {
    if (!A || !npeers) return fail(PSK_ERR_ARG, "psk_csr_halo_peers: bad arguments");
    *npeers = (int32_t)A->peers.size();
    for (size_t k = 0; k < A->peers.size(); ++k) {
        if (ranks) ranks[k] = A->peers[k].rank;
        if (send_counts) send_counts[k] = A->peers[k].send_count;
        if (recv_counts) recv_counts[k] = A->peers[k].recv_count;
        if (recv_offsets) recv_offsets[k] = A->peers[k].recv_offset;
    }
    return PSK_OK;
}

int psk_csr_halo_pack(const psk_csr *Ac, const double *x, double *out) {
    if (!Ac || !x || !out) return fail(PSK_ERR_ARG, "psk_csr_halo_pack: NULL argument");
    psk_csr *A = const_cast<psk_csr *>(Ac);
    Context *c;
    PSK_TRY(ctx(&c));
    hipStream_t s = c->stream;
    if (A->pack_count > 0) {   // the exact kernel halo_exchange runs
        hipLaunchKernelGGL(halo_pack_kernel, dim3((unsigned)((A->pack_count + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           s, A->pack_count, A->pack_idx, x, A->sendbuf.as<double>());
        PSK_HIP(hipGetLastError());
    }
    int64_t o = 0;
    for (const HaloPeer &p : A->peers) {
        if (p.send_count > 0) {
            const double *src = p.send_idx ? A->sendbuf.as<double>() + p.pack_off : x + p.send_begin;
            PSK_HIP(hipMemcpyAsync(out + o, src, (size_t)p.send_count * 8, hipMemcpyDeviceToDevice, s));
        }
        o += p.send_count;
    }
    PSK_HIP(hipStreamSynchronize(s));
    return PSK_OK;
}

int psk_csr_halo_cols(const psk_csr *A, int64_t *cols, int64_t *count) {
    if (!A || !count) return fail(PSK_ERR_ARG, "psk_csr_halo_cols: bad arguments");
    *count = (int64_t)A->halo_cols.size();
    if (cols) std::copy(A->halo_cols.begin(), A->halo_cols.end(), cols);
    return PSK_OK;
}


}  // extern "C"
