// dist.hip — row-block sharding across the GPUs of one node (one process per GPU, RCCL over xGMI).
//
// No reference counterpart: PySolvers is single-process. The sharded PCG is the same loop as
// pcg.hip; per iteration it adds (1) a halo exchange of the search direction p with the two
// neighbouring ranks (grouped ncclSend/ncclRecv of one grid line each way for the 5-point FD
// matrix: m doubles per side), and (2) two in-place ncclAllReduce(sum) of the per-workgroup dot
// partials (p.Ap; then r.r and u.r fused). Every rank then re-reduces the summed partials in the
// same fixed order, so all ranks hold bit-identical scalars and stop on the same iteration
// without further communication.
#include "psk_internal.hpp"

#include <climits>
#include <cmath>

namespace psk {

int halo_exchange(psk_csr *A, double *x, hipStream_t s) {
    if (!A->comm || A->peers.empty()) return PSK_OK;
    if (A->comm->dry) return PSK_OK;   // the caller supplied the halo entries
    ncclComm_t nc = A->comm->nccl;
    PSK_RCCL(ncclGroupStart());
    for (const HaloPeer &p : A->peers) {
        if (p.send_count > 0) {
            if (p.send_idx) return fail(PSK_ERR_UNSUPPORTED, "indexed halo sends not built");
            PSK_RCCL(ncclSend(x + p.send_begin, (size_t)p.send_count, ncclDouble, p.rank, nc, s));
        }
        if (p.recv_count > 0)
            PSK_RCCL(ncclRecv(x + A->n + p.recv_offset, (size_t)p.recv_count, ncclDouble, p.rank, nc, s));
    }
    PSK_RCCL(ncclGroupEnd());
    return PSK_OK;
}

int allreduce_sum(psk_csr *A, double *buf, int64_t count, hipStream_t s) {
    if (!A->comm || A->comm->nranks == 1) return PSK_OK;
    if (A->comm->dry) return fail(PSK_ERR_UNSUPPORTED, "collective on a dry (RCCL-less) communicator");
    PSK_RCCL(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, A->comm->nccl, s));
    return PSK_OK;
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

int psk_comm_destroy(psk_comm *c) {
    if (!c) return PSK_OK;
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    delete c;
    return PSK_OK;
}

int psk_csr_create_fd2d_dist(double a, double b, int64_t m, psk_comm *cm, psk_csr **out,
                             int64_t *row_begin, int64_t *row_end) {
    if (!cm || !out || m < 1) return fail(PSK_ERR_ARG, "psk_csr_create_fd2d_dist: bad arguments");
    const int r = cm->rank;
    if ((m == 1 ? 1 : 5 * m * m - 4 * m) > INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "nnz > int32");
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
    *out = A;
    if (row_begin) *row_begin = rb;
    if (row_end) *row_end = re;
    return PSK_OK;
}

int psk_csr_create_dist(int64_t, int64_t, int64_t, const int64_t *, const int32_t *, const double *,
                        psk_comm *, psk_csr **) {
    return fail(PSK_ERR_UNSUPPORTED, "psk_csr_create_dist: general row-block sharding not built yet");
}

}  // extern "C"
