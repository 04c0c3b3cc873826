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
    PSK_RCCL(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, A->comm->nccl, s));
    return PSK_OK;
}

}  // namespace psk

using namespace psk;

extern "C" {

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

int psk_comm_destroy(psk_comm *c) {
    if (!c) return PSK_OK;
    if (c->nccl) (void)ncclCommDestroy(c->nccl);
    delete c;
    return PSK_OK;
}

int psk_csr_create_fd2d_dist(double a, double b, int64_t m, psk_comm *cm, psk_csr **out,
                             int64_t *row_begin, int64_t *row_end) {
    if (!cm || !out || m < 1) return fail(PSK_ERR_ARG, "psk_csr_create_fd2d_dist: bad arguments");
    const int P = cm->nranks, r = cm->rank;
    if (P > m) return fail(PSK_ERR_ARG, "fd2d_dist: more ranks than grid lines");
    if ((m == 1 ? 1 : 5 * m * m - 4 * m) > INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "nnz > int32");
    Context *c;
    PSK_TRY(ctx(&c));
    // whole grid lines per rank
    const int64_t l0 = m * r / P, l1 = m * (r + 1) / P;
    const int64_t rb = l0 * m, re = l1 * m, nloc = re - rb;
    const bool lo = l0 > 0, hi = l1 < m;
    psk_csr *A = new psk_csr();
    A->n = nloc;
    A->ncols = nloc + (lo ? m : 0) + (hi ? m : 0);
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
