// ilu.hip — right-ILUT apply on the device (RightILUTPreconditioner.applyRight, ILUTPreconditioner.py:70-78).
//
// The reference calls SuperLU's ILU.solve(v) (scipy SuperLU, dgstrs): with Pr A Pc ~= L U,
//     bb[perm_r[i]] = v[i];  y = L^-1 bb (unit lower);  z = U^-1 y;  out[i] = z[perm_c[i]].
// The factors come from the same third-party factorisation on the host (scipy spilu, exactly the
// reference's call, ILUTPreconditioner.py:51-53): they are uploaded once per form() and the two
// triangular solves run on the GPU.
//
// Sparse triangular solve, "sync-free": one wave per row, rows dealt to a co-resident grid in a
// level-sorted topological order computed on the host once per form() (k-th row of that order ->
// wave k mod W, each wave walks its rows in order; every row depends only on rows earlier in the
// order, so the first unsolved row can always proceed). Level order instead of index order cut the
// apply at FD m=1024 from 255 ms to 17 ms (a wave stuck on a deep row no longer blocks shallow rows
// queued behind it). A row's lanes load its entries
// (coalesced), wait for each dependency x[c] to be PUBLISHED, then one deterministic wave reduction
// and lane 0 publishes x[i]. Publication is the value itself: the output is pre-filled with a
// signalling-NaN sentinel that arithmetic never produces, each x[i] is written by ONE 8-byte
// agent-scope store (sc1) and read by agent-scope relaxed loads that bypass the non-coherent L1
// (MI355X_MICROARCH.md, hand-off granule R2: "the data IS the flag"). Every spin is bounded and
// reports PSK_ERR instead of hanging.
#include "psk_internal.hpp"

#include <algorithm>
#include <vector>

namespace psk {

constexpr uint64_t kSentinel = 0x7FF4DEAD0000BEEFull;   // sNaN payload: never an arithmetic result
constexpr int64_t kMaxSpins = 1ll << 24;

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

__global__ void fill_sentinel_kernel(int64_t n, double *x) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) reinterpret_cast<uint64_t *>(x)[i] = kSentinel;
}

// UPPER == false: x = L^-1 rhs[perm] (unit diagonal, strictly-lower entries only)
// UPPER == true : x = U^-1 rhs       (strictly-upper entries + diag)
// Rows are visited in `order`, a topological order sorted by dependency level (host-computed):
// every wave walks order[wave], order[wave + W], ... so all waves work on the shallow levels first
// and a row waiting on a deep level never blocks shallower rows queued behind it on its wave.
template <bool UPPER>
__global__ __launch_bounds__(kBlock) void sptrsv_kernel(int64_t n, const int32_t *__restrict__ rp,
                                                        const int32_t *__restrict__ ci, const double *__restrict__ va,
                                                        const double *__restrict__ diag, const double *__restrict__ rhs,
                                                        const int32_t *__restrict__ rhs_idx, double *x,
                                                        int32_t *err, const int32_t *__restrict__ order) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const int64_t W = (int64_t)gridDim.x * kWaves;
    for (int64_t k = wave; k < n; k += W) {
        const int64_t i = order[k];
        const int32_t s = rp[i], e = rp[i + 1];
        double acc = 0.0;
        for (int32_t base = s; base < e; base += 64) {
            const int32_t idx = base + lane;
            if (idx < e) {
                const int32_t c = ci[idx];
                const double v = va[idx];
                double xv = load_pub(x + c);
                int64_t spins = 0;
                while (is_sentinel(xv)) {
                    if (++spins > kMaxSpins) {
                        atomicExch(err, 1);
                        xv = 0.0;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    xv = load_pub(x + c);
                }
                acc = fma(v, xv, acc);
            }
        }
        const double sum = wave_sum(acc);
        if (lane == 0) {
            const double bi = rhs_idx ? rhs[rhs_idx[i]] : rhs[i];
            double r = bi - sum;
            if (UPPER) r = r / diag[i];
            store_pub(x + i, r);
        }
    }
}

__global__ void gather_perm_kernel(int64_t n, const double *__restrict__ z, const int32_t *__restrict__ perm,
                                   double *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = z[perm[i]];   // out = z[perm_c]
}

static int sptrsv_grid(const Context *c, const void *kern) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, 0) != hipSuccess) per_cu = 1;
    if (per_cu > 2) per_cu = 2;   // margin below the occupancy answer (MI355X_MICROARCH.md residency)
    if (per_cu < 1) per_cu = 1;
    return c->num_cus * per_cu;
}

// out = M^-1 v for an ILU preconditioner (all device pointers; out may not alias v)
int ilu_apply(const psk_prec *M, const double *v, double *out, hipStream_t s) {
    const int64_t n = M->n;
    if (n == 0) return PSK_OK;
    Context *c;
    PSK_TRY(ctx(&c));
    const unsigned fb = (unsigned)((n + kBlock - 1) / kBlock);
    double *y = M->work, *z = M->work + n;
    int32_t *err = M->err;
    hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((2 * n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       2 * n, y);   // y and z are contiguous
    PSK_HIP(hipGetLastError());
    {
        const void *kl = reinterpret_cast<const void *>(&sptrsv_kernel<false>);
        const int g = sptrsv_grid(c, kl);
        int64_t nn = n;
        const int32_t *rp = M->l_rowptr, *ci = M->l_colidx, *pinv = M->perm_r_inv;
        const double *va = M->l_vals, *dg = nullptr;
        const int32_t *ord = M->l_order;
        void *args[] = {&nn, &rp, &ci, &va, &dg, &v, &pinv, &y, &err, &ord};
        PSK_HIP(hipLaunchCooperativeKernel(kl, dim3(g), dim3(kBlock), args, 0, s));
    }
    {
        const void *ku = reinterpret_cast<const void *>(&sptrsv_kernel<true>);
        const int g = sptrsv_grid(c, ku);
        int64_t nn = n;
        const int32_t *rp = M->u_rowptr, *ci = M->u_colidx, *none = nullptr;
        const double *va = M->u_vals, *dg = M->u_diag, *yy = y;
        const int32_t *ord = M->u_order;
        void *args[] = {&nn, &rp, &ci, &va, &dg, &yy, &none, &z, &err, &ord};
        PSK_HIP(hipLaunchCooperativeKernel(ku, dim3(g), dim3(kBlock), args, 0, s));
    }
    hipLaunchKernelGGL(gather_perm_kernel, dim3(fb), dim3(kBlock), 0, s, n, z, M->perm_c, out);
    PSK_HIP(hipGetLastError());
    return PSK_OK;
}

int ilu_check_error(const psk_prec *M, hipStream_t s) {
    int32_t h = 0;
    PSK_HIP(hipMemcpyAsync(&h, M->err, 4, hipMemcpyDeviceToHost, s));
    PSK_HIP(hipStreamSynchronize(s));
    if (h) return fail(PSK_ERR_HIP, "ILU triangular solve: dependency wait exceeded its bound (not co-resident?)");
    return PSK_OK;
}

}  // namespace psk

using namespace psk;

template <class T>
static int upload(T **d, const std::vector<T> &h) {
    if (h.empty()) {
        *d = nullptr;
        return PSK_OK;
    }
    if (hipMalloc(d, h.size() * sizeof(T)) != hipSuccess) return fail(PSK_ERR_ALLOC, "hipMalloc ILU");
    if (hipMemcpy(*d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return fail(PSK_ERR_HIP, "hipMemcpy ILU");
    return PSK_OK;
}

extern "C" int psk_prec_create_ilu(int64_t n, const int32_t *l_rowptr, const int32_t *l_colidx, const double *l_vals,
                                   const int32_t *u_rowptr, const int32_t *u_colidx, const double *u_vals,
                                   const int32_t *perm_r, const int32_t *perm_c, psk_prec **out) {
    if (!out || n < 0 || !l_rowptr || !u_rowptr || !perm_r || !perm_c)
        return fail(PSK_ERR_ARG, "psk_prec_create_ilu: NULL argument");
    // split: L strictly lower (unit diagonal implied), U strictly upper + diagonal
    std::vector<int32_t> lrp(n + 1, 0), urp(n + 1, 0), lci, uci, pinv(n), pc(perm_c, perm_c + n);
    std::vector<double> lva, uva, udg(n, 0.0);
    for (int64_t i = 0; i < n; ++i) {
        for (int32_t j = l_rowptr[i]; j < l_rowptr[i + 1]; ++j) {
            const int32_t c = l_colidx[j];
            if (c < 0 || c > i) return fail(PSK_ERR_ARG, "ILU: L has an entry above the diagonal");
            if (c == i) continue;
            lci.push_back(c);
            lva.push_back(l_vals[j]);
        }
        lrp[i + 1] = (int32_t)lci.size();
        bool has_diag = false;
        for (int32_t j = u_rowptr[i]; j < u_rowptr[i + 1]; ++j) {
            const int32_t c = u_colidx[j];
            if (c < i || c >= n) return fail(PSK_ERR_ARG, "ILU: U has an entry below the diagonal");
            if (c == i) {
                udg[i] += u_vals[j];
                has_diag = true;
                continue;
            }
            uci.push_back(c);
            uva.push_back(u_vals[j]);
        }
        if (!has_diag) return fail(PSK_ERR_ARG, "ILU: U has a missing diagonal entry");
        urp[i + 1] = (int32_t)uci.size();
    }
    std::vector<char> seen(n, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int32_t p = perm_r[i];
        if (p < 0 || p >= n || seen[p] || perm_c[i] < 0 || perm_c[i] >= n)
            return fail(PSK_ERR_ARG, "ILU: invalid permutation");
        seen[p] = 1;
        pinv[p] = (int32_t)i;   // bb[perm_r[i]] = v[i]  <=>  bb[j] = v[pinv[j]]
    }
    // dependency levels -> counting-sort the rows by level (stable: index order inside a level)
    auto level_order = [n](const std::vector<int32_t> &rp, const std::vector<int32_t> &ci, bool upper,
                           std::vector<int32_t> &order, int64_t &nlev) {
        std::vector<int32_t> lev(n, 0);
        int32_t maxl = -1;
        for (int64_t t = 0; t < n; ++t) {
            const int64_t i = upper ? n - 1 - t : t;
            int32_t l = 0;
            for (int32_t j = rp[i]; j < rp[i + 1]; ++j) l = std::max(l, lev[ci[j]] + 1);
            lev[i] = l;
            maxl = std::max(maxl, l);
        }
        nlev = maxl + 1;
        std::vector<int64_t> cnt((size_t)nlev + 1, 0);
        for (int64_t i = 0; i < n; ++i) cnt[lev[i] + 1]++;
        for (int64_t l = 0; l < nlev; ++l) cnt[l + 1] += cnt[l];
        order.assign(n, 0);
        for (int64_t t = 0; t < n; ++t) {
            const int64_t i = upper ? n - 1 - t : t;
            order[cnt[lev[i]]++] = (int32_t)i;
        }
    };
    std::vector<int32_t> lord, uord;
    int64_t nlev_l = 0, nlev_u = 0;
    level_order(lrp, lci, false, lord, nlev_l);
    level_order(urp, uci, true, uord, nlev_u);

    Context *c;
    PSK_TRY(ctx(&c));
    psk_prec *M = new psk_prec();
    M->kind = PSK_PREC_ILU;
    M->l_levels = nlev_l;
    M->u_levels = nlev_u;
    M->n = n;
    int rc = PSK_OK;
    if (rc == PSK_OK) rc = upload(&M->l_rowptr, lrp);
    if (rc == PSK_OK) rc = upload(&M->l_colidx, lci);
    if (rc == PSK_OK) rc = upload(&M->l_vals, lva);
    if (rc == PSK_OK) rc = upload(&M->u_rowptr, urp);
    if (rc == PSK_OK) rc = upload(&M->u_colidx, uci);
    if (rc == PSK_OK) rc = upload(&M->u_vals, uva);
    if (rc == PSK_OK) rc = upload(&M->u_diag, udg);
    if (rc == PSK_OK) rc = upload(&M->perm_r_inv, pinv);
    if (rc == PSK_OK) rc = upload(&M->perm_c, pc);
    if (rc == PSK_OK) rc = upload(&M->l_order, lord);
    if (rc == PSK_OK) rc = upload(&M->u_order, uord);
    if (rc == PSK_OK && n > 0 && hipMalloc(&M->work, (size_t)(2 * n) * sizeof(double)) != hipSuccess)
        rc = fail(PSK_ERR_ALLOC, "ILU work");
    if (rc == PSK_OK && hipMalloc(&M->err, sizeof(int32_t)) != hipSuccess) rc = fail(PSK_ERR_ALLOC, "ILU err");
    if (rc == PSK_OK && hipMemset(M->err, 0, sizeof(int32_t)) != hipSuccess) rc = fail(PSK_ERR_HIP, "ILU err");
    if (rc != PSK_OK) {
        psk_prec_destroy(M);
        return rc;
    }
    M->nnz_l = (int64_t)lci.size();
    M->nnz_u = (int64_t)uci.size();
    *out = M;
    return PSK_OK;
}
