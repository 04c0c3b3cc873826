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
#include <vector>

namespace psk {

struct AmgHierarchy {
    int L = 0, num_iters = 0, nu_pre = 0, nu_post = 0;
    double tau = 0.0;
    std::vector<psk_csr *> A, P, R;
    std::vector<psk_prec *> S;
    psk_prec *coarse = nullptr;
    std::vector<DevBuf> x, f, r, t;   // per level (f unused on the finest level: f = v)
    DevBuf scal;                      // [0] = ||v||^2, [1] = flag (as int64), partials after
};

void amg_free(AmgHierarchy *h) {
    if (!h) return;
    for (auto &b : h->x) b.release();
    for (auto &b : h->f) b.release();
    for (auto &b : h->r) b.release();
    for (auto &b : h->t) b.release();
    h->scal.release();
    delete h;
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
    for (int it = 0; it < nu; ++it) {
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
