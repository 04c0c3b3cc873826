// gmres.hip — device-resident right-preconditioned GMRES (GMRESSolver.solve, GMRESSolver.py:55-180).
//
// Krylov basis Q lives in HBM column-major (each q_j contiguous, n x (K+1)); the Hessenberg
// column, the Givens table and g live in HBM too and are advanced by one lane of workgroup 0.
// Per Arnoldi step k (one-shot launches, one 512-element tile per workgroup; no host sync):
//   G1      u = A M^-1 q_k, with q_0.u finished in-launch (gridsum)      (:107, first MGS dot)
//   G2_j    h_jk (G1's or G2_{j-1}'s grid sum); u -= h_jk q_j; q_{j+1}.u (:110-112, MGS, j=0..k)
//           finished in-launch (for j==k u.u, the norm)
//   G3      h_{k+1,k} = ||u||; breakdown test; q_{k+1} = u / h_{k+1,k};  (:115-125)
//           workgroup 0: old rotations, new rotation, g update, |g_{k+1}|, convergence (:133-158)
// Bytes per step (algorithmic): the SpMV's, then 32n per G2_j (u read + written, q_j, q_{j+1}),
// 24n for G2_k, 16n for G3.
// On convergence the (k+1)^2 triangular-ish least-squares system is solved on the host (it is
// 31x31 at config 3; LU with partial pivoting as LAPACK dgesv, :159), then
//   x = M^-1 (Q[:, :k+1] y) on the device (:160) and the true residual ||b - A x|| (:163-164).
// restart == 0 reproduces the reference (one cycle, Krylov dimension = maxiter). restart = m > 0
// is the restarted GMRES(m) the reference lacks: cycles of m steps from r = b - A x.
// Reference defects: self.precond never set (:71) -> we always form M;
// NameError at maxiter (:180) -> we return the MAXITER status handleMaxiter would have built.
#include "psk_internal.hpp"

#include <cmath>
#include <cstdio>

namespace psk {

struct GmresState {
    int32_t done;    // 0 running, 1 converged (recursive test or Arnoldi breakdown)
    int32_t brk;     // Arnoldi breakdown flag
    int32_t kconv;   // step k at which `done` was raised
    int32_t zero_b;  // ||b|| == 0
    double normB;
    double tauNormB;
    double rec;      // last |g[k+1]|
    double true_resid;
};

__global__ __launch_bounds__(kBlock) void gm_selfdot_kernel(int64_t n, const double *__restrict__ v,
                                                            double *__restrict__ part) {
    __shared__ double sh[kWaves];
    int64_t t0, t1;
    block_range((n + kVecTile - 1) / kVecTile, t0, t1);
    const int64_t i0 = t0 * kVecTile, i1 = (t1 * kVecTile < n) ? t1 * kVecTile : n;
    double acc = 0.0;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) acc = fma(v[i], v[i], acc);
    const double s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// cycle start: beta = ||r0||, q_0 = r0/beta, g = beta e1 (:90-97)
__global__ __launch_bounds__(kBlock) void gm_start_kernel(int64_t n, const double *__restrict__ r0,
                                                          double *__restrict__ q0, const double *__restrict__ part,
                                                          int np, double *__restrict__ g, int Kp1, GmresState *st,
                                                          double tau, int first, double normb_caller) {
    __shared__ double sh[kWaves];
    const double bb = reduce_partials(part, np, 1, sh);
    const double beta = sqrt(bb);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (first) {
            // self.norm(b)  :66: == npla.norm(r0) since r0 = b, or the caller's norm of b
            const double nb = normb_caller > 0.0 ? normb_caller : beta;
            st->normB = nb;
            st->tauNormB = tau * nb;
            st->zero_b = beta == 0.0;
            if (beta == 0.0) st->done = 1;     // :67-68
        }
        for (int j = 0; j < Kp1; ++j) g[j] = beta * (j == 0 ? 1.0 : 0.0);   // g = beta*e1
    }
    if (beta == 0.0) return;
    int64_t t0, t1;
    block_range((n + kVecTile - 1) / kVecTile, t0, t1);
    const int64_t i0 = t0 * kVecTile, i1 = (t1 * kVecTile < n) ? t1 * kVecTile : n;
    for (int64_t i = i0 + threadIdx.x; i < i1; i += kBlock) q0[i] = r0[i] / beta;   // :91
}

// MGS step j of Arnoldi column k, one-shot (one 512-element tile per workgroup, 16-B accesses):
// h = HBar[j,k] (the previous launch's grid sum), u -= h q_j, and the next dot — q_{j+1}.u, or u.u
// for j == k (the norm of :115) — finished in-launch by gridsum into hout.
__global__ __launch_bounds__(kBlock) void gm_mgs_kernel(int64_t n, double *__restrict__ u,
                                                        const double *__restrict__ qj,
                                                        const double *__restrict__ qnext,
                                                        const double *__restrict__ hin, double *__restrict__ hcol,
                                                        int j, GridSum gs, const GmresState *st) {
    if (st->done) return;
    __shared__ double sh[kWaves];
    const double h = *hin;                                  // HBar[j,k] = np.dot(Q[:,j], u)  :111
    if (blockIdx.x == 0 && threadIdx.x == 0) hcol[j] = h;
    const int64_t i = (int64_t)blockIdx.x * kVecTile + 2 * threadIdx.x;
    uint32_t ticket = 0;
    double acc = 0.0;
    if (i + 1 < n) {
        // q_j is not read again this step (non-temporal); u and q_{j+1} are read by the next launch
        dv2 uv = ld2(u + i);
        const dv2 qv = ld2nt(qj + i);
        dv2 nv = uv;
        if (qnext) nv = ld2(qnext + i);
        ticket = gridsum_ticket(gs);
        uv.x = uv.x - h * qv.x;                             // u -= HBar[j,k]*Q[:,j]  :112
        uv.y = uv.y - h * qv.y;
        st2(u + i, uv);
        if (!qnext) nv = uv;
        acc = fma(nv.x, uv.x, acc);
        acc = fma(nv.y, uv.y, acc);
    } else if (i < n) {
        ticket = gridsum_ticket(gs);
        const double ui = u[i] - h * qj[i];
        u[i] = ui;
        acc = (qnext ? qnext[i] : ui) * ui;
    }
    const double v = block_sum(acc, sh);
    gridsum_publish<1>(gs, &v, sh, ticket);
}

__device__ __forceinline__ void givens_apply(double *x, double c, double s, int i) {
    const double xi = x[i], xi1 = x[i + 1];            // Givens.py:30-34
    x[i] = c * xi + s * xi1;
    x[i + 1] = -s * xi + c * xi1;
}

// h_{k+1,k}, breakdown, q_{k+1}, Givens, convergence; one-shot like gm_mgs_kernel (hsq: the grid
// sum u.u of the last MGS launch)
__global__ __launch_bounds__(kBlock) void gm_normalize_kernel(
    int64_t n, const double *__restrict__ u, double *__restrict__ qnext, const double *__restrict__ hsq,
    double *__restrict__ H, double *__restrict__ R, double *__restrict__ CS, double *__restrict__ g, int ld, int k,
    int64_t it, GmresState *st, double *__restrict__ hist) {
    if (st->done) return;
    const double hk = sqrt(*hsq);                                   // npla.norm(u)  :115
    const double *hcol = H + (int64_t)k * ld;
    double hh = 0.0;
    for (int j = 0; j <= k; ++j) hh += hcol[j] * hcol[j];
    const double hlast = sqrt(hh);                                  // npla.norm(HBar[0:k+1,k])  :121
    const bool brk = fabs(hk) <= 1.0e-16 * hlast;                    // :122
    const int64_t i = (int64_t)blockIdx.x * kVecTile + 2 * threadIdx.x;
    if (!brk) {                                                     // Q[:,k+1] = u / HBar[k+1,k]  :125
        if (i + 1 < n) {
            const dv2 uv = ld2nt(u + i);
            dv2 q;
            q.x = uv.x / hk;
            q.y = uv.y / hk;
            st2(qnext + i, q);
        } else if (i < n) {
            qnext[i] = u[i] / hk;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        H[(int64_t)k * ld + k + 1] = hk;
        double *rc = R + (int64_t)k * ld;
        for (int j = 0; j <= k; ++j) rc[j] = hcol[j];
        rc[k + 1] = hk;
        for (int j = 0; j < k; ++j) givens_apply(rc, CS[2 * j], CS[2 * j + 1], j);   // :133-135
        const double hyp = sqrt(rc[k + 1] * rc[k + 1] + rc[k] * rc[k]);          // Givens.py:8-10
        const double s = rc[k + 1] / hyp;
        const double c = rc[k] / hyp;
        CS[2 * k] = c;
        CS[2 * k + 1] = s;
        givens_apply(rc, c, s, k);                                                 // :145
        givens_apply(g, c, s, k);                                                  // :148
        const double nr = fabs(g[k + 1]);                                          // :152
        hist[it] = nr;
        st->rec = nr;
        if (brk || nr <= st->tauNormB) {                                           // :158
            st->brk = brk;
            st->kconv = k;
            st->done = 1;
        }
    }
}

// x (+)= M^-1 (Q[:, :k1] y)   (:160)
__global__ __launch_bounds__(kBlock) void gm_update_x_kernel(int64_t n, const double *__restrict__ Q,
                                                             int64_t ldq, const double *__restrict__ y, int k1,
                                                             const double *__restrict__ dinv,
                                                             double *__restrict__ x, int accumulate) {
    __shared__ double ys[1024];
    for (int j = threadIdx.x; j < k1 && j < 1024; j += kBlock) ys[j] = y[j];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;
    for (int j = 0; j < k1; ++j) s = fma(Q[(int64_t)j * ldq + i], j < 1024 ? ys[j] : y[j], s);
    const double v = dinv ? dinv[i] * s : s;
    x[i] = accumulate ? x[i] + v : v;
}

__global__ __launch_bounds__(kBlock) void gm_add_or_copy_kernel(int64_t n, const double *__restrict__ v,
                                                                double *__restrict__ x, int accumulate) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) x[i] = accumulate ? x[i] + v[i] : v[i];
}

__global__ __launch_bounds__(kBlock) void gm_true_resid_kernel(const double *part, int np, GmresState *st) {
    __shared__ double sh[kWaves];
    const double rr = reduce_partials(part, np, 1, sh);
    if (threadIdx.x == 0) st->true_resid = sqrt(rr);   // self.norm(resid)  :164
}

// LU with partial pivoting (LAPACK dgesv semantics) on a small dense column-major system.
static bool small_solve(int m, const double *Rcm, int ld, const double *rhs, std::vector<double> &y) {
    std::vector<double> a((size_t)m * m);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) a[(size_t)i * m + j] = Rcm[(size_t)j * ld + i];
    y.assign(rhs, rhs + m);
    std::vector<int> piv(m);
    for (int kk = 0; kk < m; ++kk) {
        int p = kk;
        double best = std::fabs(a[(size_t)kk * m + kk]);
        for (int i = kk + 1; i < m; ++i)
            if (std::fabs(a[(size_t)i * m + kk]) > best) {
                best = std::fabs(a[(size_t)i * m + kk]);
                p = i;
            }
        if (a[(size_t)p * m + kk] == 0.0) return false;
        if (p != kk) {
            for (int j = 0; j < m; ++j) std::swap(a[(size_t)p * m + j], a[(size_t)kk * m + j]);
            std::swap(y[p], y[kk]);
        }
        for (int i = kk + 1; i < m; ++i) {
            const double l = a[(size_t)i * m + kk] / a[(size_t)kk * m + kk];
            a[(size_t)i * m + kk] = l;
            for (int j = kk + 1; j < m; ++j) a[(size_t)i * m + j] -= l * a[(size_t)kk * m + j];
            y[i] -= l * y[kk];
        }
    }
    for (int i = m - 1; i >= 0; --i) {
        double s = y[i];
        for (int j = i + 1; j < m; ++j) s -= a[(size_t)i * m + j] * y[j];
        y[i] = s / a[(size_t)i * m + i];
    }
    return true;
}

static inline size_t aup(size_t v) { return (v + 255) / 256 * 256; }

}  // namespace psk

using namespace psk;

extern "C" int psk_gmres(const psk_csr *Ac, const psk_prec *M, const double *b, double *xout,
                         const psk_ctl *ctl, psk_result *res, double *hist, int32_t loc) {
    if (!Ac || !b || !xout || !ctl || !res) return fail(PSK_ERR_ARG, "psk_gmres: NULL argument");
    if (ctl->maxiter < 0 || ctl->restart < 0) return fail(PSK_ERR_ARG, "psk_gmres: negative maxiter/restart");
    if (M && M->n != Ac->n) return fail(PSK_ERR_ARG, "psk_gmres: preconditioner size mismatch");
    if (!Ac->comm && Ac->ncols != Ac->n) return fail(PSK_ERR_ARG, "psk_gmres: matrix must be square");
    psk_csr *A = const_cast<psk_csr *>(Ac);
    if (A->comm && A->comm->nranks > 1)
        return fail(PSK_ERR_UNSUPPORTED, "psk_gmres: sharded GMRES not built (replicas only)");
    Context *c;
    PSK_TRY(ctx(&c));
    std::lock_guard<std::mutex> solve_lock(c->solve_mu);
    hipStream_t s = c->stream;
    std::memset(res, 0, sizeof(*res));
    const int64_t n = A->n, maxiter = ctl->maxiter;
    int64_t K = ctl->restart > 0 ? ctl->restart : maxiter;
    if (K > maxiter) K = maxiter;
    if (K < 1) K = 1;
    const int ld = (int)(K + 1);
    const double *dinv = (M && M->kind == PSK_PREC_JACOBI) ? M->dinv : nullptr;
    const int gs = 1;   // partials of a dot-mode SpMV: it finishes its sum in-launch (gridsum)
    const int gv = grid_for_rows(c, n, kVecTile);
    const int64_t nv = n > 0 ? (n + kVecTile - 1) / kVecTile : 1;   // one-shot grid of the MGS kernels
    if (nv > INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "psk_gmres: vector too long for a one-shot grid");
    const size_t vec = aup((size_t)n * 8);
    const size_t qbytes = vec * (size_t)(K + 1);
    {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && qbytes + 4 * vec > fr)
            return fail(PSK_ERR_ALLOC, "psk_gmres: Krylov basis of " + std::to_string(K + 1) +
                                           " vectors does not fit in HBM; use restart");
    }
    // general (ILU) preconditioner: M^-1 q_k is materialised in w before the SpMV; t is scratch
    const bool gen = prec_is_general(M);
    PSK_TRY(A->ws.ensure(qbytes + (gen ? 5 : 3) * vec));
    char *wb = A->ws.as<char>();
    double *Q = reinterpret_cast<double *>(wb);
    double *u = reinterpret_cast<double *>(wb + qbytes);
    double *x = reinterpret_cast<double *>(wb + qbytes + vec);
    double *bv = reinterpret_cast<double *>(wb + qbytes + 2 * vec);
    double *w = gen ? reinterpret_cast<double *>(wb + qbytes + 3 * vec) : nullptr;
    double *tt = gen ? reinterpret_cast<double *>(wb + qbytes + 4 * vec) : nullptr;
    const size_t hb = aup((size_t)ld * K * 8);
    const size_t small = aup(sizeof(GmresState)) + 2 * hb + aup((size_t)2 * K * 8) + aup((size_t)ld * 8) +
                         aup((size_t)kMaxGrid * 8) + aup((size_t)(maxiter + 1) * 8) + aup((size_t)ld * 8) +
                         aup((size_t)(K + 2) * 8);
    PSK_TRY(A->ws_small.ensure(small));
    char *sb = A->ws_small.as<char>();
    GmresState *st = reinterpret_cast<GmresState *>(sb);
    sb += aup(sizeof(GmresState));
    double *H = reinterpret_cast<double *>(sb);
    sb += hb;
    double *R = reinterpret_cast<double *>(sb);
    sb += hb;
    double *CS = reinterpret_cast<double *>(sb);
    sb += aup((size_t)2 * K * 8);
    double *g = reinterpret_cast<double *>(sb);
    sb += aup((size_t)ld * 8);
    double *pa = reinterpret_cast<double *>(sb);   // partials of the cycle-start norm / the residual's sum
    sb += aup((size_t)kMaxGrid * 8);
    double *dhist = reinterpret_cast<double *>(sb);
    sb += aup((size_t)(maxiter + 1) * 8);
    double *dy = reinterpret_cast<double *>(sb);
    sb += aup((size_t)ld * 8);
    double *hv = reinterpret_cast<double *>(sb);   // K + 2 grid sums of a step (gm_mgs_kernel)

    // events and the poll words come from the device's SolveKit (allocated once, round 4)
    SolveKit *kit;
    PSK_TRY(solve_kit(c, false, &kit));
    hipEvent_t ev0 = kit->ev0, ev1 = kit->ev1;
    PSK_HIP(hipMemsetAsync(st, 0, sizeof(GmresState), s));
    // Hessenberg and rotated copies start at zero: entries below the subdiagonal are never written
    // and the least-squares solve reads them (HBar = np.zeros, GMRESSolver.py:80)
    PSK_HIP(hipMemsetAsync(H, 0, hb, s));
    PSK_HIP(hipMemsetAsync(R, 0, hb, s));
    PSK_TRY(to_device_vec(b, loc, n, bv, s));
    PSK_HIP(hipMemsetAsync(x, 0, (size_t)n * 8, s));
    PSK_HIP(hipEventRecord(ev0, s));

    const int L = 2, NS = kPollSlots;
    static_assert(kPollSlots >= L + 2, "poll slots");
    int32_t *hflag = reinterpret_cast<int32_t *>(static_cast<char *>(kit->hstage) + 1024);   // pinned, NS words
    hipEvent_t *fev = kit->fev;

    int rc = PSK_OK;
    int64_t it = 0;          // global iterations completed before this cycle
    bool first = true, finished = false, hit_maxiter = false;
    GmresState hs{};
    std::vector<double> hR, hg, y;
    int64_t spmv_count = 0;

    auto run_finalize = [&](int kc, bool accumulate) -> int {
        // y = solve(R[:kc+1,:kc+1], g[:kc+1]); x (+)= M^-1 Q y
        hR.resize((size_t)ld * K);
        hg.resize((size_t)ld);
        PSK_HIP(hipMemcpyAsync(hR.data(), R, (size_t)ld * K * 8, hipMemcpyDeviceToHost, s));
        PSK_HIP(hipMemcpyAsync(hg.data(), g, (size_t)ld * 8, hipMemcpyDeviceToHost, s));
        PSK_HIP(hipStreamSynchronize(s));
        if (!small_solve(kc + 1, hR.data(), ld, hg.data(), y))
            return fail(PSK_ERR_ARG, "GMRES least-squares system is singular (LinAlgError in the reference)");
        PSK_HIP(hipMemcpyAsync(dy, y.data(), (size_t)(kc + 1) * 8, hipMemcpyHostToDevice, s));
        const unsigned nb = (unsigned)((n + kBlock - 1) / kBlock);
        if (!gen) {
            hipLaunchKernelGGL(gm_update_x_kernel, dim3(nb), dim3(kBlock), 0, s, n, Q, (int64_t)(vec / 8), dy,
                               kc + 1, dinv, x, accumulate ? 1 : 0);
            PSK_HIP(hipGetLastError());
            return PSK_OK;
        }
        // x (+)= M^-1 (Q y): gemv into w, apply the preconditioner into tt, then add/copy
        hipLaunchKernelGGL(gm_update_x_kernel, dim3(nb), dim3(kBlock), 0, s, n, Q, (int64_t)(vec / 8), dy, kc + 1,
                           (const double *)nullptr, w, 0);
        PSK_HIP(hipGetLastError());
        PSK_TRY(prec_apply_dev(M, n, w, tt, s));
        hipLaunchKernelGGL(gm_add_or_copy_kernel, dim3(nb), dim3(kBlock), 0, s, n, tt, x, accumulate ? 1 : 0);
        PSK_HIP(hipGetLastError());
        return PSK_OK;
    };

    while (rc == PSK_OK && !finished) {
        // ---- cycle start: r0 = b (first cycle, :87) or b - A x (restart)
        if (first) {
            hipLaunchKernelGGL(gm_selfdot_kernel, dim3(gv), dim3(kBlock), 0, s, n, bv, pa);
            hipLaunchKernelGGL(gm_start_kernel, dim3(gv), dim3(kBlock), 0, s, n, bv, Q, pa, gv, g, ld, st,
                               ctl->tau, 1, ctl->norm_b);
        } else {
            if ((rc = launch_spmv(A, kSpmvResid, x, u, nullptr, bv, pa, nullptr, s)) != PSK_OK) break;
            ++spmv_count;
            hipLaunchKernelGGL(gm_start_kernel, dim3(gv), dim3(kBlock), 0, s, n, u, Q, pa, gs, g, ld, st,
                               ctl->tau, 0, 0.0);
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(PSK_ERR_HIP, "gmres start"); break; }
        if (first && n > 0) {
            if (hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "gmres state"); break; }
            if (hs.zero_b) {   // b = 0: handleConvergence(0, zeros, 0, 0)
                finished = true;
                break;
            }
        }
        if (n == 0) {
            hs.zero_b = 1;
            finished = true;
            break;
        }
        first = false;
        const int64_t Kc = (maxiter - it) < K ? (maxiter - it) : K;
        int64_t k = 0;
        for (; k < Kc; ++k) {
            if (k > 0) {   // poll with a lag of L steps
                const int slot = (int)((k - 1) % NS);
                if (hipMemcpyAsync(&hflag[slot], &st->done, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipEventRecord(fev[slot], s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "poll"); break; }
                if (k - 1 - L >= 0) {
                    const int os = (int)((k - 1 - L) % NS);
                    if (hipEventSynchronize(fev[os]) != hipSuccess) { rc = fail(PSK_ERR_HIP, "poll sync"); break; }
                    if (hflag[os]) break;
                }
            }
            const double *qk = Q + (size_t)k * (vec / 8);
            const double *q0 = Q;
            if (gen) {   // u = A (M^-1 q_k): materialise M^-1 q_k (GMRESSolver.py:107)
                if ((rc = prec_apply_dev(M, n, qk, w, s)) != PSK_OK) break;
                if ((rc = launch_spmv(A, kSpmvPlainDot, w, u, nullptr, q0, hv, &st->done, s)) != PSK_OK) break;
            } else if ((rc = launch_spmv(A, dinv ? kSpmvJacobiDot : kSpmvPlainDot, qk, u, dinv, q0, hv, &st->done,
                                         s)) != PSK_OK)
                break;
            ++spmv_count;
            // hv[0] = q_0.u (the SpMV's grid sum), hv[j+1] = the dot MGS step j finishes
            double *hcol = H + (size_t)k * ld;
            for (int64_t j = 0; j <= k; ++j) {
                const double *qj = Q + (size_t)j * (vec / 8);
                const double *qn = j < k ? Q + (size_t)(j + 1) * (vec / 8) : nullptr;
                GridSum gsj;
                if ((rc = gridsum_prepare(c, nv, 1, hv + j + 1, &gsj)) != PSK_OK) break;
                hipLaunchKernelGGL(gm_mgs_kernel, dim3((unsigned)nv), dim3(kBlock), 0, s, n, u, qj, qn, hv + j, hcol,
                                   (int)j, gsj, st);
            }
            if (rc != PSK_OK) break;
            hipLaunchKernelGGL(gm_normalize_kernel, dim3((unsigned)nv), dim3(kBlock), 0, s, n, u,
                               Q + (size_t)(k + 1) * (vec / 8), hv + k + 1, H, R, CS, g, ld, (int)k, it + k, st,
                               dhist);
            if (hipGetLastError() != hipSuccess) { rc = fail(PSK_ERR_HIP, "gmres step launch"); break; }
        }
        if (rc != PSK_OK) break;
        if (hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "gmres state"); break; }
        if (hs.done) {
            // converged at step kc: x = M^-1 Q y, true residual (:159-174)
            const int kc = hs.kconv;
            if ((rc = run_finalize(kc, it > 0)) != PSK_OK) break;
            if ((rc = launch_spmv(A, kSpmvResid, x, u, nullptr, bv, pa, nullptr, s)) != PSK_OK) break;
            ++spmv_count;
            hipLaunchKernelGGL(gm_true_resid_kernel, dim3(1), dim3(kBlock), 0, s, pa, gs, st);
            if (hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "gmres state"); break; }
            res->iters = it + kc + 1;
            res->exit = hs.brk ? PSK_EXIT_ARNOLDI_BREAKDOWN : PSK_EXIT_TOLERANCE;
            res->resid = hs.true_resid;
            res->resid_recursive = hs.rec;
            if (hs.true_resid <= hs.tauNormB) {
                res->status = PSK_CONVERGED;
                res->success = 1;
            } else {
                res->status = PSK_TRUE_RESID_FAIL;
                res->success = 0;
                std::snprintf(res->msg, sizeof(res->msg),
                              "GMRES failure: true residual %12.5g did not meet tolerance tau=%12.5g. "
                              "Recursive residual was %12.5g.",
                              hs.true_resid, ctl->tau, hs.rec);
            }
            finished = true;
        } else {
            it += Kc;
            if ((rc = run_finalize((int)Kc - 1, it - Kc > 0)) != PSK_OK) break;
            if (it >= maxiter) {
                // maxiter reached (reference: NameError at :180) -> handleMaxiter(k, x, |g|, ...)
                hit_maxiter = true;
                res->exit = PSK_EXIT_MAXITER;
                res->iters = maxiter > 0 ? maxiter - 1 : 0;
                res->resid = hs.rec;
                res->resid_recursive = hs.rec;
                if (ctl->fail_on_maxiter) {
                    res->status = PSK_MAXITER;
                    res->success = 0;
                    std::snprintf(res->msg, sizeof(res->msg), "failure to converge");
                } else {
                    res->status = PSK_CONVERGED;
                    res->success = 1;
                }
                finished = true;
            }
        }
    }
    if (rc == PSK_OK && hipEventRecord(ev1, s) != hipSuccess) rc = fail(PSK_ERR_HIP, "event");
    if (rc == PSK_OK && hipStreamSynchronize(s) != hipSuccess) rc = fail(PSK_ERR_HIP, "gmres sync");
    // an expired in-launch reduction wait (MGS / normalisation / SpMV dots) poisons h with NaN; report it
    // as the error it is rather than as a numerical non-convergence (and never to a later solve)
    if (rc == PSK_OK) rc = gridsum_check(c);
    if (rc == PSK_OK && gen) rc = prec_check_error(M, s);
    if (rc == PSK_OK) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ev0, ev1);
        res->loop_ms = ms;
        res->norm_b = hs.normB;
        res->spmv_launches = spmv_count;
        if (hs.zero_b) {
            res->status = PSK_CONVERGED;
            res->success = 1;
            res->iters = 1;
            res->resid = 0.0;
            res->exit = PSK_EXIT_NONE;
        }
        // every step reported one residual (reportIter, :155): iters + 1 entries at maxiter (k = maxiter - 1)
        const int64_t nh = res->iters + (hit_maxiter ? 1 : 0);
        const int64_t nhc = hs.zero_b ? 0 : (nh < maxiter ? nh : maxiter);
        res->hist_len = nhc;
        if (hist && nhc > 0 &&
            hipMemcpy(hist, dhist, (size_t)nhc * 8, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(PSK_ERR_HIP, "hist copy");
        if (rc == PSK_OK) rc = from_device_vec(x, loc, n, xout, s);
        if (rc == PSK_OK && hipStreamSynchronize(s) != hipSuccess) rc = fail(PSK_ERR_HIP, "x copy");
    }
    return rc;
}
