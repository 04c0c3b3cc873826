// pcg_state.hpp — the PCG solver state and the K3 scalar logic (PCGSolver.py:113-138), shared by pcg.hip
// (the loop, K0/K2/K3) and spmv.hip (the PCG init fused into the first SpMV of the diagonal layout).
#pragma once
#include "psk_internal.hpp"

namespace psk {

struct PcgState {
    int32_t done;      // 0 running, 1 converged, 2 breakdown
    int32_t brk_kind;  // 1: dot(u,r)==0 at start, 2: dot(p,Ap)==0
    int64_t iters;
    double resid;
    double normB;
    double tauNormB;
    int64_t live;      // k of the last K2 that ran to completion (no breakdown); -1 before the loop
    int64_t *hdone;    // host-mapped stamp of the iteration that set `done` (nullptr: none), see set_done
    int64_t hgen;      // this solve's generation in the stamp's high bits (kStampGenShift)
    double last_hist;  // the latest reported ||r_k|| (resid_recursive without copying the history back)
    int32_t x_written; // 1 once x has been stored (Jacobi/identity: x0 = 0 is implicit until the first flush)
    int32_t pad;
};

// done = v != 0, and the host-mapped stamp the solve loop polls: k + 2 for a kernel of iteration k, 1
// for the init (0 = running) — a system-scope store drained before the kernel ends, so once an event
// recorded after this kernel has completed the host reads the word directly, with no per-chunk
// device-to-host copy (a blit kernel) on the solver's stream. The stamp lets the host act on the state
// as of the chunk it waited for, not a later one its GPU has already run: every rank of a sharded
// solve then stops after the same chunk and enqueues the same collectives.
// The word is shared by every solve on the device; each solve tags its stamps with its own generation
// (high bits), so a kernel still queued from an earlier solve that failed on the host side cannot leave a
// stamp the next solve's poll would act on.
constexpr int kStampGenShift = 40;
constexpr int64_t kStampMask = ((int64_t)1 << kStampGenShift) - 1;
__device__ __forceinline__ void set_done(PcgState *st, int32_t v, int64_t stamp) {
    st->done = v;
    if (st->hdone) {
        __hip_atomic_store(st->hdone, st->hgen | stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
    }
}

// the solver state after the init sums bb = b.b and ur = u.r (PCGSolver.py:86-105)
__device__ __forceinline__ void pcg_init_state(double bb, double ur, double tau, PcgState *st, double *udr,
                                               int64_t *hdone, int64_t hgen, int32_t x_written) {
    const double normB = sqrt(bb);                 // self.norm(b)   :86
    st->normB = normB;
    st->tauNormB = tau * normB;
    st->iters = 0;
    st->resid = 0.0;
    st->brk_kind = 0;
    st->live = -1;
    st->hdone = hdone;
    st->hgen = hgen;
    st->last_hist = normB;
    st->x_written = x_written;
    udr[0] = ur;
    if (normB == 0.0) {                            // :87-88 handleConvergence(0, zeros, 0, 0)
        st->iters = 1;
        set_done(st, 1, 1);
    } else if (ur == 0.0) {                        // :104-105
        st->brk_kind = 1;
        st->iters = 0;
        set_done(st, 2, 1);
    } else {
        st->done = 0;
    }
}

// fused init finish: runs once, in thread 0 of the workgroup that completes the init's grid sums
struct PcgInitFin {
    double tau;
    PcgState *st;
    double *udr;
    int64_t *hdone;
    int64_t hgen;
    int32_t x_written;
    int32_t off;   // b.b and u.r are sums off, off + 1 of the launch (the diagonal layout's fused init: 1)
    __device__ void operator()(const double *r) const {
        pcg_init_state(r[off], r[off + 1], tau, st, udr, hdone, hgen, x_written);
    }
};

// Deferred x updates (Jacobi/identity K3): x is read and written every kPcgDefer-th iteration only.
// p_j lives in ring buffer j mod kPcgDefer; K3 of iteration k reads p_k and writes p_{k+1} over
// p_{k+1-kPcgDefer}, which the last flush consumed (or, on a flush, which this K3 reads first, element
// by element). A flush applies the pending updates in iteration order, x = ((x + a_{k-q} p_{k-q}) + ...)
// + a_k p_k, the reference's two roundings per update in its order (PCGSolver.py:121), so x is
// bit-identical to updating every iteration. x traffic per iteration: 16 B/row updated every
// iteration, 8 (kPcgDefer + 1) / kPcgDefer deferred (12 at 2, 10 at 4, 9 at 8). Round 5 A/B
// (profiles/r5_pcg_defer_ab.txt, same bits): 8 = 4 at N = 10M, +2.2% at 16384^2; 2 and 3 slower.
#ifndef PSK_PCG_DEFER
#define PSK_PCG_DEFER 8
#endif
constexpr int kPcgDefer = PSK_PCG_DEFER;
static_assert(kPcgDefer >= 1 && kPcgDefer <= 8, "kPcgDefer");
struct PRing {
    double *b[kPcgDefer];
};
// iterations whose x update is still pending when K3 of iteration k runs: k - q .. k - 1
__host__ __device__ inline int pcg_pending(int64_t k) { return (int)(k % kPcgDefer); }

// x[j] with the pending updates of iterations k - q .. k - 1 applied (ring: their p; alphas[i] = a_i)
__device__ __forceinline__ double pcg_catch_up(double xj, const PRing *pr, int q, int64_t k,
                                               const double *__restrict__ alphas, int64_t j) {
    for (int t = q; t >= 1; --t) xj = xj + alphas[k - t] * pr->b[(k - t) % kPcgDefer][j];   // :121
    return xj;
}

// K3 prologue shared by the Jacobi/identity and general-preconditioner variants: alpha again
// (K2's expression on the same partials), the convergence test, beta. Returns false when the
// solve stopped at this iteration; x (which K3 owns) is then still advanced over the tile.
// pr != nullptr: the q = pcg_pending(k) deferred x updates are applied first.
__device__ inline bool pcg_direction_scalars(int64_t n, double *__restrict__ x, const double *__restrict__ p,
                                             double pTAp, double rr, double ur, double udk, double tauNB,
                                             PcgState *st, double *__restrict__ udr, double *__restrict__ hist, int64_t k,
                                             int64_t maxiter, int fail_on_maxiter, double &alpha, double &beta,
                                             int64_t tile, const PRing *pr = nullptr,
                                             const double *__restrict__ alphas = nullptr) {
    alpha = udk / pTAp;                                      // :118 (udk = udr[k])
    const double normR = sqrt(rr);                           // self.norm(r)  :125
    if (tile == 0 && threadIdx.x == 0) {
        hist[k] = normR;                                     // reportIter  :126
        st->last_hist = normR;
    }
    if (normR <= tauNB || (!fail_on_maxiter && k == maxiter - 1)) {   // :129-131 (tauNB = st->tauNormB)
        const int64_t i = tile * kVecTile + 2 * threadIdx.x;
        // deferred updates (pr): before the first flush (k < kPcgDefer) x is still the implicit x0 = 0
        const bool x0 = pr && k < kPcgDefer;
        for (int64_t j = i; j < i + 2 && j < n; ++j) {
            double xj = x0 ? 0.0 : x[j];
            if (pr) xj = pcg_catch_up(xj, pr, pcg_pending(k), k, alphas, j);
            x[j] = xj + alpha * p[j];                        // :121
        }
        if (tile == 0 && threadIdx.x == 0) {
            st->iters = k + 1;                               // handleConvergence(k, ...)
            st->resid = normR;
            st->x_written = 1;
            set_done(st, 1, k + 2);
        }
        return false;
    }
    beta = ur / udk;                                         // :134-135
    if (tile == 0 && threadIdx.x == 0) udr[k + 1] = ur;   // :136
    return true;
}

// the PCG init fused into the first SpMV (spmv.hip, pcg_init_diag_kernel): the diagonal layout in the
// 5-diagonal DPP order, unsharded; xs = the one DInv value (Jacobi) or 1.0 (none). [p_0.Ap_0, b.b, u.r] into
// out3[0..2], p_0 into p, Ap_0 into Ap; fin runs on sums 1 and 2 (fin.off = 1)
bool pcg_init_diag_eligible(const psk_csr *A);
int launch_pcg_init_diag(const psk_csr *A, const double *b, double xs, double *p, double *Ap, double *out3,
                         const PcgInitFin &fin, hipStream_t s);

}  // namespace psk
