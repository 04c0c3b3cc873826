// pcg.hip — device-resident preconditioned CG (PCGSolver.solve, PCGSolver.py:64-142).
//
// Per iteration k three launches, no host synchronisation:
//   K1  Ap = A p  and p.Ap                                         (spmv.hip, kSpmvDot)   :111,:113
//   K2  alpha = uDotR/pTAp; r -= alpha Ap; u = M^-1 r; r.r and u.r   :114-125,:134
//   K3  x += alpha p (alpha recomputed from K1's sum); ||r|| test (tau*||b||, or
//       k==maxiter-1 when !failOnMaxiter); beta; p = u + beta p       :121,:125-138
// x is updated in K3 rather than K2 because K3 streams p anyway: that saves one read of p (8n
// bytes per iteration). x depends on nothing else in the iteration, so the order is invisible.
// All three are one-shot launches (one tile per workgroup); K1 and K2 finish their dot products in
// the same launch with a fixed reduction order (gridsum, psk_internal.hpp), so every workgroup
// (and every rank, after the RCCL sum) reads bit-identical scalars and takes identical branches; the
// control state (done flag, iteration count, residual) lives in HBM and the host only polls it
// every `check_every` iterations with a lag, keeping the launch queue full.
// u is never stored: K2 and K3 both recompute u_i = DInv_i * r_i (one rounding, as np.multiply).
// Elementwise updates use two roundings (-ffp-contract=off), exactly as numpy's x + alpha*p.
#include "psk_internal.hpp"
#include "pcg_state.hpp"

#include <cstdlib>

#include <climits>
#include <cmath>
#include <cstdio>


namespace psk {

// ---- K0 (Jacobi/identity): p_0 = M b; [b.b, u.r] --------------------------------------------
// One-shot, the two sums finished in the same launch by gridsum and, unsharded, the solver state set by the
// wave that completes them (PcgInitFin; a sharded solve gathers the per-rank sums and runs
// pcg_init_finish_kernel). x0 = 0 is not stored: K3's first flush of the deferred x updates starts from the
// literal 0.0 (x = np.zeros_like(b) :100, then x + alpha*p :121: the same roundings). r = np.copy(b) (:97) is
// not stored either (round 5): K2 of iteration 0 reads b where it would read r, and writes r. 16 B/row.
// Round 5: the sums run over the SpMV's 256-row gridsum tiles with one row per lane (two tiles per
// workgroup) and the SpMV's tile epilogue (per-row products, wave totals in wave order): the diagonal
// layout's init fused into the first SpMV (spmv.hip pcg_init_diag_kernel) then has the same bits.
template <int JAC, bool FUSED>
__global__ __launch_bounds__(kBlock) void pcg_init_kernel(int64_t n, const double *__restrict__ b,
                                                          const double *__restrict__ dinv, double ds,
                                                          double *__restrict__ p, GridSum gs, PcgInitFin fin,
                                                          int64_t ntiles) {
    constexpr int TPW = 2;
    const int tid = threadIdx.x;
    int64_t tl[TPW];
    bool tv[TPW];
    double acc[TPW][2];
    uint32_t ticket[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        const int64_t t = (int64_t)blockIdx.x * TPW + q;
        tv[q] = t < ntiles;
        tl[q] = tv[q] ? t : ntiles - 1;
        const int64_t row = tl[q] * kBlock + tid;
        const bool has = tv[q] && row < n;
        const double bi = has ? __builtin_nontemporal_load(b + row) : 0.0;
        const double d = JAC == 1 ? (has ? dinv[row] : 0.0) : ds;
        const double u = JAC ? d * bi : bi;                     // p = precond.applyRight(r)  :98
        if (has) p[row] = u;                                    // (r = np.copy(b) :97 is read from b by K2)
        acc[q][0] = has ? bi * bi : 0.0;                        // self.norm(b)  :86
        acc[q][1] = has ? u * bi : 0.0;                         // uDotR = np.dot(u, r)  :102
    }
    __shared__ GridSumTile<2> gsl[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
        ticket[q] = 0;
        if (tv[q] && gs.grp_log2 >= 0 && tid == 0)
            ticket[q] = gridsum_draw(gridsum_counter(gs, gridsum_group_of(tl[q], gs.grp_log2)));
    }
    if (tid < TPW) gsl[tid].cnt = 0;
    if (tid == 0 && blockIdx.x == 0 && (gs.nt + TPW - 1) / TPW != gridDim.x) atomicOr(gs.err, 2);
    __syncthreads();
    if (FUSED)
        gridsum_tiles_publish<TPW, 2>(gs, gsl, acc, ticket, tl, tv, fin);
    else
        gridsum_tiles_publish<TPW, 2>(gs, gsl, acc, ticket, tl, tv);
}

// sharded init: the per-rank sums all-gathered, added in rank order (bit-identical on every rank)
__global__ void pcg_init_finish_kernel(const double *g, int P, double tau, PcgState *st, double *udr,
                                       int64_t *hdone, int64_t hgen) {
    if (threadIdx.x == 0) pcg_init_state(rank_sum(g, P, 2, 0), rank_sum(g, P, 2, 1), tau, st, udr, hdone, hgen, 0);
}

// ---- K2: r update + grid sums [r.r, u.r] -------------------------------------------------
// One-shot: workgroup b owns elements [512b, 512b+512), two per lane (16-B accesses). Round 6 measured three other
// forms of its grid sums, none better at both N = 10M and 16384^2 (profiles/r6_k2_wave_ab.txt,
// r6_k2_gridmask_ab.txt): one tile per WAVE with the workgroup's bits (-1 to -2%), one tile per wave with DPP wave
// totals (+1% / -2%), DPP wave totals combined in LDS instead of block_sum (+-0). JAC: Jacobi
// preconditioner fused: 1 = DInv streamed, 2 = every DInv entry the same double `ds` (constant-
// diagonal matrices such as stencils: the same products, 8 B/row less per kernel).
// FIRST (iteration 0): r_0 = b is read from b (the init does not copy it, K0 above).
template <int JAC, bool FIRST>
__global__ __launch_bounds__(kBlock) void pcg_update_kernel(
    int64_t n, double *__restrict__ r, const double *__restrict__ b, const double *__restrict__ Ap,
    const double *__restrict__ dinv, double ds, const double *__restrict__ pap, int nparts, GridSum gs, PcgState *st,
    const double *__restrict__ udr, int64_t k, TileMap tm) {
    // the done flag, p.Ap and udr[k] loaded together (one scalar round trip, not three in a chain): every
    // address is valid whatever the flag says, and the asm keeps the loads above the branch (round 6: +0.5-1.8%
    // PCG it/s at N = 10M, profiles/r6_prologue_ab.txt)
    const double udk = udr[k];
    const int32_t dn = st->done;
    const double pap0 = pap[0];
    __asm__ volatile("" ::"s"(dn), "s"(pap0), "s"(udk));
    if (dn) return;
    double pTAp = pap0;                                      // np.dot(p, Ap)  :113 (K1's grid sum; rank_sum)
    for (int q = 1; q < nparts; ++q) pTAp += pap[q];
    __shared__ double sh[2 * kWaves];
    if (pTAp == 0.0) {                                       // :114-115 handleBreakdown(k, ...)
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->brk_kind = 2;
            st->iters = k;
            set_done(st, 2, k + 2);
        }
        return;
    }
    const double alpha = udk / pTAp;                         // :118
    // K3 (x update) runs iff this K2 did: it tests `live`, written by the previous kernel, never its
    // own done flag, which its first workgroup may set while later ones are still starting
    if (blockIdx.x == 0 && threadIdx.x == 0) st->live = k;
    // tile of this workgroup: XCD-banded like the SpMV's (tm), so the Ap rows a tile reads were
    // written through the same XCD's L2; the grid sums are published by tile (order-independent)
    const int64_t tile = tile_of_block(tm);
    const int64_t i = tile * kVecTile + 2 * threadIdx.x;
    const bool pair = i + 1 < n;
    uint32_t ticket = 0;   // gridsum ticket, drawn by thread 0 once its loads are issued
    double rr = 0.0, ur = 0.0;
    if (pair) {
        // (issued after the done test: issued before it, K2 measured 1-5% slower, profiles/r6_k2_early_sum2_ab.txt)
        const dv2 ro = FIRST ? ld2nt(b + i) : ld2(r + i), a = ld2nt(Ap + i);
        dv2 d{ds, ds};
        if (JAC == 1) d = ld2(dinv + i);
        ticket = gridsum_ticket(gs, tile);
        dv2 rn;
        rn.x = ro.x - alpha * a.x;                           // r = r - alpha*Ap  :122
        rn.y = ro.y - alpha * a.y;
        double u0 = rn.x, u1 = rn.y;
        if (JAC) {
            u0 = d.x * rn.x;                                 // u = precond.applyRight(r)  :123
            u1 = d.y * rn.y;
        }
        st2(r + i, rn);
        rr = fma(rn.x, rn.x, rr);
        rr = fma(rn.y, rn.y, rr);
        ur = fma(u0, rn.x, ur);
        ur = fma(u1, rn.y, ur);
    } else if (i < n) {   // odd tail element
        ticket = gridsum_ticket(gs, tile);
        const double rn = (FIRST ? b[i] : r[i]) - alpha * Ap[i];
        const double u0 = JAC == 2 ? ds * rn : JAC ? dinv[i] * rn : rn;
        r[i] = rn;
        rr = rn * rn;
        ur = u0 * rn;
    }
    block_sum2(rr, ur, sh);   // both sums in one barrier pair (same bits as two block_sums; round 6: +0.3%)
    const double v[2] = {rr, ur};
    // wave 0 alone publishes the tile and, holding its group's last ticket, reduces the group and takes part in the
    // final stage in the wave forms (gridsum_take<2, 64>, gridsum_final_wave): no barrier after the totals (round 6:
    // +0.3-0.7% PCG it/s at N = 10M, profiles/r6_k2_wpub_ab.txt; the group and final sums run in the wave order)
    if (threadIdx.x >= 64) return;
    const bool lane0 = threadIdx.x == 0;
    if (gs.grp_log2 < 0) {
        if (lane0) {
            gridsum_put(gs.gslots + tile * 2, v[0]);
            gridsum_put(gs.gslots + tile * 2 + 1, v[1]);
        }
        gridsum_final_wave<2>(gs);
        return;
    }
    if (lane0) {
        gridsum_put(gs.slots + gridsum_slot(gs, tile) * 2, v[0]);
        gridsum_put(gs.slots + gridsum_slot(gs, tile) * 2 + 1, v[1]);
    }
    const uint32_t tk = __builtin_amdgcn_readfirstlane(ticket);
    const int64_t g = gridsum_group_of(tile, gs.grp_log2);
    int64_t base;
    const int64_t cnt = gridsum_members(gs, g, base);
    if (tk != (uint32_t)(cnt - 1)) return;
    double gr[2];
    gridsum_take<2, 64>(gs.slots, g << gs.grp_log2, cnt, gs.err, nullptr, gr);
    if (lane0) {
        gridsum_reset(gridsum_counter(gs, g));
        gridsum_put(gs.gslots + g * 2, gr[0]);
        gridsum_put(gs.gslots + g * 2 + 1, gr[1]);
    }
    gridsum_final_wave<2>(gs);
}

// ---- K3: x += alpha p (deferred, above), convergence test, beta, p = u + beta p (one-shot, as K2) --
// A breakdown leaves the updates of the iterations since the last flush pending (pcg_flush_kernel).
template <int JAC>
__global__ __launch_bounds__(kBlock) void pcg_direction_kernel(
    int64_t n, double *__restrict__ x, const double *__restrict__ r, PRing pr, const double *__restrict__ dinv,
    double ds, const double *__restrict__ pap, const double *__restrict__ rrur, int nparts, PcgState *st,
    double *__restrict__ udr, double *__restrict__ hist, double *__restrict__ alphas, int64_t k, int64_t maxiter,
    int fail_on_maxiter, int64_t tile_base, TileMap tm) {
    // every solver scalar loaded together with the live flag (one scalar round trip; see K2)
    const double udk = udr[k];
    const int64_t live = st->live;
    const double tauNB = st->tauNormB, pap0 = pap[0], rr0 = rrur[0], ur0 = rrur[1];
    __asm__ volatile("" ::"s"(live), "s"(pap0), "s"(rr0), "s"(ur0), "s"(udk), "s"(tauNB));
    if (live != k) return;   // K2 returned (stopped earlier, or breakdown at :114)
    double pTAp = pap0, rr = rr0, ur = ur0;   // rank_sum's order
    for (int q = 1; q < nparts; ++q) {
        pTAp += pap[q];
        rr += rrur[2 * q];
        ur += rrur[2 * q + 1];
    }
    // tile_base: a sharded solve launches the tiles holding the rows its neighbours need first (the
    // halo exchange then overlaps the rest); tile 0 alone writes the solver state. tm: XCD bands
    // over the launch's tiles (see K2)
    const int64_t tile = tile_base + tile_of_block(tm);
    const double *pcur = pr.b[k % kPcgDefer];
    // NOT __restrict__: on a flush iteration pnext is p_{k+1-kPcgDefer}'s buffer, which the x catch-up
    // below reads through pr.b first; the store to pnext must stay after those loads
    double *pnext = pr.b[(k + 1) % kPcgDefer];
    const int q = pcg_pending(k);
    double alpha, beta;
    if (!pcg_direction_scalars(n, x, pcur, pTAp, rr, ur, udk, tauNB, st, udr, hist, k, maxiter, fail_on_maxiter,
                               alpha, beta, tile, &pr, alphas))
        return;
    const bool flush = q == kPcgDefer - 1 || k == maxiter - 1;
    const bool x0 = k < kPcgDefer;   // no flush yet: x is the implicit x0 = 0 (never loaded)
    if (tile == 0 && threadIdx.x == 0) {
        alphas[k] = alpha;
        if (flush) st->x_written = 1;
    }
    const int64_t i = tile * kVecTile + 2 * threadIdx.x;
    // r, dinv and x are not needed again this iteration (non-temporal); p is gathered by the next SpMV
    if (i + 1 < n) {
        const dv2 ro = ld2nt(r + i), po = ld2(pcur + i);
        dv2 d{ds, ds};
        if (JAC == 1) d = ld2nt(dinv + i);
        double u0 = ro.x, u1 = ro.y;
        if (JAC) {
            u0 = d.x * ro.x;
            u1 = d.y * ro.y;
        }
        if (flush) {
            dv2 xo{0.0, 0.0};
            if (!x0) xo = ld2nt(x + i);
            dv2 pp[kPcgDefer > 1 ? kPcgDefer - 1 : 1];
#pragma unroll
            for (int t = 1; t < kPcgDefer; ++t)
                if (t <= q) pp[t - 1] = ld2nt(pr.b[(k - t) % kPcgDefer] + i);
#pragma unroll
            for (int t = kPcgDefer - 1; t >= 1; --t)
                if (t <= q) {
                    const double a = alphas[k - t];
                    xo.x = xo.x + a * pp[t - 1].x;           // x = x + alpha*p  :121 (iteration k-t)
                    xo.y = xo.y + a * pp[t - 1].y;
                }
            dv2 xn;
            xn.x = xo.x + alpha * po.x;                      // :121
            xn.y = xo.y + alpha * po.y;
            st2nt(x + i, xn);
        }
        dv2 pn;
        pn.x = u0 + beta * po.x;                             // p = u + beta*p  :138
        pn.y = u1 + beta * po.y;
        st2(pnext + i, pn);   // (non-temporal and write-through p stores measured no faster, round 4)
    } else if (i < n) {
        const double u0 = JAC == 2 ? ds * r[i] : JAC ? dinv[i] * r[i] : r[i];
        const double pi = pcur[i];
        if (flush) x[i] = pcg_catch_up(x0 ? 0.0 : x[i], &pr, q, k, alphas, i) + alpha * pi;
        pnext[i] = u0 + beta * pi;
    }
}

// the x updates a breakdown at iteration k left pending: iterations k - q .. k - 1, q = pcg_pending(k)
__global__ void pcg_flush_kernel(int64_t n, double *__restrict__ x, PRing pr, const double *__restrict__ alphas,
                                 int64_t k) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) x[i] = pcg_catch_up(k < kPcgDefer ? 0.0 : x[i], &pr, pcg_pending(k), k, alphas, i);
}

// ---- end of a solve: the state, the scan of the gridsum ticket counters (gridsum_counter_check_kernel's)
// and the gridsum error word into the host-mapped words at kit->hmap + kPcgFinishWord (system scope)
constexpr int kPcgStateWords = (int)(sizeof(PcgState) / 8);
constexpr int kPcgFinishWord = 8;
static_assert(sizeof(PcgState) % 8 == 0 && kPcgFinishWord + kPcgStateWords + 1 <= 64, "SolveKit::hmap words");
__global__ __launch_bounds__(kBlock) void pcg_finish_kernel(const PcgState *st, const uint32_t *cnt, const int32_t *err,
                                                            int64_t *hw) {
    // every counter (kGridSumMaxGroups + 1) loaded at once, unconditionally (indices clamped): one memory
    // round trip instead of a dependent chain of nine
    constexpr int kPer = (kGridSumMaxGroups + kBlock) / kBlock;
    uint32_t v[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int g = (int)threadIdx.x + i * kBlock;
        v[i] = cnt[(int64_t)(g < kGridSumMaxGroups ? g : kGridSumMaxGroups) * kGridSumCntStride];
    }
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) any |= v[i];
    const bool bad = __syncthreads_or(any != 0);
    if (threadIdx.x < kPcgStateWords)
        __hip_atomic_store(hw + threadIdx.x, reinterpret_cast<const int64_t *>(st)[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 0)
        __hip_atomic_store(hw + kPcgStateWords, (int64_t)(*err | (bad ? 4 : 0)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- general preconditioner (ILU, ...): u = M^-1 r is materialised by the preconditioner's own
// kernels between K2 and K3, so u.r gets its own reduction and K3 reads u ----------------------
__global__ __launch_bounds__(kBlock) void pcg_gen_init_kernel(int64_t n, const double *__restrict__ b,
                                                              double *__restrict__ x, double *__restrict__ r) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        r[i] = b[i];   // r = np.copy(b)        :97
        x[i] = 0.0;    // x = np.zeros_like(b)  :100
    }
}

// p = u (copy of M^-1 r, :98-99); [b.b, u.r] finished in-launch and the state set (one-shot, as K0)
__global__ __launch_bounds__(kBlock) void pcg_gen_init2_kernel(int64_t n, const double *__restrict__ r,
                                                               const double *__restrict__ u, double *__restrict__ p,
                                                               GridSum gs, PcgInitFin fin) {
    __shared__ double sh[kWaves];
    const int64_t i = (int64_t)blockIdx.x * kVecTile + 2 * threadIdx.x;
    const uint32_t ticket = gridsum_ticket(gs);
    double bb = 0.0, ur = 0.0;
    for (int64_t j = i; j < i + 2 && j < n; ++j) {
        const double rj = r[j], uj = u[j];
        p[j] = uj;
        bb = fma(rj, rj, bb);
        ur = fma(uj, rj, ur);
    }
    const double v[2] = {block_sum(bb, sh), block_sum(ur, sh)};
    gridsum_publish<2>(gs, v, sh, ticket, fin);
}

__global__ __launch_bounds__(kBlock) void pcg_dot_kernel(int64_t n, const double *__restrict__ a,
                                                         const double *__restrict__ c, GridSum gs,
                                                         const PcgState *st) {
    if (st->done) return;
    __shared__ double sh[kWaves];
    const int64_t i = (int64_t)blockIdx.x * kVecTile + threadIdx.x;
    const uint32_t ticket = gridsum_ticket(gs);
    double acc = 0.0;
    if (i < n) acc = a[i] * c[i];                                               // np.dot(u, r) :134
    if (i + kBlock < n) acc = fma(a[i + kBlock], c[i + kBlock], acc);
    const double v = block_sum(acc, sh);
    gridsum_publish<1>(gs, &v, sh, ticket);
}

__global__ __launch_bounds__(kBlock) void pcg_gen_direction_kernel(
    int64_t n, double *__restrict__ x, const double *__restrict__ u, double *__restrict__ p,
    const double *__restrict__ pap, const double *__restrict__ rrur, const double *__restrict__ ur_gen, PcgState *st,
    double *__restrict__ udr, double *__restrict__ hist, int64_t k, int64_t maxiter, int fail_on_maxiter) {
    if (st->live != k) return;
    double alpha, beta;
    if (!pcg_direction_scalars(n, x, p, *pap, rrur[0], *ur_gen, udr[k], st->tauNormB, st, udr, hist, k, maxiter,
                               fail_on_maxiter, alpha, beta, blockIdx.x))
        return;
    const int64_t i = (int64_t)blockIdx.x * kVecTile + 2 * threadIdx.x;
    for (int64_t j = i; j < i + 2 && j < n; ++j) {
        const double pj = p[j];
        x[j] = x[j] + alpha * pj;                            // :121
        p[j] = u[j] + beta * pj;                             // :138
    }
}

// -------------------------------------------------------------------------------------------------
// host driver

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

struct PcgWork {
    double *x, *r, *p, *Ap, *u, *part1, *part2, *part3, *udr, *hist;
    PRing pr;              // Jacobi/identity K3: p_j in pr.b[j % kPcgDefer] (pr.b[0] = p)
    double *alphas;        // alpha_k (deferred x updates)
    double *pinit;         // the init's two grid sums [b.b, u.r] (this rank's, sharded)
    // sharded (P ranks): the ranks' gathered scalars, [P] p.Ap, [P][2] (r.r, u.r) and [P][2] init sums;
    // unsharded: part1g/part2g alias part1/part2
    double *part1g, *part2g, *initg;
    PcgState *st;
};

static int pcg_workspace(psk_csr *A, int64_t maxiter, bool gen, bool own_x, int P, PcgWork &w) {
    const size_t vec = align_up((size_t)A->n * 8, 256), vecc = align_up((size_t)A->ncols * 8, 256);
    // x lives in the caller's device vector when the solve writes there directly (own_x false)
    const size_t nx = own_x ? 1 : 0;
    const size_t big = (2 + nx + (gen ? 1 : 0)) * vec + (gen ? 1 : kPcgDefer) * vecc;
    PSK_TRY(A->ws.ensure(big > 0 ? big : 256));
    char *b = A->ws.as<char>();
    w.r = reinterpret_cast<double *>(b);
    w.Ap = reinterpret_cast<double *>(b + vec);
    w.x = own_x ? reinterpret_cast<double *>(b + 2 * vec) : nullptr;
    char *pb = b + (2 + nx) * vec;
    w.p = reinterpret_cast<double *>(pb);
    w.u = gen ? reinterpret_cast<double *>(pb + vecc) : nullptr;
    for (int t = 0; t < kPcgDefer; ++t)
        w.pr.b[t] = gen ? (t == 0 ? w.p : nullptr) : reinterpret_cast<double *>(pb + t * vecc);
    const size_t small = align_up(sizeof(PcgState), 256) + 2 * align_up(kMaxGrid * 8, 256) +
                         align_up(2 * kMaxGrid * 8, 256) + align_up((size_t)(maxiter + 2) * 8, 256) +
                         align_up((size_t)(maxiter + 1) * 8, 256) + align_up((size_t)(maxiter + 1) * 8, 256) + 256;
    const size_t gath = P > 1 ? align_up((size_t)P * 8, 256) + 2 * align_up((size_t)P * 16, 256) : 0;
    PSK_TRY(A->ws_small.ensure(small + gath));
    char *s = A->ws_small.as<char>();
    w.st = reinterpret_cast<PcgState *>(s);
    s += align_up(sizeof(PcgState), 256);
    w.part1 = reinterpret_cast<double *>(s);
    s += align_up(kMaxGrid * 8, 256);
    w.part3 = reinterpret_cast<double *>(s);
    s += align_up(kMaxGrid * 8, 256);
    w.part2 = reinterpret_cast<double *>(s);
    s += align_up(2 * kMaxGrid * 8, 256);
    w.udr = reinterpret_cast<double *>(s);
    s += align_up((size_t)(maxiter + 2) * 8, 256);
    w.hist = reinterpret_cast<double *>(s);
    s += align_up((size_t)(maxiter + 1) * 8, 256);
    w.alphas = reinterpret_cast<double *>(s);
    s += align_up((size_t)(maxiter + 1) * 8, 256);
    w.pinit = reinterpret_cast<double *>(s);
    s += 256;
    if (P > 1) {
        w.part1g = reinterpret_cast<double *>(s);
        s += align_up((size_t)P * 8, 256);
        w.part2g = reinterpret_cast<double *>(s);
        s += align_up((size_t)P * 16, 256);
        w.initg = reinterpret_cast<double *>(s);
    } else {
        w.part1g = w.part1;
        w.part2g = w.part2;
        w.initg = w.pinit;
    }
    return PSK_OK;
}

static void set_msg(psk_result *res, const char *m) {
    std::snprintf(res->msg, sizeof(res->msg), "%s", m);
}

}  // namespace psk

using namespace psk;

// Per-call cost (round 4): the host-mapped poll word, the staging buffer and every
// event come from the device's SolveKit (allocated once); the init's sums and the solver state are
// finished inside the init launch; a device-resident b is read in place and a device-resident x is
// written in place (no staging copies); the history is copied back only when the caller asks for it;
// the state, the gridsum error word and the end event share ONE stream synchronisation.
extern "C" int psk_pcg(const psk_csr *Ac, const psk_prec *M, const double *b, double *xout,
                       const psk_ctl *ctl, psk_result *res, double *hist, int32_t loc) {
    if (!Ac || !b || !xout || !ctl || !res) return fail(PSK_ERR_ARG, "psk_pcg: NULL argument");
    if (ctl->maxiter < 0) return fail(PSK_ERR_ARG, "psk_pcg: maxiter < 0");
    if (M && M->n != Ac->n) return fail(PSK_ERR_ARG, "psk_pcg: preconditioner size mismatch");
    if (!Ac->comm && Ac->ncols != Ac->n) return fail(PSK_ERR_ARG, "psk_pcg: matrix must be square");
    psk_csr *A = const_cast<psk_csr *>(Ac);
    Context *c;
    PSK_TRY(ctx(&c));
    std::lock_guard<std::mutex> solve_lock(c->solve_mu);
    hipStream_t s = c->stream;
    std::memset(res, 0, sizeof(*res));
    const int64_t n = A->n, maxiter = ctl->maxiter;
    // general preconditioner (ILU): u = M^-1 r materialised between K2 and K3
    const bool gen = prec_is_general(M);
    if (gen && A->comm) return fail(PSK_ERR_UNSUPPORTED, "psk_pcg: ILU preconditioning of a sharded matrix");
    // sharded: P ranks, scalars gathered (not all-reduced) and summed in rank order on every rank
    const bool sharded = A->comm != nullptr;
    const int P = sharded ? A->comm->nranks : 1;
    const bool dev_io = loc == PSK_DEVICE;
    PcgWork w;
    PSK_TRY(pcg_workspace(A, maxiter, gen, !dev_io, P, w));
    if (dev_io) w.x = xout;   // b and x in HBM: read b in place, write x in place
    SolveKit *kit;
    PSK_TRY(solve_kit(c, ctl->time_kernels > 0, &kit));
    const double *dinv = (M && M->kind == PSK_PREC_JACOBI) ? M->dinv : nullptr;
    const int jac = !dinv ? 0 : M->dinv_uniform ? 2 : 1;
    const double ds = jac == 2 ? M->dinv_value : 0.0;
    // one-shot grid of K0/K2/K3 (one 512-element tile per workgroup); K0/K1/K2 finish their dot products
    // in-launch (gridsum), so the loop's scalars are part1[0] = p.Ap and part2[0..1] = (r.r, u.r)
    const int64_t nv = n > 0 ? (n + kVecTile - 1) / kVecTile : 1;
    if (nv > INT32_MAX) return fail(PSK_ERR_UNSUPPORTED, "psk_pcg: vector too long for a one-shot grid");
    // the init: unsharded with the diagonal layout (5 diagonals, one DInv value or none) fused into the first
    // SpMV (spmv.hip pcg_init_diag_kernel, [p.Ap, b.b, u.r] into part1); otherwise pcg_init_kernel over the
    // SpMV's 256-row tiles (the same bits for b.b and u.r), or the general path's init over 512-element tiles
    const bool init_diag = !gen && !sharded && (jac == 0 || jac == 2) && pcg_init_diag_eligible(A);
    const int64_t nsl = n > 0 ? (n + kBlock - 1) / kBlock : 1;
    GridSum gs0, gs2, gs3;
    if (!init_diag) PSK_TRY(gridsum_prepare(c, gen ? nv : nsl, 2, w.pinit, &gs0));
    PSK_TRY(gridsum_prepare(c, nv, 2, w.part2, &gs2));
    PSK_TRY(gridsum_prepare(c, nv, 1, w.part3, &gs3));
    // the host-mapped done stamp the kernels write (set_done); no kernel of an earlier solve is running
    volatile int64_t *hdone = kit->hmap;
    const int64_t hgen = (int64_t)(++kit->solve_gen & 0x7FFFFF) << kStampGenShift;
    *hdone = 0;
    const PcgInitFin fin{ctl->tau, w.st, w.udr, const_cast<int64_t *>(hdone), hgen, gen ? 1 : 0, 0};
    const double *bd = b;
    if (!dev_io) {   // host b staged in r (r_0 = b already: K2 of iteration 0 then reads r as usual), or, on
                     // the general path, in Ap (unused until the first SpMV; its init copies r = b)
        PSK_TRY(to_device_vec(b, loc, n, gen ? w.Ap : w.r, s));
        bd = gen ? w.Ap : w.r;
    }
    // sharded with a mailbox (psk_comm_mailbox): the ranks' scalars go kernel -> mailbox -> gather kernel
    // instead of ncclAllGather; same gathered arrays, same rank-order sums
    psk_comm *mbc = sharded && A->comm->mb ? A->comm : nullptr;
    uint64_t seq0 = 0;
    if (mbc) seq0 = mbox_next(mbc, &gs0);
    PSK_HIP(hipEventRecord(kit->ev0, s));
    const dim3 gk((unsigned)nv);
    if (gen) {
        const unsigned nb = (unsigned)((n + kBlock - 1) / kBlock);
        if (n > 0) hipLaunchKernelGGL(pcg_gen_init_kernel, dim3(nb), dim3(kBlock), 0, s, n, bd, w.x, w.r);
        PSK_TRY(prec_apply_dev(M, n, w.r, w.u, s));                   // p = precond.applyRight(r)  :98
        hipLaunchKernelGGL(pcg_gen_init2_kernel, gk, dim3(kBlock), 0, s, n, w.r, w.u, w.p, gs0, fin);
    } else if (init_diag) {
        PcgInitFin fin3 = fin;
        fin3.off = 1;
        PSK_TRY(launch_pcg_init_diag(A, bd, jac == 2 ? ds : 1.0, w.p, w.Ap, w.part1, fin3, s));
    } else {
        const dim3 gi((unsigned)((nsl + 1) / 2));
#define PSK_PCG_INIT(J, F) \
        hipLaunchKernelGGL((pcg_init_kernel<J, F>), gi, dim3(kBlock), 0, s, n, bd, dinv, ds, w.p, gs0, fin, nsl)
        if (jac == 2) { if (sharded) PSK_PCG_INIT(2, false); else PSK_PCG_INIT(2, true); }
        else if (jac == 1) { if (sharded) PSK_PCG_INIT(1, false); else PSK_PCG_INIT(1, true); }
        else { if (sharded) PSK_PCG_INIT(0, false); else PSK_PCG_INIT(0, true); }
#undef PSK_PCG_INIT
    }
    PSK_HIP(hipGetLastError());
    if (sharded) {
        if (mbc) PSK_TRY(mbox_gather(mbc, seq0, 2, w.initg, nullptr, s));
        else PSK_TRY(allgather(A, w.pinit, w.initg, 2, s));
        hipLaunchKernelGGL(pcg_init_finish_kernel, dim3(1), dim3(64), 0, s, w.initg, P, ctl->tau, w.st, w.udr,
                           const_cast<int64_t *>(hdone), hgen);
        PSK_HIP(hipGetLastError());
    }

    // polling: every C iterations an event; the host waits on the event L chunks back and then reads the
    // host-mapped done word the kernels set (set_done)
    const int L = 2, NS = kPollSlots;
    static_assert(kPollSlots >= L + 2, "poll slots");
    int C = ctl->check_every > 0 ? ctl->check_every : (n >= (1 << 20) ? 2 : 16);
    hipEvent_t *fev = kit->fev;
    // optional SpMV timing ring
    const int TP = kTimedSlots;
    hipEvent_t *ta = kit->ta, *tb = kit->tb;
    int64_t tk[kTimedSlots];
    bool tgat[kTimedSlots], thalo[kTimedSlots];   // sharded: the slot's gather / halo events were recorded
    for (int i = 0; i < TP; ++i) {
        tk[i] = -1;
        tgat[i] = thalo[i] = false;
    }
    std::vector<float> spmv_ms;
    if (ctl->time_kernels) spmv_ms.assign((size_t)maxiter, -1.0f);   // -1: not sampled
    double gat_sum = 0.0, halo_sum = 0.0;
    int64_t gat_n = 0, halo_n = 0;
    auto harvest = [&](int slot) -> int {
        if (tk[slot] < 0) return PSK_OK;
        float ms = 0.f;
        PSK_HIP(hipEventSynchronize(tb[slot]));
        PSK_HIP(hipEventElapsedTime(&ms, ta[slot], tb[slot]));
        spmv_ms[(size_t)tk[slot]] = ms;
        tk[slot] = -1;
        if (tgat[slot]) {
            PSK_HIP(hipEventSynchronize(kit->gb[slot]));
            PSK_HIP(hipEventElapsedTime(&ms, kit->ga[slot], kit->gb[slot]));
            gat_sum += ms;
            ++gat_n;
            tgat[slot] = false;
        }
        if (thalo[slot]) {
            PSK_HIP(hipEventSynchronize(kit->hb[slot]));
            PSK_HIP(hipEventElapsedTime(&ms, kit->ha[slot], kit->hb[slot]));
            halo_sum += ms;
            ++halo_n;
            thalo[slot] = false;
        }
        return PSK_OK;
    };

    // halo overlap (sharded, Jacobi/identity): when every row a neighbour needs lies in the first ov_lo
    // or the last nv - ov_hi K3 tiles (row-block shards of a banded matrix: one grid line each side),
    // those tiles run first and the exchange of p overlaps the remaining tiles of K3
    int64_t ov_lo = 0, ov_hi = nv;
    // On by default (PSK_HALO_OVERLAP=0 turns it off); DESIGN.md §6 states the rule: the overlap moves
    // no arithmetic (sharded histories are bit-identical either way) and takes the halo's latency off
    // the critical path whenever K3's interior tiles outlast the exchange, which they do at every
    // size the 8-GPU run uses (>= 1.25M rows per rank); an 8-GPU A/B of the driver's run decides it.
    static const bool overlap_on = [] {
        const char *e = std::getenv("PSK_HALO_OVERLAP");
        return !(e && std::atoi(e) == 0);
    }();
    const bool overlap = overlap_on && sharded && !gen && halo_split(A, kVecTile, nv, ov_lo, ov_hi);
    hipStream_t cs = nullptr;
    hipEvent_t ev_k3a = kit->ev_a, ev_halo = kit->ev_b;
    bool halo_pending = false;
    if (overlap) PSK_TRY(comm_stream(c, &cs));

    int64_t launched = 0;
    int rc = PSK_OK;
    for (int64_t k = 0; k < maxiter && rc == PSK_OK; ++k) {
        if (k > 0 && k % C == 0) {
            const int64_t chunk = k / C;   // chunks fully launched
            const int slot = (int)((chunk - 1) % NS);
            if (hipEventRecord(fev[slot], s) != hipSuccess) rc = fail(PSK_ERR_HIP, "event");
            if (rc == PSK_OK && chunk - 1 - L >= 0) {
                const int os = (int)((chunk - 1 - L) % NS);
                if (hipEventSynchronize(fev[os]) != hipSuccess) rc = fail(PSK_ERR_HIP, "event sync");
                else {
                    const int64_t hv = *hdone;   // a stamp of this solve only (its generation)
                    if ((hv & ~kStampMask) == hgen && (hv & kStampMask) != 0 &&
                        (hv & kStampMask) <= (chunk - L) * (int64_t)C + 1)
                        break;
                }
            }
            if (rc != PSK_OK) break;
        }
        // p_k and the buffer K3 writes p_{k+1} into (Jacobi/identity: a ring of kPcgDefer; general: in place)
        double *pk = gen ? w.p : w.pr.b[k % kPcgDefer];
        double *pn = gen ? w.p : w.pr.b[(k + 1) % kPcgDefer];
        // every time_kernels-th SpMV between two events (sampled: an event pair costs ~5% of an
        // iteration at N = 10M); sharded, the same iterations time this rank's p.Ap gather and the halo
        // exchange of the iteration (ABI 4: psk_result.gather_ms / halo_ms)
        // (init_diag: iteration 0's SpMV ran inside the init launch, not sampled)
        const bool timed = ctl->time_kernels > 0 && k % ctl->time_kernels == 0 && !(init_diag && k == 0);
        int slot = (int)((k / (ctl->time_kernels > 0 ? ctl->time_kernels : 1)) % TP);
        if (timed) {
            if ((rc = harvest(slot)) != PSK_OK) break;
            tk[slot] = k;
        }
        if (halo_pending) {   // exchanged during the previous K3
            if (hipStreamWaitEvent(s, ev_halo, 0) != hipSuccess) { rc = fail(PSK_ERR_HIP, "halo wait"); break; }
            halo_pending = false;
        } else if (A->comm) {
            const bool th = timed && !A->comm->dry && !A->peers.empty();
            if (th && hipEventRecord(kit->ha[slot], s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "event"); break; }
            if ((rc = halo_exchange(A, pk, s)) != PSK_OK) break;
            if (th) {
                if (hipEventRecord(kit->hb[slot], s) != hipSuccess) { rc = fail(PSK_ERR_HIP, "event"); break; }
                thalo[slot] = true;
            }
        }
        // a timed launch records its events in its own dispatch (kernel start / end)
        uint64_t seq1 = 0;
        if (!(init_diag && k == 0) &&
            (rc = launch_spmv(A, kSpmvDot, pk, w.Ap, nullptr, nullptr, w.part1, &w.st->done, s, timed ? ta[slot] : nullptr,
                              timed ? tb[slot] : nullptr, 0, mbc ? &seq1 : nullptr)) != PSK_OK)
            break;
        // K2/K3 tiles in block order: XCD bands matching the SpMV's, and bands walked in alternating
        // directions (a serpentine over SpMV, K2, K3 meant to re-read Ap, r and p from the Infinity Cache),
        // measured no faster (round 4, profiles/r4_spmv_ab.txt: band1 / band2)
        const TileMap tm2 = tile_map_for(nv, false);
        if (sharded) {
            hipEvent_t g0 = timed ? kit->ga[slot] : nullptr, g1 = timed ? kit->gb[slot] : nullptr;
            if (mbc) {
                rc = mbox_gather(mbc, seq1, 1, w.part1g, &w.st->done, s, g0, g1);
            } else {
                if (g0 && hipEventRecord(g0, s) != hipSuccess) rc = fail(PSK_ERR_HIP, "event");
                if (rc == PSK_OK) rc = allgather(A, w.part1, w.part1g, 1, s);
                if (rc == PSK_OK && g1 && hipEventRecord(g1, s) != hipSuccess) rc = fail(PSK_ERR_HIP, "event");
            }
            if (rc != PSK_OK) break;
            if (timed) tgat[slot] = true;
        }
        GridSum gs2k = gs2;   // this iteration's mailbox slot (sharded with a mailbox)
        const uint64_t seq2 = mbc ? mbox_next(mbc, &gs2k) : 0;
        // the general path copied r = b in its init (pcg_gen_init_kernel): it never takes the FIRST form
        const bool first = k == 0 && !gen && dev_io;
        const double *pap_k = w.part1g;
#define PSK_PCG_K2(J, F)                                                                                       \
        hipLaunchKernelGGL((pcg_update_kernel<J, F>), gk, dim3(kBlock), 0, s, n, w.r, bd, w.Ap, dinv, ds, pap_k,     \
                           P, gs2k, w.st, w.udr, k, tm2)
        if (jac == 2) { if (first) PSK_PCG_K2(2, true); else PSK_PCG_K2(2, false); }
        else if (jac == 1) { if (first) PSK_PCG_K2(1, true); else PSK_PCG_K2(1, false); }
        else { if (first) PSK_PCG_K2(0, true); else PSK_PCG_K2(0, false); }
#undef PSK_PCG_K2
        if (sharded && (rc = mbc ? mbox_gather(mbc, seq2, 2, w.part2g, &w.st->done, s)
                                 : allgather(A, w.part2, w.part2g, 2, s)) != PSK_OK)
            break;
        if (gen) {
            if ((rc = prec_apply_dev(M, n, w.r, w.u, s)) != PSK_OK) break;          // u = M^-1 r  :123
            hipLaunchKernelGGL(pcg_dot_kernel, gk, dim3(kBlock), 0, s, n, w.u, w.r, gs3, w.st);
            hipLaunchKernelGGL(pcg_gen_direction_kernel, gk, dim3(kBlock), 0, s, n, w.x, w.u, w.p, w.part1, w.part2,
                               w.part3, w.st, w.udr, w.hist, k, maxiter, ctl->fail_on_maxiter);
        } else {
            auto k3 = [&](int64_t t0, int64_t t1) {   // K3 over tiles [t0, t1)
                if (t1 <= t0) return;
                const dim3 g3((unsigned)(t1 - t0));
                const TileMap tm3 = tile_map_for(t1 - t0, false);
                if (jac == 2)
                    hipLaunchKernelGGL(pcg_direction_kernel<2>, g3, dim3(kBlock), 0, s, n, w.x, w.r, w.pr, dinv, ds,
                                       w.part1g, w.part2g, P, w.st, w.udr, w.hist, w.alphas, k, maxiter,
                                       ctl->fail_on_maxiter, t0, tm3);
                else if (jac == 1)
                    hipLaunchKernelGGL(pcg_direction_kernel<1>, g3, dim3(kBlock), 0, s, n, w.x, w.r, w.pr, dinv, ds,
                                       w.part1g, w.part2g, P, w.st, w.udr, w.hist, w.alphas, k, maxiter,
                                       ctl->fail_on_maxiter, t0, tm3);
                else
                    hipLaunchKernelGGL(pcg_direction_kernel<0>, g3, dim3(kBlock), 0, s, n, w.x, w.r, w.pr, dinv, ds,
                                       w.part1g, w.part2g, P, w.st, w.udr, w.hist, w.alphas, k, maxiter,
                                       ctl->fail_on_maxiter, t0, tm3);
            };
            if (overlap && k + 1 < maxiter) {
                // the tiles holding the rows the neighbours need first, then their halo exchange on the
                // second stream while the other tiles run; the next SpMV waits for it
                k3(0, ov_lo);
                k3(ov_hi, nv);
                if ((rc = halo_exchange_async(A, pn, s, cs, ev_k3a, ev_halo, timed ? kit->ha[slot] : nullptr,
                                              timed ? kit->hb[slot] : nullptr)) != PSK_OK)
                    break;
                if (timed) thalo[slot] = true;
                k3(ov_lo, ov_hi);
                halo_pending = true;
            } else {
                k3(0, nv);
            }
        }
        if (hipGetLastError() != hipSuccess) { rc = fail(PSK_ERR_HIP, "pcg launch"); break; }
        launched = k + 1;
    }
    // a halo exchange still in flight (the host stopped enqueueing first) completes before the end
    if (halo_pending && hipStreamWaitEvent(s, ev_halo, 0) != hipSuccess && rc == PSK_OK) rc = fail(PSK_ERR_HIP, "halo wait");
    if (rc == PSK_OK && hipEventRecord(kit->ev1, s) != hipSuccess) rc = fail(PSK_ERR_HIP, "event");
    // one launch and one synchronisation for the state, the ticket-counter scan and the gridsum error word,
    // all written by pcg_finish_kernel into the host-mapped words (round 5: was two copies and a kernel)
    int64_t *hw = kit->hmap + kPcgFinishWord;
    if (rc == PSK_OK) {
        hipLaunchKernelGGL(pcg_finish_kernel, dim3(1), dim3(kBlock), 0, s, w.st, c->gs_cnt, c->gs_err, hw);
        if (hipGetLastError() != hipSuccess) rc = fail(PSK_ERR_HIP, "pcg finish");
    }
    if (rc == PSK_OK && hipStreamSynchronize(s) != hipSuccess) rc = fail(PSK_ERR_HIP, "pcg sync");
    PcgState hs;
    std::memcpy(&hs, hw, sizeof(PcgState));
    if (rc == PSK_OK) rc = gridsum_check_result(c, (int32_t)hw[kPcgStateWords]);
    if (rc == PSK_OK && gen) rc = prec_check_error(M, s);
    if (rc == PSK_OK && ctl->time_kernels)
        for (int i = 0; i < TP && rc == PSK_OK; ++i) rc = harvest(i);
    if (rc == PSK_OK) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, kit->ev0, kit->ev1);
        res->loop_ms = ms;
        res->norm_b = hs.normB;
        // nk: iterations whose SpMV ran (the timing count); nhist: iterations that reported a
        // residual (K3 wrote hist[k]) — a dot(p,Ap) breakdown at k ran the SpMV of k but reports
        // only 0..k-1, as the reference's loop does (PCGSolver.py:114-115 returns before :126)
        int64_t nk = 0, nhist = 0;
        if (hs.done == 1) {
            res->status = PSK_CONVERGED;
            res->success = 1;
            res->iters = hs.iters;
            res->resid = hs.resid;
            res->exit = hs.normB == 0.0 ? PSK_EXIT_NONE
                        : hs.resid <= hs.tauNormB ? PSK_EXIT_TOLERANCE : PSK_EXIT_MAXITER;
            nk = nhist = hs.normB == 0.0 ? 0 : hs.iters;
        } else if (hs.done == 2) {
            res->status = PSK_BREAKDOWN;
            res->exit = PSK_EXIT_DOT_BREAKDOWN;
            res->success = 0;
            res->iters = hs.iters;
            res->resid = NAN;
            set_msg(res, hs.brk_kind == 1 ? "breakdown dot(u,r)==0" : "breakdown dot(p, Ap)==0");
            nk = hs.brk_kind == 1 ? 0 : hs.iters + 1;
            nhist = hs.brk_kind == 1 ? 0 : hs.iters;
        } else {
            // handleMaxiter(k=maxiter-1, ...) (IterativeSolver.py:115-129); maxiter==0 -> k unset
            res->status = PSK_MAXITER;
            res->exit = PSK_EXIT_MAXITER;
            res->success = 0;
            res->iters = maxiter > 0 ? maxiter - 1 : 0;
            set_msg(res, "failure to converge");
            nk = nhist = launched;
        }
        // residual history (only when asked for), the recursive residual and the solution
        const int64_t nh = nhist < maxiter ? nhist : maxiter;
        if (hist && nh > 0 && hipMemcpy(hist, w.hist, (size_t)nh * 8, hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(PSK_ERR_HIP, "hist copy");
        if (rc == PSK_OK) {
            res->hist_len = nh;
            res->resid_recursive = nh > 0 ? hs.last_hist : hs.normB;
            if (res->status == PSK_MAXITER) res->resid = maxiter > 0 ? res->resid_recursive : hs.normB;
            bool x_written = hs.x_written != 0;
            // a dot(p,Ap) breakdown at k: the iterations since the last flush deferred their x updates
            bool more = !dev_io;   // work enqueued after the sync: the caller's x is ready only after another sync
            if (!gen && hs.done == 2 && hs.brk_kind != 1 && pcg_pending(hs.iters) > 0 && n > 0) {
                hipLaunchKernelGGL(pcg_flush_kernel, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n,
                                   w.x, w.pr, w.alphas, (int64_t)hs.iters);
                if (hipGetLastError() != hipSuccess) rc = fail(PSK_ERR_HIP, "pcg flush");
                x_written = true;
                more = true;   // also when an earlier flush had already stored x
            }
            // no iteration stored x (b = 0, dot(u,r) = 0 at the start, maxiter = 0, or a dot(p,Ap)
            // breakdown at k = 0): the solution is x0 = 0
            if (rc == PSK_OK && !x_written && n > 0) {
                if (hipMemsetAsync(w.x, 0, (size_t)n * 8, s) != hipSuccess) rc = fail(PSK_ERR_HIP, "x zero");
                more = true;
            }
            if (rc == PSK_OK && !dev_io) rc = from_device_vec(w.x, loc, n, xout, s);
            if (rc == PSK_OK && more && hipStreamSynchronize(s) != hipSuccess) rc = fail(PSK_ERR_HIP, "x copy");
        }
        if (ctl->time_kernels) {
            double tot = 0.0;
            const int64_t cnt = nk < (int64_t)spmv_ms.size() ? nk : (int64_t)spmv_ms.size();
            int64_t nt = 0;
            for (int64_t i = 0; i < cnt; i += ctl->time_kernels)
                if (spmv_ms[(size_t)i] >= 0.0f) {
                    tot += spmv_ms[(size_t)i];
                    ++nt;
                }
            res->spmv_launches = nt;
            res->spmv_ms = nt > 0 ? tot / (double)nt : 0.0;
            res->gather_ms = gat_n > 0 ? gat_sum / (double)gat_n : 0.0;
            res->halo_ms = halo_n > 0 ? halo_sum / (double)halo_n : 0.0;
            res->comm_samples = gat_n;
        }
    }
    // a solve that failed on the host side leaves no kernel of its own running behind the next solve
    if (rc != PSK_OK) (void)hipStreamSynchronize(s);
    return rc;
}
