/*
 * psk.h — C ABI of libpsk.so, the MI355X (gfx950) Krylov engine behind
 * pysolvers_amd.Linear (a drop-in for krlong014/PySolvers' PySolvers/Linear).
 *
 * Plain C: pointers, sizes and PODs only; no torch/HIP types cross this line.
 * Every entry point returns PSK_OK (0) or a negative PSK_ERR_* code; the text
 * of the last error of the calling thread is available from psk_last_error().
 * NUMERICAL failure (breakdown, maxiter, GMRES true-residual miss) is NOT an
 * error: it is reported in psk_result.status exactly as the reference reports
 * it through SolveStatus(success=False, ...) (IterativeSolver.py:101-129).
 *
 * Reference interfaces each group replaces (paths relative to the reference root):
 *   psk_csr_*        scipy.sparse CSR handed to LinearSolver.solve(A, b)
 *                    (LinearSolver.py:30-33) — uploaded once, kept in HBM.
 *   psk_spmv         mvmult(A, x)                 IterativeLinearSolver.py:94-106
 *   psk_dot/nrm2     np.dot / IterativeSolver.norm (npla.norm)  IterativeSolver.py:86-88
 *   psk_axpy         x + alpha*p style updates    PCGSolver.py:121-122,138
 *   psk_prec_*       PreconditionerType.form(A) -> applyRight(vec)
 *                    PreconditionerType.py:4-19, Preconditioner.py:3-68;
 *                    JACOBI = DInv*v with DInv = reciprocal(diag(A)) (ClassicSmoothers.py:8,14)
 *   psk_pcg          PCGSolver.solve              PCGSolver.py:64-142
 *   psk_gmres        GMRESSolver.solve            GMRESSolver.py:55-180 (restart==0)
 *   psk_comm_*, psk_csr_create_fd2d_dist: row-block sharding across GPUs (RCCL over
 *                    xGMI); no reference counterpart (the reference is single-process).
 *   psk_csr_create_fd2d: examples/FDLaplacian2D.py:5-23 generated on the device,
 *                    bit-identical arrays and entry order.
 *   psk_prec_create_trisolve  RightIC applyRight (ICPreconditioner.py:58-63), Gauss-Seidel
 *                    smoother U^-1 (ClassicSmoothers.py:28-36), coarse SuperLU solve
 *                    (VCycleManager.py:34-37): one sync-free triangular-solve chain.
 *   psk_prec_create_amg  AMGPreconditioner.apply (AMGPreconditioner.py:46-51) ->
 *                    AMGVCycleSolver.solve (VCycleSolver.py:52-95) -> VCycleManager.runLevel
 *                    (VCycleManager.py:31-62), hierarchy built on the host.
 *   psk_mm_*         scipy.io.mmread(path).tocsr() (examples/DHTestProblem.py:27-28).
 *   psk_sa_aggregate BuildAggregates + BuildFilteredMatrix (SmoothedAggregation.py:57-183),
 *                    O(nnz) host code.
 */
#ifndef PSK_H
#define PSK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSK_ABI_VERSION 4

/* return codes */
#define PSK_OK               0
#define PSK_ERR_ARG         -1   /* bad argument (AssertionError in the reference, PCGSolver.py:79-83) */
#define PSK_ERR_HIP         -2
#define PSK_ERR_RCCL        -3
#define PSK_ERR_ALLOC       -4
#define PSK_ERR_UNSUPPORTED -5

/* psk_result.status */
#define PSK_CONVERGED        0   /* handleConvergence            IterativeSolver.py:101-107 */
#define PSK_MAXITER          1   /* handleMaxiter                IterativeSolver.py:115-129 */
#define PSK_BREAKDOWN        2   /* handleBreakdown              IterativeSolver.py:109-113 */
#define PSK_TRUE_RESID_FAIL  3   /* GMRES true residual missed   GMRESSolver.py:167-174 */

/* psk_result.exit: why the iteration loop stopped (gates the host-side checks a caller-supplied
   norm needs, e.g. the GMRES true-residual test GMRESSolver.py:163-174, without inferring it from
   the history length) */
#define PSK_EXIT_NONE             0   /* no loop ran (b = 0: IterativeSolver.py:86-88 / GMRESSolver.py:67-68) */
#define PSK_EXIT_TOLERANCE        1   /* recursive residual <= tau*||b||  PCGSolver.py:129, GMRESSolver.py:158 */
#define PSK_EXIT_ARNOLDI_BREAKDOWN 2  /* GMRES: h_{k+1,k} <= 1e-16 ||h_k|| (counts as convergence, :122,:158) */
#define PSK_EXIT_MAXITER          3   /* maxiter reached (k == maxiter-1 with !failOnMaxiter for PCG, :130) */
#define PSK_EXIT_DOT_BREAKDOWN    4   /* PCG dot(u,r) == 0 or dot(p,Ap) == 0  :104-105, :114-115 */

/* where the vector pointers of a call live */
#define PSK_HOST   0
#define PSK_DEVICE 1

/* preconditioner kinds */
#define PSK_PREC_IDENTITY 0      /* IdentityPreconditionerType   PreconditionerType.py:13-19 */
#define PSK_PREC_JACOBI   1      /* DInv*v                        ClassicSmoothers.py:5-16 pattern */
#define PSK_PREC_ILU      2      /* triangular-solve chain: SuperLU ILU.solve ILUTPreconditioner.py:70-78,
                                    IC, Gauss-Seidel, coarse LU (psk_prec_create_trisolve) */
#define PSK_PREC_AMG      3      /* smoothed-aggregation V-cycles  AMGPreconditioner.py:46-51 */
#define PSK_PREC_DENSE    4      /* x = A^-1 f by a dense inverse: the AMG coarse solve spsolve(A_c, f),
                                    VCycleManager.py:34-37 (psk_prec_create_dense_inverse) */

typedef struct psk_csr  psk_csr;    /* device CSR (int32 rowptr/colidx, f64 vals), library-owned */
typedef struct psk_prec psk_prec;   /* formed preconditioner, library-owned */
typedef struct psk_comm psk_comm;   /* RCCL communicator + rank geometry */

/* CommonSolverArgs (IterativeSolver.py:42-57) minus the print knobs. */
typedef struct psk_ctl {
    int64_t maxiter;          /* CommonSolverArgs.maxiter */
    double  tau;              /* relative residual tolerance */
    int32_t fail_on_maxiter;  /* CommonSolverArgs.failOnMaxiter */
    int32_t restart;          /* GMRES only: 0 = reference non-restarted (Krylov dim = maxiter) */
    int32_t check_every;      /* host polls the device status every N iterations; 0 = auto */
    int32_t time_kernels;     /* S > 0: HIP-event timing of every S-th SpMV launch (iterations k with
                                 k % S == 0; psk_result.spmv_ms); 0 = off */
    double  norm_b;           /* GMRES: > 0 = ||b|| in the caller's norm (CommonSolverArgs.norm,
                                 GMRESSolver.py:66) for the threshold tau*||b|| and psk_result.norm_b;
                                 0 = the device 2-norm. PCG ignores it (a non-2-norm PCG is driven by
                                 the host, IterativeSolver.py:86-88). Zero-initialise. */
} psk_ctl;

typedef struct psk_result {
    int32_t status;           /* PSK_CONVERGED / MAXITER / BREAKDOWN / TRUE_RESID_FAIL */
    int32_t success;          /* SolveStatus.success() */
    int64_t iters;            /* SolveStatus.iters() (reference conventions, incl. k on maxiter) */
    double  resid;            /* SolveStatus.resid(): PCG recursive ||r||; GMRES true ||b-Ax|| */
    double  resid_recursive;  /* last recursive residual estimate */
    double  norm_b;           /* ||b|| */
    double  loop_ms;          /* device wall time of the solve (HIP events) */
    double  spmv_ms;          /* mean duration of the timed SpMV launches when ctl.time_kernels */
    int64_t spmv_launches;    /* number of SpMV launches (the timed ones when ctl.time_kernels) */
    int64_t hist_len;         /* valid entries written to hist */
    char    msg[256];         /* SolveStatus.msg() */
    int32_t exit;             /* PSK_EXIT_* (ABI 3) */
    int32_t reserved;
    /* ABI 4, sharded PCG with ctl.time_kernels: the iterations whose SpMV is timed also time, on this rank,
     * the scalar exchange after that SpMV (p.Ap: the mailbox gather kernel — its duration is the wait for the
     * slowest rank plus the transport — or the RCCL all-gather) and the halo exchange of p that feeds the
     * next SpMV (pack + send/recv, on the stream that runs it: the second stream when overlapped with K3).
     * Means over the samples; 0 when unsharded or untimed. */
    double  gather_ms;
    double  halo_ms;
    int64_t comm_samples;
} psk_result;

/* ---- library / device ---------------------------------------------------------------- */
int         psk_abi_version(void);
const char *psk_last_error(void);
int         psk_device_count(int32_t *n);
int         psk_set_device(int32_t dev);
int         psk_synchronize(void);
/* Drain every device stream and release the library's process-lifetime resources (streams, events,
 * host-mapped words, reduction arrays) while the HIP runtime is alive; call once at process exit
 * (the Python binding registers it with atexit). Afterwards entry points that need a device return
 * PSK_ERR_ARG and psk_csr_destroy / psk_prec_destroy / psk_dfree are no-ops. No reference
 * counterpart (process teardown). */
int         psk_shutdown(void);
/* psk_shutdown with options. PSK_SHUTDOWN_RESET_DEVICE: afterwards hipDeviceReset() every device the
 * library used, releasing the HIP runtime's own per-device state (e.g. its cooperative-launch queue) while
 * HSA is alive; only for a process in which libpsk is the only HIP user (the Python binding passes it
 * when torch was never imported) and skipped while an RCCL communicator is alive. No reference
 * counterpart (process teardown). */
#define PSK_SHUTDOWN_RESET_DEVICE 1
int         psk_shutdown_ex(int32_t flags);
/* device memory helpers (so a host binding can keep vectors resident in HBM) */
int psk_dmalloc(int64_t bytes, void **dptr);
int psk_dfree(void *dptr);
int psk_h2d(void *dst, const void *src, int64_t bytes);
int psk_d2h(void *dst, const void *src, int64_t bytes);
int psk_dmemset0(void *dst, int64_t bytes);

/* ---- CSR matrices ---------------------------------------------------------------------- */
/* Copy a CSR matrix (rowptr[n+1], colidx[nnz], vals[nnz]; stored entry order is kept,
 * sorted or not) into HBM. loc says where the three arrays live. int32 indices:
 * nnz <= 2^31 - 1 - 1536 (PSK_ERR_UNSUPPORTED beyond; FD 16384^2 has 1.34e9). */
int psk_csr_create(int64_t n, int64_t nnz, const int32_t *rowptr, const int32_t *colidx,
                   const double *vals, int32_t loc, psk_csr **out);
/* FDLaplacian2D(a, b, m) generated on the device (examples/FDLaplacian2D.py:5-23). */
int psk_csr_create_fd2d(double a, double b, int64_t m, psk_csr **out);
/* Rectangular nrows x ncols CSR (AMG prolongators / restrictions, MLHierarchy.py:283-292). */
int psk_csr_create_rect(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t *rowptr, const int32_t *colidx,
                        const double *vals, int32_t loc, psk_csr **out);
int psk_csr_info(const psk_csr *A, int64_t *n, int64_t *nnz);
/* SpMV storage layout of A (same y bit for bit either way; the CSR arrays are always kept):
 *   PSK_LAYOUT_CSR          one workgroup per tile of rows, the tile's entries streamed in stored
 *                           order and the products staged through LDS;
 *   PSK_LAYOUT_SLICED       a sliced copy: 256-row slices, slot-major inside a slice, one row per
 *                           lane, padding slots up to the slice's widest row, values in slot pairs
 *                           (16-B loads); a slice whose columns all lie within +-32767 of their rows
 *                           stores 16-bit column deltas two to a 32-bit word, any other slice 32-bit
 *                           columns;
 *   PSK_LAYOUT_SLICED_WIDE  the same with 32-bit columns in every slice;
 *   PSK_LAYOUT_SLICED_DICT  SLICED with the values replaced by one-byte indices into a dictionary of
 *                           the matrix's distinct values (at most 8 bit patterns: stencils, graph
 *                           Laplacians), 3 B per slot with 16-bit columns;
 *   PSK_LAYOUT_DIAG         (round 5) diagonal storage: every row's entries lie, in stored order, on
 *                           a subsequence of K <= 8 diagonals c = row + d_j (a row-block shard's
 *                           outside columns mapped to its halo) and all entries of a diagonal hold
 *                           one value (constant-coefficient stencils such as FDLaplacian2D); the
 *                           offsets and values are kernel arguments, one presence byte per row.
 * Every creation path picks DIAG when the matrix has one, else SLICED_DICT (values permitting) or
 * SLICED when its stream is no larger than the CSR stream (12 B/entry + 4 B/row); env
 * PSK_SPMV_LAYOUT=csr|sliced|sliced_wide|sliced_dict|diag overrides (sliced: no dictionary),
 * PSK_SPMV_DIAG=0 leaves DIAG out of the automatic choice. Forcing SLICED_DICT on a matrix with more
 * than 8 distinct values, or DIAG on one without the diagonal structure, fails with
 * PSK_ERR_UNSUPPORTED. set = -1 queries, a PSK_LAYOUT_*
 * value switches (building or freeing the copy). Out: *slots = padded slots of the sliced copy (0
 * without one; DIAG: n K), *packed_slots = those in 16-bit slices, *stream_bytes = matrix bytes one
 * SpMV streams in the current layout (CSR: 12 nnz + 4 (n+1); DIAG: n). Out pointers may be NULL. Replaces
 * nothing in the reference (scipy keeps CSR): a device storage choice under mvmult
 * (IterativeLinearSolver.py:94-106). */
#define PSK_LAYOUT_CSR         0
#define PSK_LAYOUT_SLICED      1
#define PSK_LAYOUT_SLICED_WIDE 2
#define PSK_LAYOUT_SLICED_DICT 3
#define PSK_LAYOUT_DIAG        4
int psk_csr_layout(psk_csr *A, int32_t set, int32_t *layout, int64_t *slots, int64_t *packed_slots,
                   int64_t *stream_bytes);
/* Copy the arrays back to host buffers (any pointer may be NULL). */
int psk_csr_download(const psk_csr *A, int32_t *rowptr, int32_t *colidx, double *vals);
int psk_csr_destroy(psk_csr *A);

/* ---- kernels on the hot path ------------------------------------------------------------ */
/* y = A x, per-row stored-order sum from 0.0, product rounded before the add:
 * bit-identical to scipy csr_matvec. For a distributed matrix x is the local
 * [owned | halo] vector and the halo is refreshed first (collective). */
int psk_spmv(const psk_csr *A, const double *x, double *y, int32_t loc);
/* Measurement: `reps` back-to-back y = A x launches (device pointers) between two HIP events on
 * the library stream; *avg_ms = elapsed / reps (one untimed warm-up launch first). */
int psk_spmv_timed(const psk_csr *A, const double *x, double *y, int32_t reps, double *avg_ms);
int psk_dot(int64_t n, const double *x, const double *y, int32_t loc, double *out);
int psk_nrm2(int64_t n, const double *x, int32_t loc, double *out);
/* y = y + alpha*x (two roundings, as numpy's y + alpha*x) */
int psk_axpy(int64_t n, double alpha, const double *x, double *y, int32_t loc);

/* ---- preconditioners (PreconditionerType.form / applyRight) ---------------------------- */
int psk_prec_create(const psk_csr *A, int32_t kind, psk_prec **out);
/* ILU from host factors of SuperLU spilu (RightILUTPreconditioner, ILUTPreconditioner.py:51-53):
 * L (unit lower, diagonal optional) and U (upper with diagonal) as CSR, perm_r / perm_c as in
 * scipy's SuperLU (Pr A Pc = L U). apply(v) = (U^-1 L^-1 (v scattered by perm_r))[perm_c]. */
int psk_prec_create_ilu(int64_t n, const int32_t *l_rowptr, const int32_t *l_colidx, const double *l_vals,
                        const int32_t *u_rowptr, const int32_t *u_colidx, const double *u_vals,
                        const int32_t *perm_r, const int32_t *perm_c, psk_prec **out);
/* General triangular-solve chain on the device (host CSR arrays, copied):
 *   bb[j] = v[gather_in[j]]          (gather_in NULL: bb = v)
 *   y = L^-1 bb                      (L lower; l_unit: unit diagonal, stored diagonal entries ignored;
 *                                     else the stored diagonal divides; L NULL: y = bb)
 *   z = U^-1 y                       (U upper; same rules with u_unit; U NULL: z = y)
 *   out[i] = z[gather_out[i]]        (gather_out NULL: out = z)
 * Row i's off-diagonal products are accumulated in stored order with FMA, then one wave sum. */
int psk_prec_create_trisolve(int64_t n, const int32_t *l_rowptr, const int32_t *l_colidx, const double *l_vals,
                             int32_t l_unit, const int32_t *u_rowptr, const int32_t *u_colidx,
                             const double *u_vals, int32_t u_unit, const int32_t *gather_in,
                             const int32_t *gather_out, psk_prec **out);
/* Direct solve x = A^-1 f through the explicit inverse, formed once on the device (rocSOLVER getrf +
 * getri, loaded at first use) and applied as one streamed GEMV per solve, with `refine` (0..4) steps of
 * x <- x + A^-1 (f - A x) after it. Replaces spsolve(A_c, f) for the AMG coarse level
 * (VCycleManager.py:34-37; pass it as psk_prec_create_amg's `coarse`). A is BORROWED (refinement).
 * PSK_ERR_UNSUPPORTED when n > 32768 (8.6 GB) or rocSOLVER cannot be loaded, PSK_ERR_ARG when A is
 * singular. The input vector of an apply must be 16-byte aligned. */
int psk_prec_create_dense_inverse(const psk_csr *A, int32_t refine, psk_prec **out);
/* Smoothed-aggregation AMG preconditioner over a host-built hierarchy (levels 0 = coarsest ..
 * num_levels-1 = finest, MLHierarchy.py:250-258). Arrays of num_levels handles, all BORROWED
 * (they must outlive the preconditioner): A[k] level matrices (A[num_levels-1] = the fine A),
 * P[k] (n_{k+1} x n_k) and R[k] (n_k x n_{k+1}) for k < num_levels-1, smoother[k] for k >= 1
 * (any preconditioner S: one sweep is x <- x + S^-1 (f - A x): PSK_PREC_ILU upper solve with
 * triu(A_k) = Gauss-Seidel, PSK_PREC_JACOBI = Jacobi; ClassicSmoothers.py:5-36), coarse = the
 * level-0 direct solve. apply(v): x = v; num_iters V-cycles, stopping after the first cycle whose
 * ||v - A x|| < tau ||v|| (VCycleSolver.py:119-146). */
int psk_prec_create_amg(int32_t num_levels, psk_csr *const *A, psk_csr *const *P, psk_csr *const *R,
                        psk_prec *const *smoother, psk_prec *coarse, int32_t num_iters, int32_t nu_pre,
                        int32_t nu_post, double tau, psk_prec **out);
/* Schedule of factor `which` (0 = L, 1 = U) of a triangular-solve chain: 0 = sync-free (one wave per
 * row, global dependency levels), 1 = band (one workgroup per block of the solve order, local levels
 * behind barriers, LDS ring of ring_words doubles), 2 = LDS (factors of at most 18432 rows: one
 * workgroup, sync-free inside it with x in LDS), 3 = grid (2-D stencil factors: one wave per band of
 * 64 lines advancing along a skewed coordinate), 4 = part (rows cut into strips of their natural
 * index, one workgroup per CU, in-strip dependencies through LDS; its layout is built when chosen or
 * when PSK_TRISOLVE_PART=1 at creation), 5 = levels (round 5: ONE workgroup, a dependency level per step
 * behind a barrier, x in an LDS ring; for factors with narrow levels and dependencies a bounded number of
 * solve positions back; built when chosen or when PSK_TRISOLVE_LEVELS=1 at creation). The library picks the fastest by host cost models
 * (est_*_us); set = 0..5 forces one (PSK_ERR_UNSUPPORTED when the factor has no such layout), -1 only
 * queries. Any out pointer may be NULL. */
int psk_prec_trisolve_schedule(psk_prec *M, int32_t which, int32_t set, int32_t *schedule, int64_t *blocks,
                               int32_t *ring_words, double *est_syncfree_us, double *est_band_us);
/* Grid-schedule shape of factor `which` (0 = L, 1 = U): out[0..6] = line width w, lines H, twice the
 * skew sigma2 and its phase (a solve-order position y*w + x - off runs at step x + ((sigma2*y + phase)
 * >> 1)), leading empty positions off, steps per 64-line band, dictionary records (0 = per-step
 * records). PSK_ERR_UNSUPPORTED when the factor is not a 2-D stencil. No compute (diagnostics, tests). */
int psk_prec_trisolve_grid_info(const psk_prec *M, int32_t which, int64_t *out);
/* Host-only: the grid plan psk_prec_create_trisolve would make for one triangular factor (CSR with its
 * diagonal; upper = 1: solved from the last row up), without any device work — out[0..6] = w, H,
 * sigma2, phase, off, steps per band, record width K. PSK_ERR_UNSUPPORTED when it is not a 2-D stencil. */
int psk_trisolve_grid_plan(int64_t n, const int32_t *rowptr, const int32_t *colidx, const double *vals,
                           int32_t upper, int64_t *out);
/* kind, size and triangular-solve shape of a preconditioner (any out pointer may be NULL). */
int psk_prec_info(const psk_prec *M, int32_t *kind, int64_t *n, int64_t *nnz_l, int64_t *nnz_u,
                  int64_t *levels_l, int64_t *levels_u);
/* Jacobi: *uniform = 1 when every DInv entry is the same double (*value; constant-diagonal matrices
 * such as stencils), in which case psk_pcg reads that scalar instead of streaming DInv (same
 * products bit for bit, 16 B per row and iteration less). PSK_JACOBI_UNIFORM=0 at creation disables. */
int psk_prec_jacobi_uniform(const psk_prec *M, int32_t *uniform, double *value);
int psk_prec_apply(const psk_prec *M, int64_t n, const double *v, double *out, int32_t loc);
int psk_prec_destroy(psk_prec *M);

/* ---- MatrixMarket input (host only, except psk_csr_create_mm) --------------------------------- */
/* scipy.io.mmread(path).tocsr() (examples/DHTestProblem.py:27-28) for coordinate files:
 * real/integer/pattern, general/symmetric/skew-symmetric; symmetric files expanded, rows sorted by
 * column, duplicates summed, explicit zeros kept. psk_mm_info gives the sizes (nnz_max = entries,
 * doubled for symmetric files) so the caller can allocate rowptr[nrows+1], colidx/vals[nnz_max];
 * psk_mm_read fills them and returns the actual nnz. */
int psk_mm_info(const char *path, int64_t *nrows, int64_t *ncols, int64_t *nnz_max);
int psk_mm_read(const char *path, int32_t *rowptr, int32_t *colidx, double *vals, int64_t *nnz);
int psk_csr_create_mm(const char *path, psk_csr **out);

/* ---- AMG setup (host only, no GPU needed) --------------------------------------------------- */
/* Smoothed-aggregation coarsening of one level, SmoothedAggregation.py:41-183 in O(nnz):
 * agg[i] = aggregate of node i (the reference's list order: isolated nodes, then phase-1
 * aggregates; phase 2 by strongest |A[i,k]|), *count = number of aggregates, and af_vals =
 * the values of the filtered matrix A_f (same structure as A; entries outside N_i lumped onto
 * the diagonal in stored order, including the neighbourhood growth the reference's set aliasing
 * causes). tol is the strength threshold (0.08 * 0.5^(lvl-1) by default). */
int psk_sa_aggregate(int64_t n, const int32_t *rowptr, const int32_t *colidx, const double *vals, double tol,
                     int32_t *agg, int64_t *count, double *af_vals);

/* ---- solvers ------------------------------------------------------------------------------ */
/* M == NULL means identity. b, x: length n (local length for a distributed A); with loc ==
 * PSK_DEVICE b is read in place and x written in place during the solve (x must not alias b). hist: nullable
 * HOST array of ctl->maxiter doubles receiving the per-iteration residual norms reportIter
 * sees (PCG ||r_k||, GMRES |g[k+1]|); entries past res->iters+1 are left untouched.
 * x is overwritten with the solution (SolveStatus.soln()). */
int psk_pcg(const psk_csr *A, const psk_prec *M, const double *b, double *x, const psk_ctl *ctl,
            psk_result *res, double *hist, int32_t loc);
int psk_gmres(const psk_csr *A, const psk_prec *M, const double *b, double *x, const psk_ctl *ctl,
              psk_result *res, double *hist, int32_t loc);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ------------------------------------- */
#define PSK_UNIQUE_ID_BYTES 128
int psk_comm_unique_id(uint8_t *id /* PSK_UNIQUE_ID_BYTES */);
int psk_comm_init(int32_t nranks, int32_t rank, const uint8_t *id, psk_comm **out);
/* Validation only: a communicator of `nranks` with no RCCL behind it. Sharded matrices can be
 * built on ONE GPU for any rank and psk_spmv then takes the full local [owned | halo] x from the
 * caller; collectives (and hence sharded solves) return PSK_ERR_UNSUPPORTED. */
int psk_comm_init_dry(int32_t nranks, int32_t rank, psk_comm **out);
/* Validation only: a communicator whose collectives run through a POSIX shared-memory segment
 * `name` ("/..."; the same on every rank, unique per job) between nranks processes of ONE host,
 * stream-ordered like the RCCL calls they stand in for (D2H, host barrier, H2D). Lets the sharded
 * solvers run with nranks > 1 on a single GPU, where RCCL refuses duplicate devices. Slow; never
 * used for timing. */
int psk_comm_init_host(int32_t nranks, int32_t rank, const char *name, psk_comm **out);
/* Device-side exchange of the sharded solvers' scalars (round 5): attach the host-shared mailbox `name`
 * ('/...', a POSIX shared-memory name, the same on every rank; collective over the ranks of c, which
 * must share one node). psk_pcg then exchanges its per-rank dot products by direct system-scope stores
 * of the kernels that finish them into every rank's mailbox slot and a one-wave gather kernel per rank,
 * instead of ncclAllGather (the halo of p stays on RCCL / the host transport). Same bits as the
 * all-gather: every rank still sums the P values in rank order. Replaces nothing in the reference. */
int psk_comm_mailbox(psk_comm *c, const char *name);
/* Self-check of the attached mailbox (collective over c's ranks): `rounds` exchanges of known values
 * through the same kernel stores and gather the solvers use; PSK_ERR_RCCL when a value is wrong or never
 * arrives (bounded wait). bench.py runs it before a multi-GPU run and falls back to RCCL all-gathers. */
int psk_comm_mailbox_check(psk_comm *c, int32_t rounds);
int psk_comm_destroy(psk_comm *c);
/* Rank `rank`'s row block of FDLaplacian2D(a,b,m): rows [row_begin,row_end) split on
 * whole grid lines; local columns are [owned | halo_lo | halo_hi]. */
int psk_csr_create_fd2d_dist(double a, double b, int64_t m, psk_comm *c, psk_csr **out,
                             int64_t *row_begin, int64_t *row_end);
/* Host-only: the row block and local column layout psk_csr_create_fd2d_dist uses for `rank`
 * (callable without a GPU; the CPU tests check the sharding plan with it). */
int psk_fd2d_dist_plan(int64_t m, int32_t nranks, int32_t rank, int64_t *row_begin, int64_t *row_end,
                       int64_t *ncols, int64_t *halo_lo, int64_t *halo_hi);
/* General row-block sharding: rank c->rank's rows [row_starts[rank], row_starts[rank+1]) of a
 * global n_global x n_global CSR (the row split of every rank in row_starts[nranks+1], 0 ..
 * n_global). Host arrays of the local rows only, GLOBAL column indices: rowptr[nloc+1] may start
 * anywhere (entry j of local row i is colidx[rowptr[i]-rowptr[0]+j']); stored order is kept.
 * Local columns are [owned | halo], the halo being the distinct off-block columns in ascending
 * global order (psk_csr_halo_cols). The pattern must be structurally symmetric across ranks (as
 * any matrix PCG runs on): each rank sends a peer the owned rows that reference the peer's block,
 * which is then exactly what the peer needs; under RCCL every rank checks this at creation and all
 * of them return PSK_ERR_ARG otherwise. Halo sends that are not a contiguous row range are packed
 * by one gather kernel before the grouped ncclSend/ncclRecv. Replaces: nothing in the reference
 * (single-process); the solvers take such a matrix with rank-local b and x. */
int psk_csr_create_dist(int64_t n_global, const int64_t *row_starts, const int64_t *rowptr,
                        const int32_t *colidx, const double *vals, psk_comm *c, psk_csr **out);
/* Global index of every halo column of a sharded matrix, in local column order (cols may be
 * NULL to query the count). */
int psk_csr_halo_cols(const psk_csr *A, int64_t *cols, int64_t *count);
/* Halo plan of a sharded matrix, one entry per peer rank (ascending): what is sent to it and which
 * segment of the halo it fills. Arrays may be NULL; *npeers <= nranks-1. */
int psk_csr_halo_peers(const psk_csr *A, int32_t *ranks, int64_t *send_counts, int64_t *recv_counts,
                       int64_t *recv_offsets, int32_t *npeers);
/* Validation: the values halo_exchange sends, peer by peer, for the local vector x (device
 * pointers; out holds sum(send_counts) doubles), packed by the same kernel. No communication. */
int psk_csr_halo_pack(const psk_csr *A, const double *x, double *out);

#ifdef __cplusplus
}
#endif
#endif /* PSK_H */
