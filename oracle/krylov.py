"""ORACLE — test infrastructure only (see oracle/__init__.py).

Op-for-op numpy/scipy restatement of the reference Krylov loops.  Each
arithmetic statement mirrors one reference line, in the same order and with
the same temporaries, so that the result is bit-identical to the reference on
the same machine (checked by tests/golden/make_golden.py against the imported
reference).  Control-flow outcomes are returned as a plain dict instead of a
SolveStatus so the checker does not depend on the product's classes.

Reference defects are NOT reproduced as crashes:
  * GMRESSolver.py:71 reads ``self.precond`` which is never set -> we behave
    as if it were None (the preconditioner is built every solve);
  * GMRESSolver.py:180 references undefined ``norm_k`` at maxiter -> we return
    the failure status handleMaxiter would have built (IterativeSolver.py:115-129)
    with the recursive residual ``|g[k+1]|`` and the current iterate.
"""
import numpy as np
import numpy.linalg as npla


# ---------------------------------------------------------------------------
# preconditioner applies (Preconditioner.py:58-68; ClassicSmoothers.py:8,14)

def identity_apply(v):
    """IdentityPreconditioner.applyRight returns the very same array (Preconditioner.py:66-68)."""
    return v


def jacobi_form(A):
    """DInv = np.reciprocal(A.diagonal())  (pattern of ClassicSmoothers.py:8)."""
    DInv = np.reciprocal(A.diagonal())
    return lambda v: np.multiply(DInv, v)          # ClassicSmoothers.py:14


def ilut_form(A, drop_tol=0.001, fill_factor=15):
    """RightILUTPreconditioner: SuperLU spilu with the reference's arguments (ILUTPreconditioner.py:51-53);
    applyRight = ILU.solve (:77-78)."""
    import scipy.sparse.linalg as spla
    ilu = spla.spilu(A.tocsc(), drop_tol=drop_tol, fill_factor=fill_factor, diag_pivot_thresh=0.0)
    return ilu.solve


def ic_form(A, drop_tol=0.001, fill_factor=15):
    """RightIC: ICRightPreconditioner setup (ICPreconditioner.py:45-56) and applyRight (:58-63),
    the same scipy calls in the same order."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    ilu = spla.spilu(A.tocsc(), drop_tol=drop_tol, fill_factor=fill_factor, diag_pivot_thresh=0.0,
                     options={'ColPerm': 'NATURAL'})
    n = A.shape[0]
    dinv = sp.dia_matrix((np.reciprocal(np.sqrt(ilu.U.diagonal())), [0]), shape=(n, n))
    Lt = dinv * ilu.U
    L = Lt.transpose().tocsr()
    Lt = Lt.tocsr()

    def apply(v):
        u = spla.spsolve_triangular(L, v, lower=True)
        return spla.spsolve_triangular(Lt, u, lower=False)
    return apply


def mvmult(A, x):
    """IterativeLinearSolver.py:94-106: ``A*x`` -> scipy csr_matvec for sparse A."""
    return A @ x


def _status(success, iters, soln, resid, msg=None, hist=None):
    return dict(success=success, iters=iters, soln=soln, resid=resid, msg=msg,
                hist=np.array(hist if hist is not None else [], dtype=np.float64))


# ---------------------------------------------------------------------------
# PCG  (PCGSolver.py:64-142)

def pcg(A, b, maxiter=100, tau=1.0e-8, fail_on_maxiter=True, precond=identity_apply, on_iter=None,
        norm=npla.norm):
    """on_iter(k): optional hook called at the top of iteration k (bench.py's cpu_baseline times
    single iterations with it); it sees no solver state. norm: CommonSolverArgs.norm, used where the
    reference calls self.norm (IterativeSolver.py:86-88: PCGSolver.py:86 and :125)."""
    n, nc = A.shape
    assert n == nc                                   # :79-81
    assert n == len(b)                               # :83
    hist = []
    normB = norm(b)                                  # :86 (IterativeSolver.norm -> npla.norm)
    if normB == 0.0:                                 # :87-88 -> handleConvergence(0,...)
        return _status(True, 1, np.zeros_like(b), 0, hist=hist)
    r = np.copy(b)                                   # :97
    p = precond(r)                                   # :98
    u = np.copy(p)                                   # :99
    x = np.zeros_like(b)                             # :100
    uDotR = np.dot(u, r)                             # :102
    if uDotR == 0.0:                                 # :104-105
        return _status(False, 0, None, None, 'breakdown dot(u,r)==0', hist)
    k = -1
    normR = None
    for k in range(maxiter):                         # :109
        if on_iter is not None:
            on_iter(k)
        Ap = mvmult(A, p)                            # :111
        pTAp = np.dot(p, Ap)                         # :113
        if pTAp == 0.0:                              # :114-115
            return _status(False, k, None, None, 'breakdown dot(p, Ap)==0', hist)
        alpha = uDotR / pTAp                         # :118
        x = x + alpha * p                            # :121
        r = r - alpha * Ap                           # :122
        u = precond(r)                               # :123
        normR = norm(r)                              # :125
        hist.append(normR)
        if (normR <= tau * normB) or ((not fail_on_maxiter) and k == maxiter - 1):   # :129-131
            return _status(True, k + 1, x, normR, hist=hist)
        newUDotR = np.dot(u, r)                      # :134
        beta = newUDotR / uDotR                      # :135
        uDotR = newUDotR                             # :136
        p = u + beta * p                             # :138
    # handleMaxiter(k, x, normR, normB) (IterativeSolver.py:115-129); maxiter=0 -> k undefined
    # in the reference (NameError); we report iters=0.
    it = max(k, 0)
    if fail_on_maxiter:
        return _status(False, it, x, normR, 'failure to converge', hist)
    return _status(True, it, x, normR, hist=hist)


# ---------------------------------------------------------------------------
# Givens (Givens.py:7-34)

def find_givens_coefficients(x, i):
    hyp = np.sqrt(x[i + 1] * x[i + 1] + x[i] * x[i])     # Givens.py:8
    s = x[i + 1] / hyp                                   # :9
    c = x[i] / hyp                                       # :10
    return (c, s)


def apply_givens_in_place(x, c, s, i):
    xi = x[i]                                            # Givens.py:30
    xi1 = x[i + 1]
    x[i] = c * xi + s * xi1                              # :33
    x[i + 1] = -s * xi + c * xi1                         # :34


# ---------------------------------------------------------------------------
# GMRES (GMRESSolver.py:55-180), non-restarted, right preconditioned

def gmres(A, b, maxiter=100, tau=1.0e-8, fail_on_maxiter=True, precond=identity_apply,
          return_internals=False, norm=npla.norm):
    """norm: CommonSolverArgs.norm where the reference calls self.norm (GMRESSolver.py:66, :164); the
    Arnoldi norms are npla.norm in the reference itself (:90, :115, :121)."""
    n, nc = A.shape
    assert n == nc                                       # :61
    assert n == len(b)                                   # :63
    hist = []
    norm_b = norm(b)                                     # :66 (self.norm)
    if norm_b == 0.0:                                    # :67-68
        return _status(True, 1, np.zeros_like(b), 0, hist=hist)
    maxiters = maxiter                                   # :75
    Q = np.zeros([n, maxiters + 1])                      # :77 (C order: columns are strided)
    HBar = np.zeros([maxiters + 1, maxiters])            # :80
    CS = np.zeros([maxiters, 2])                         # :83
    r0 = b                                               # :87
    beta = npla.norm(r0)                                 # :90
    Q[:, 0] = r0 / beta                                  # :91
    e1 = np.zeros(maxiters + 1)                          # :95
    e1[0] = 1.0
    g = beta * e1                                        # :97
    arnoldiBreakdown = False
    k = -1
    norm_r_k = None
    for k in range(maxiters):                            # :104
        u = mvmult(A, precond(Q[:, k]))                  # :107
        for j in range(k + 1):                           # :110-112 (MGS)
            HBar[j, k] = np.dot(Q[:, j], u)
            u -= HBar[j, k] * Q[:, j]
        HBar[k + 1, k] = npla.norm(u)                    # :115
        hLastColNorm = npla.norm(HBar[0:k + 1, k])       # :121
        if abs(HBar[k + 1, k]) <= 1.0e-16 * hLastColNorm:   # :122
            arnoldiBreakdown = True
        else:
            Q[:, k + 1] = u / HBar[k + 1, k]             # :125
        for j in range(k):                               # :133-135
            apply_givens_in_place(HBar[:, k], CS[j, 0], CS[j, 1], j)
        CS[k, :] = find_givens_coefficients(HBar[:, k], k)     # :140
        apply_givens_in_place(HBar[:, k], CS[k, 0], CS[k, 1], k)   # :145
        apply_givens_in_place(g, CS[k, 0], CS[k, 1], k)            # :148
        norm_r_k = np.abs(g[k + 1])                      # :152
        hist.append(norm_r_k)
        if arnoldiBreakdown or (norm_r_k <= tau * norm_b):   # :158
            y = npla.solve(HBar[0:k + 1, 0:k + 1], g[0:k + 1])   # :159
            x = precond(np.dot(Q[:, 0:k + 1], y))        # :160
            resid = b - mvmult(A, x)                     # :163
            norm_r_true = norm(resid)                    # :164
            extra = dict(HBar=HBar[:k + 2, :k + 1].copy(), g=g[:k + 2].copy(), y=y) \
                if return_internals else {}
            if norm_r_true <= tau * norm_b:              # :165-166 -> handleConvergence
                st = _status(True, k + 1, x, norm_r_true, hist=hist)
            else:                                        # :167-174
                st = _status(False, k + 1, x, norm_r_true,
                             'GMRES failure: true residual did not meet tolerance', hist)
            st.update(extra)
            return st
    # maxiter reached: reference NameError at :180; we return what handleMaxiter(k, x, ...)
    # would have returned, with the current iterate assembled from the Krylov basis.
    it = max(k, 0)
    x = None
    if k >= 0:
        y = npla.solve(HBar[0:k + 1, 0:k + 1], g[0:k + 1])
        x = precond(np.dot(Q[:, 0:k + 1], y))
    if fail_on_maxiter:
        return _status(False, it, x, norm_r_k, 'failure to converge', hist)
    return _status(True, it, x, norm_r_k, hist=hist)


# ---------------------------------------------------------------------------
# Restarted GMRES(m): the reference has no restart (GMRESSolver.py:104 runs one Krylov space of
# dimension maxiter). GMRES(m) is cycles of the reference's own loop (:87-160) on the residual
# system A dx = r_c (r_0 = b, r_c = b - A x_c), each at most m steps, with the reference's
# convergence test against the ORIGINAL ||b|| (tau * ||b||, :158); x_{c+1} = x_c + dx_c.
# tests/golden/make_restarted.py pins every cycle bit for bit to the reference's own solve on
# (A, r_c) and writes the fixtures.

def gmres_cycle(A, r0, K, thresh, precond):
    """One cycle: at most K Arnoldi steps of GMRESSolver.py:87-158 from r0, stopping when |g[k+1]|
    <= thresh or Arnoldi breaks down. Returns (k, converged, hist, dx) with dx = M^-1 (Q y) (:159-160)
    over the k+1 basis vectors built."""
    n = A.shape[0]
    Q = np.zeros([n, K + 1])                             # :77
    HBar = np.zeros([K + 1, K])                          # :80
    CS = np.zeros([K, 2])                                # :83
    beta = npla.norm(r0)                                 # :90
    Q[:, 0] = r0 / beta                                  # :91
    e1 = np.zeros(K + 1)                                 # :95
    e1[0] = 1.0
    g = beta * e1                                        # :97
    hist = []
    for k in range(K):                                   # :104
        u = mvmult(A, precond(Q[:, k]))                  # :107
        for j in range(k + 1):                           # :110-112
            HBar[j, k] = np.dot(Q[:, j], u)
            u -= HBar[j, k] * Q[:, j]
        HBar[k + 1, k] = npla.norm(u)                    # :115
        hLastColNorm = npla.norm(HBar[0:k + 1, k])       # :121
        brk = abs(HBar[k + 1, k]) <= 1.0e-16 * hLastColNorm   # :122
        if not brk:
            Q[:, k + 1] = u / HBar[k + 1, k]             # :125
        for j in range(k):                               # :133-135
            apply_givens_in_place(HBar[:, k], CS[j, 0], CS[j, 1], j)
        CS[k, :] = find_givens_coefficients(HBar[:, k], k)         # :140
        apply_givens_in_place(HBar[:, k], CS[k, 0], CS[k, 1], k)   # :145
        apply_givens_in_place(g, CS[k, 0], CS[k, 1], k)            # :148
        norm_r_k = np.abs(g[k + 1])                      # :152
        hist.append(norm_r_k)
        if brk or norm_r_k <= thresh or k == K - 1:      # :158 (or the cycle's last step)
            y = npla.solve(HBar[0:k + 1, 0:k + 1], g[0:k + 1])   # :159
            dx = precond(np.dot(Q[:, 0:k + 1], y))       # :160
            return k, bool(brk or norm_r_k <= thresh), hist, dx
    raise ValueError("gmres_cycle: K must be >= 1")


def gmres_restarted(A, b, restart, maxiter=100, tau=1.0e-8, fail_on_maxiter=True, precond=identity_apply,
                    cycles=None):
    """GMRES(restart) with the reference's status conventions: convergence as :158-174 (iters =
    steps so far + 1, true residual ||b - A x|| checked); maxiter as the non-restarted solver's
    handleMaxiter(k, ...) with k = maxiter - 1 (iters = maxiter - 1, resid = last |g[k+1]|).
    `cycles`, if a list, receives (r_c, steps, dx_c) per cycle (make_restarted.py checks each
    against the reference)."""
    n, nc = A.shape
    assert n == nc and n == len(b)
    assert restart >= 1 and maxiter >= 1
    norm_b = npla.norm(b)                                # :66
    if norm_b == 0.0:                                    # :67-68
        return _status(True, 1, np.zeros_like(b), 0, hist=[])
    thresh = tau * norm_b                                # :158
    hist = []
    it = 0
    r = b                                                # :87 (first cycle)
    x = None
    while True:
        Kc = min(maxiter - it, restart)
        k, conv, h, dx = gmres_cycle(A, r, Kc, thresh, precond)
        hist += h
        if cycles is not None:
            cycles.append((r, k + 1, dx))
        x = dx if x is None else x + dx
        if conv:                                         # :159-174
            resid = b - mvmult(A, x)                     # :163
            norm_r_true = npla.norm(resid)               # :164
            if norm_r_true <= thresh:
                return _status(True, it + k + 1, x, norm_r_true, hist=hist)
            return _status(False, it + k + 1, x, norm_r_true,
                           'GMRES failure: true residual did not meet tolerance', hist)
        it += Kc
        if it >= maxiter:                                # handleMaxiter(maxiter - 1, ...)
            if fail_on_maxiter:
                return _status(False, maxiter - 1, x, h[-1], 'failure to converge', hist)
            return _status(True, maxiter - 1, x, h[-1], hist=hist)
        r = b - mvmult(A, x)                             # next cycle's residual system


def givens_selftest_matrix():
    """The 4x3 Hessenberg matrix and RHS of the reference's self-test (Givens.py:40-56)."""
    H = np.array([[1.0, -2.0, 3.0], [4.0, 5.0, 6.0], [0.0, 7.0, 8.0], [0.0, 0.0, 9.0]])
    g = np.array([1.0, 0.0, 0.0, 0.0])
    return H, g


def givens_triangularize(H, g):
    """Column-by-column Givens reduction of a Hessenberg matrix (Givens.py:86-101)."""
    H = H.copy()
    g = g.copy()
    n, m = H.shape
    CS = np.zeros([m, 2])
    for i in range(m):
        for j in range(i):
            apply_givens_in_place(H[:, i], CS[j, 0], CS[j, 1], j)
        CS[i, :] = find_givens_coefficients(H[:, i], i)
        apply_givens_in_place(H[:, i], CS[i, 0], CS[i, 1], i)
        apply_givens_in_place(g, CS[i, 0], CS[i, 1], i)
    y = npla.solve(H[0:m, :], g[0:m])
    return H, g, CS, y
