"""CPU restatement of the reference's smoothed-aggregation AMG preconditioner (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (pysolvers_amd) never does.

Restates, with the same scipy/numpy operations where the reference uses them and O(nnz) loops where
the reference uses quadratic Python set loops:

* SmoothedAggregation.py:41-55   getNeighborhood      -> strong_mask()
* SmoothedAggregation.py:57-143  BuildAggregates      -> build_aggregates()
* SmoothedAggregation.py:145-155 BuildTentativeProlongator (column = aggregate index)
* SmoothedAggregation.py:157-183 BuildFilteredMatrix  -> filtered_matrix()
* SmoothedAggregation.py:185-205 SmoothProlongator    -> smooth_prolongator()
* SmoothedAggregation.py:208-229 SA_coarsen           -> sa_coarsen()
* MLHierarchy.py:294-322         _setUpdate / makeRestrictionOp -> restriction(), hierarchy()
* VCycleManager.py:31-62, ClassicSmoothers.py:5-36, VCycleSolver.py:52-95,
  AMGPreconditioner.py:46-51      -> vcycle(), amg_apply()

Pinned bitwise against the reference (tests/golden/make_golden.py, amg_* fixtures: P, R, A_c and
one apply output per case).
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def default_tol(lvl):
    """Vanek's default strength tolerance (SmoothedAggregation.py:62-63, 214-215)."""
    return 0.08 * (0.5) ** (lvl - 1)


def _rows(A):
    return np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))


def strong_mask(A, tol):
    """Per stored entry: |a_ij| >= tol*sqrt(a_ii*a_jj) (SmoothedAggregation.py:49-54).

    N_i = {i} U {j : mask}. numpy float64 arithmetic in the reference's order (tol * sqrt(.)).
    """
    d = A.diagonal()
    rows = _rows(A)
    with np.errstate(invalid="ignore"):
        thr = tol * np.sqrt(d[rows] * d[A.indices])
    return np.abs(A.data) >= thr


def build_aggregates(A, tol):
    """Aggregate index of every node, and the aggregate count (SmoothedAggregation.py:57-143).

    List order of the reference: isolated nodes first (index order, :72-77), then phase-1
    aggregates in creation order (:83-89). Phase 2 (:96-127) attaches each remaining node i to the
    phase-1-snapshot aggregate with the strictly largest |A[i,k]| over its members k among the
    aggregates intersecting N_i (first in list order on ties); with no positive strength it goes to
    aggregates[-1]. Phase 2 never removes i from R, so phase 3 (:135) never runs.

    Returns (agg, count, root, late): root[c] = the node whose neighbourhood SET OBJECT aggregate c
    is (the reference appends neighborhoods[i] itself, :75 and :88), late[j] = j joined in phase 2.
    Phase 2's `aggregates[idx].add(i)` therefore also grows neighborhoods[root[idx]], which
    BuildFilteredMatrix reads afterwards (see filter_mask).
    """
    n = A.shape[0]
    ip, ix = A.indptr, A.indices
    strong = strong_mask(A, tol)
    nbr = []
    for i in range(n):
        s = ix[ip[i]:ip[i + 1]][strong[ip[i]:ip[i + 1]]]
        nbr.append(set(s.tolist()) | {i})
    agg = np.full(n, -1, dtype=np.int64)
    in_r = np.ones(n, dtype=bool)
    late = np.zeros(n, dtype=bool)
    root = []
    count = 0
    for i in range(n):                      # isolated nodes (:73-77)
        if len(nbr[i]) == 1:
            agg[i] = count
            in_r[i] = False
            root.append(i)
            count += 1
    for i in range(n):                      # phase 1 (:84-89)
        if in_r[i] and all(in_r[j] for j in nbr[i]):
            for j in nbr[i]:
                agg[j] = count
                in_r[j] = False
            root.append(i)
            count += 1
    snap = agg.copy()                       # aggcopy (:101)
    if count == 0 and in_r.any():
        raise IndexError("no aggregate to attach remaining nodes to (reference: aggregates[-1])")
    for i in range(n):                      # phase 2 (:104-127)
        if not in_r[i]:
            continue
        cand = {snap[j] for j in nbr[i] if snap[j] >= 0}
        vals = {}
        for kk in range(ip[i], ip[i + 1]):  # A[i,k] sums duplicate entries
            k = ix[kk]
            if snap[k] in cand:
                vals[k] = vals.get(k, 0.0) + A.data[kk]
        best, best_c = 0.0, -1
        for c in sorted(cand):
            for k, v in vals.items():
                if snap[k] == c and abs(v) > best:
                    best, best_c = abs(v), c
        agg[i] = best_c if best_c >= 0 else count - 1
        late[i] = True
    return agg, count, np.array(root, dtype=np.int64), late


def filter_mask(A, strong, agg, root, late):
    """Per stored entry (i,j): j in neighborhoods[i] as BuildFilteredMatrix sees it (:165, :177):
    the original N_i, plus -- when i is the root of aggregate c -- every node that joined c in
    phase 2 (aliasing of the aggregate and neighbourhood sets, see build_aggregates)."""
    n = A.shape[0]
    rows = _rows(A)
    is_root_of = np.full(n, -1, dtype=np.int64)
    is_root_of[root] = np.arange(root.shape[0])
    j = A.indices
    grown = (is_root_of[rows] >= 0) & late[j] & (agg[j] == is_root_of[rows])
    return strong | (j == rows) | grown


def tentative_prolongator(agg, count):
    """P_hat[j, agg[j]] = 1 (SmoothedAggregation.py:145-155), as CSR."""
    n = agg.shape[0]
    return sp.csr_matrix((np.ones(n), agg.astype(np.int32), np.arange(n + 1, dtype=np.int32)), shape=(n, count))


def filtered_matrix(A, keep):
    """A_f: entries outside N_i lumped onto the (first) diagonal entry in stored order (:157-183).
    `keep` = filter_mask(): per stored entry, whether its column is in N_i."""
    Af = A.copy()
    n = A.shape[0]
    ip, ix = Af.indptr, Af.indices
    d = Af.data
    iptr = None
    for i in range(n):
        row = range(ip[i], ip[i + 1])
        nbr = {ix[k] for k in row if keep[k]} | {i}
        for k in row:
            if ix[k] == i:
                iptr = k
                break
        for k in row:
            if ix[k] not in nbr:
                d[iptr] -= d[k]
                d[k] = 0
    return Af


def smooth_prolongator(Phat, A, Af, omega=(2 / 3)):
    """P = (I - omega D^-1 A_f) P_hat with the reference's elementwise order (:185-205)."""
    S = omega * Af
    dA = A.diagonal()
    rows = _rows(S)
    v = S.data / dA[rows]
    S.data[:] = np.where(S.indices == rows, 1 - v, -v)
    return S.dot(Phat)


def sa_coarsen(A, lvl=1):
    """Prolongator of one level (SA_coarsen, :208-229)."""
    tol = default_tol(lvl)
    strong = strong_mask(A, tol)
    agg, count, root, late = build_aggregates(A, tol)
    Phat = tentative_prolongator(agg, count)
    Af = filtered_matrix(A, filter_mask(A, strong, agg, root, late))
    return smooth_prolongator(Phat, A, Af).tocsr(), agg


def restriction(P):
    """makeRestrictionOp(P, normalize=True) (MLHierarchy.py:304-322) = P^T, UNnormalised.

    The reference's normalisation is a no-op: `row = I_down.getrowview(r); row /= nrm` rebinds
    the view's row list inside lil __itruediv__ (`self[:,:] = self / other`) and never writes back
    into I_down (measured: R == P^T bitwise on DH-8). What remains is P^T through lil: sorted
    columns, duplicates summed, explicit zeros kept.
    """
    R = P.transpose(copy=True).tocsr()
    R.sum_duplicates()
    return R


def hierarchy(A, num_levels=2):
    """ops[k], updates[k] (P: level k -> k+1), downdates[k] (R) as SmoothedAggregationMLHierarchy
    (SmoothedAggregation.py:14-22, MLHierarchy.py:294-301). Level num_levels-1 is the finest."""
    ops = [None] * num_levels
    P = [None] * num_levels
    R = [None] * num_levels
    ops[num_levels - 1] = A
    for lev in reversed(range(num_levels - 1)):
        P[lev], _ = sa_coarsen(ops[lev + 1], lvl=lev + 1)
        R[lev] = restriction(P[lev])
        ops[lev] = R[lev] * (ops[lev + 1] * P[lev])
    return ops, P, R


def smooth(kind, A, aux, f, x, nu, tri=False):
    """ClassicSmoothers.py: Gauss-Seidel (:28-36, aux = triu(A).tocsr()) or Jacobi (:5-14, aux = DInv).

    tri=True replaces the reference's spsolve(triu(A), r) (a full SuperLU factorisation per call:
    98 s at 4M rows) by spsolve_triangular — the same upper solve, rounded differently (measured
    8e-16 relative at -FD 2048^2); only for the large-size tests, never for the pinned fixtures."""
    for _ in range(nu):
        r = f - A * x
        if kind == "gs":
            x = x + (spla.spsolve_triangular(aux, r, lower=False) if tri else spla.spsolve(aux, r))
        else:
            x = x + np.multiply(aux, r)
    return x


def smoother_aux(kind, A):
    return sp.triu(A).tocsr() if kind == "gs" else np.reciprocal(A.diagonal())


def vcycle(ops, P, R, aux, kind, f, x, lev, nu_pre=2, nu_post=2, tri=False):
    """VCycleManager.runLevel (VCycleManager.py:31-62)."""
    if lev == 0:
        return spla.spsolve(ops[0], f)
    x = smooth(kind, ops[lev], aux[lev], f, x, nu_pre, tri)
    r = f - ops[lev] * x
    r2 = R[lev - 1] * r
    x2 = vcycle(ops, P, R, aux, kind, r2, np.zeros_like(r2), lev - 1, nu_pre, nu_post, tri)
    x = x + P[lev - 1] * x2
    return smooth(kind, ops[lev], aux[lev], f, x, nu_post, tri)


class AMGApply:
    """AMGPreconditioner.apply (AMGPreconditioner.py:46-51) -> AMGVCycleSolver.solve with
    CommonSolverArgs(maxiter=num_iters, failOnMaxiter=False) (VCycleSolver.py:52-95)."""

    def __init__(self, A, num_iters=5, num_levels=2, nu_pre=2, nu_post=2, smoother="gs", tau=1e-8, levels=None,
                 tri=False):
        """levels: a prebuilt (ops, P, R) (large-size tests hand in a hierarchy checked separately);
        tri: Gauss-Seidel by spsolve_triangular (see smooth())."""
        self.A = A
        self.ops, self.P, self.R = levels if levels is not None else hierarchy(A, num_levels)
        self.tri = tri
        self.aux = [smoother_aux(smoother, M) for M in self.ops]
        self.kind, self.num_iters, self.nu_pre, self.nu_post, self.tau = smoother, num_iters, nu_pre, nu_post, tau
        self.L = len(self.ops)

    def __call__(self, b):
        nb = np.linalg.norm(b)
        if nb == 0.0:
            return np.zeros_like(b)
        x = np.copy(b)
        for _ in range(self.num_iters):
            x = vcycle(self.ops, self.P, self.R, self.aux, self.kind, b, x, self.L - 1, self.nu_pre, self.nu_post,
                       self.tri)
            r = b - self.A * x
            if np.linalg.norm(r) < self.tau * nb:
                return x
        return x
