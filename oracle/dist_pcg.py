"""ORACLE — test infrastructure only (see oracle/__init__.py).

Row-block distributed restatement of PCG (PCGSolver.py:64-142) with the SAME sharding plan the
device engine uses (psk_fd2d_dist_plan: whole grid lines per rank, local columns
[owned | halo_lo | halo_hi]) and the same communication structure: one halo exchange of p per
iteration with ranks r-1 / r+1, and sum-all-reduces of the local dot partials. Runs on CPU over a
torch.distributed gloo group; tests/test_dist_gloo.py checks it against the serial oracle, which
pins the plan, the local column remap and the exchange/reduction schedule on CPU.
"""
import numpy as np
import numpy.linalg as npla
import scipy.sparse as sp

from . import fdlap


def local_block(m, plan, a=-1.0, b=1.0):
    """Rows [rb, re) of FDLaplacian2D(a,b,m) with columns remapped to [owned | halo_lo | halo_hi]."""
    rb, re, ncols, hlo, hhi = plan
    ip, ix, dt = fdlap.fd_laplacian_2d_arrays(a, b, m)
    s, e = int(ip[rb]), int(ip[re])
    cols = ix[s:e].astype(np.int64)
    loc = np.empty_like(cols)
    own = (cols >= rb) & (cols < re)
    lo = cols < rb
    hi = cols >= re
    loc[own] = cols[own] - rb
    loc[lo] = (re - rb) + (cols[lo] - (rb - m))
    loc[hi] = (re - rb) + hlo + (cols[hi] - re)
    indptr = (ip[rb:re + 1] - s).astype(np.int64)
    return sp.csr_matrix((dt[s:e], loc, indptr), shape=(re - rb, ncols))


def _allreduce(dist, vals):
    import torch
    t = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(t)
    return t.numpy()


def _halo(dist, p_ext, nloc, m, hlo, hhi, rank):
    import torch
    reqs = []
    bufs = []
    if hlo:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(p_ext[:m])), rank - 1))
        rb_ = torch.empty(m, dtype=torch.float64)
        reqs.append(dist.irecv(rb_, rank - 1))
        bufs.append((nloc, rb_))
    if hhi:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(p_ext[nloc - m:nloc])), rank + 1))
        rh = torch.empty(m, dtype=torch.float64)
        reqs.append(dist.irecv(rh, rank + 1))
        bufs.append((nloc + hlo, rh))
    for r in reqs:
        r.wait()
    for off, t in bufs:
        p_ext[off:off + m] = t.numpy()


def dist_pcg(dist, m, Aloc, b, plan, maxiter, tau, fail_on_maxiter=True, jacobi=True):
    rank = dist.get_rank()
    rb, re, ncols, hlo, hhi = plan
    nloc = re - rb
    dinv = np.reciprocal(Aloc[:, :nloc].diagonal()) if jacobi else None
    M = (lambda v: np.multiply(dinv, v)) if jacobi else (lambda v: v)
    hist = []
    bb, = _allreduce(dist, [np.dot(b, b)])
    normB = np.sqrt(bb)
    r = np.copy(b)
    p = np.zeros(ncols)
    p[:nloc] = M(r)
    x = np.zeros_like(b)
    uDotR, = _allreduce(dist, [np.dot(p[:nloc], r)])
    for k in range(maxiter):
        _halo(dist, p, nloc, m, hlo, hhi, rank)
        Ap = Aloc @ p
        pTAp, = _allreduce(dist, [np.dot(p[:nloc], Ap)])
        alpha = uDotR / pTAp
        x = x + alpha * p[:nloc]
        r = r - alpha * Ap
        u = M(r)
        rr, ur = _allreduce(dist, [np.dot(r, r), np.dot(u, r)])
        normR = np.sqrt(rr)
        hist.append(normR)
        if normR <= tau * normB or ((not fail_on_maxiter) and k == maxiter - 1):
            return dict(iters=k + 1, x=x, hist=np.array(hist), success=True)
        beta = ur / uDotR
        uDotR = ur
        p[:nloc] = u + beta * p[:nloc]
    return dict(iters=max(maxiter - 1, 0), x=x, hist=np.array(hist), success=False)
