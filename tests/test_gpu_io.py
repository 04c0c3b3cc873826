"""configs[0] end to end from the file: DH-Matrix-8.mtx read natively into HBM, then PCG (identity),
compared with the reference's own run (tests/golden/pcg_dh8_identity.npz)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden_matrix, load_golden

pytestmark = pytest.mark.gpu


def test_from_mtx_spmv_and_pcg():
    import pysolvers_amd as psk
    d = load_golden("pcg_dh8_identity.npz")
    A_ref = golden_matrix(d)
    dA = psk.DeviceCSR.from_mtx(os.path.join(GOLDEN, "mtx", "DH-Matrix-8.mtx"))
    assert dA.shape == A_ref.shape and dA.nnz == A_ref.nnz
    B = dA.to_scipy()
    assert np.array_equal(B.indptr, A_ref.indptr) and np.array_equal(B.indices, A_ref.indices)
    assert np.array_equal(B.data, A_ref.data)
    x = d["x_exact"]
    assert np.array_equal(psk.Linear.spmv(dA, x), d["b"])          # b = mvmult(A, x), bitwise
    ctl = psk.CommonSolverArgs(maxiter=2000, tau=1e-8, showIters=False, showFinal=False)
    st = psk.PCG(control=ctl).makeSolver().solve(dA, d["b"])
    assert st.success() and st.iters() == int(d["iters"]) == 61
    assert np.linalg.norm(st.soln() - d["soln"]) <= 1e-9 * np.linalg.norm(d["soln"])
