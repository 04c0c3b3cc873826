import json
import os
import sys

import numpy as np
import pytest
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libpsk)")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_matrix(d, prefix=""):
    n = int(d[prefix + "n"])
    A = sp.csr_matrix((d[prefix + "data"], d[prefix + "indices"], d[prefix + "indptr"]), shape=(n, n))
    A.has_sorted_indices = False
    return A


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def solver_cases(kind=None):
    return [c for c in manifest()["cases"] if kind is None or c["kind"] == kind]


# AMG preconditioner variants of the golden cases (tests/golden/make_golden.py AMG_VARIANTS):
# name -> (numIters, numLevels, smoother)
AMG_VARIANTS = {"amg": (2, 2, "gs"), "amg_jacobi": (2, 2, "jacobi"), "amg3": (2, 3, "gs")}


def case_precond(case):
    return case.get("precond", "jacobi" if case["jacobi"] else "identity")


def oracle_prec(A, name):
    """The oracle's preconditioner apply for a golden-case preconditioner name."""
    from oracle import amg, krylov
    if name in AMG_VARIANTS:
        it, lv, sm = AMG_VARIANTS[name]
        return amg.AMGApply(A, num_iters=it, num_levels=lv, smoother=sm)
    return {"identity": lambda: krylov.identity_apply, "jacobi": lambda: krylov.jacobi_form(A),
            "ilut": lambda: krylov.ilut_form(A), "ic": lambda: krylov.ic_form(A)}[name]()


def product_prec_type(psk, name):
    """pysolvers_amd PreconditionerType for a golden-case preconditioner name."""
    if name in AMG_VARIANTS:
        it, lv, sm = AMG_VARIANTS[name]
        kw = {"smoother": psk.JacobiSmoother} if sm == "jacobi" else {}
        return psk.AMG(numIters=it, numLevels=lv, **kw)
    return {"identity": psk.IdentityPreconditionerType, "jacobi": psk.JacobiPreconditionerType,
            "ilut": psk.RightILUT, "ic": psk.RightIC}[name]()


def restarted_cases():
    """GMRES(m) golden cases (tests/golden/make_restarted.py: every cycle pinned to the reference's
    own GMRES solve on the residual system)."""
    with open(os.path.join(GOLDEN, "manifest_restarted.json")) as f:
        return json.load(f)["cases"]


def direct_manifest():
    """DefaultDirect / Newton-with-default-solver fixtures (tests/golden/make_direct.py)."""
    with open(os.path.join(GOLDEN, "manifest_direct.json")) as f:
        return json.load(f)


def dense_cases():
    """Dense-ndarray-A solver fixtures (tests/golden/make_dense.py: the reference's np.dot path)."""
    with open(os.path.join(GOLDEN, "manifest_dense.json")) as f:
        return json.load(f)["cases"]
