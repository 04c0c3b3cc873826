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
