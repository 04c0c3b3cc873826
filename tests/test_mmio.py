"""Native MatrixMarket reader (psk_mm_read) == scipy.io.mmread(path).tocsr(), bit for bit (CPU only).

Inputs: the reference's DH-8 / DH-10 test matrices (TestMatrices/, copied as data into
tests/golden/mtx/) and hand-written files covering every header combination the reader accepts.
"""
import os

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

from conftest import GOLDEN

MTX = os.path.join(GOLDEN, "mtx")


def _same(A, B):
    A, B = sp.csr_matrix(A), sp.csr_matrix(B)
    return (A.shape == B.shape and np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
            and np.array_equal(np.asarray(A.data, dtype=np.float64).view(np.uint64),
                               np.asarray(B.data, dtype=np.float64).view(np.uint64)))


@pytest.mark.parametrize("name", ["DH-Matrix-8.mtx", "DH-Matrix-10.mtx"])
def test_dh_matrices(name):
    from pysolvers_amd.io import mmread_csr
    p = os.path.join(MTX, name)
    A = mmread_csr(p)
    R = scipy.io.mmread(p).tocsr()
    assert _same(A, R)


FILES = {
    "general_real": "%%MatrixMarket matrix coordinate real general\n% comment\n3 4 5\n1 1 1.5\n3 4 -2e-3\n"
                    "2 2 0.0\n1 3 7\n3 1 0.1\n",
    "symmetric_upper_entries": "%%MatrixMarket matrix coordinate real symmetric\n4 4 5\n1 1 2\n2 1 -1\n1 3 0.25\n"
                               "4 4 1e300\n3 2 -3.5\n",
    "skew": "%%MatrixMarket matrix coordinate real skew-symmetric\n3 3 2\n2 1 5\n3 1 -0.5\n",
    "pattern": "%%MatrixMarket matrix coordinate pattern general\n3 3 3\n1 2\n2 3\n3 1\n",
    "integer_sym": "%%MatrixMarket matrix coordinate integer symmetric\n3 3 3\n1 1 4\n2 1 -7\n3 3 9\n",
    "duplicates": "%%MatrixMarket matrix coordinate real general\n2 2 4\n1 1 1.0\n1 1 2.5\n2 1 3\n1 2 4\n",
    "crlf_and_comments": "%%MatrixMarket matrix coordinate real general\r\n%c\r\n2 2 2\r\n1 1 0.1\r\n2 2 0.3\r\n",
    "empty_rows": "%%MatrixMarket matrix coordinate real general\n5 5 2\n5 1 1\n1 5 2\n",
    "upper_case_banner": "%%MatrixMarket MATRIX Coordinate REAL General\n1 1 1\n1 1 3.14159265358979\n",
}


@pytest.mark.parametrize("name", sorted(FILES))
def test_header_variants(tmp_path, name):
    from pysolvers_amd.io import mmread_csr
    p = tmp_path / (name + ".mtx")
    p.write_bytes(FILES[name].encode())
    A = mmread_csr(p)
    R = scipy.io.mmread(str(p)).tocsr()
    assert _same(A, R), (A.toarray(), R.toarray())


@pytest.mark.parametrize("text", [
    "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",              # dense array format
    "%%MatrixMarket matrix coordinate complex general\n1 1 1\n1 1 1 0\n",        # complex field
    "%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1\n3 1 1\n",     # index out of range
    "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n",            # too few entries
    "not a matrix market file\n",
    # size lines claiming more than the file can hold / more than int32 CSR (found by the ASan run,
    # scripts/asan_host.sh: the first one made the reader's reserve throw through the C ABI)
    "%%MatrixMarket matrix coordinate real general\n3 3 9000000000000000000\n1 1 1\n",
    "%%MatrixMarket matrix coordinate real symmetric\n3 3 4611686018427387904\n1 1 1\n",
    "%%MatrixMarket matrix coordinate real general\n99999999999 3 1\n1 1 1\n",
])
def test_rejects(tmp_path, text):
    from pysolvers_amd import _native as N
    from pysolvers_amd.io import mmread_csr
    p = tmp_path / "bad.mtx"
    p.write_bytes(text.encode())
    with pytest.raises(N.PskError):
        mmread_csr(p)


def test_random_roundtrip(tmp_path):
    from pysolvers_amd.io import mmread_csr
    rng = np.random.default_rng(0)
    M = sp.random(300, 200, density=0.05, random_state=rng, format="csr")
    M.data = rng.standard_normal(M.nnz) * 10.0 ** rng.integers(-20, 20, M.nnz)
    p = tmp_path / "r.mtx"
    scipy.io.mmwrite(str(p), M, precision=17)
    assert _same(mmread_csr(p), scipy.io.mmread(str(p)).tocsr())
    S = sp.random(150, 150, density=0.05, random_state=rng)
    S = (S + S.T).tocsr()
    p2 = tmp_path / "s.mtx"
    scipy.io.mmwrite(str(p2), S, symmetry="symmetric", precision=17)
    assert _same(mmread_csr(p2), scipy.io.mmread(str(p2)).tocsr())
