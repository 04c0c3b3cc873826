"""libpsk.so loads without a GPU and exports every symbol include/psk.h declares."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "psk.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(psk_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_entry_points():
    names = _declared()
    for must in ("psk_pcg", "psk_gmres", "psk_spmv", "psk_dot", "psk_nrm2", "psk_axpy", "psk_csr_create",
                 "psk_prec_create", "psk_comm_init", "psk_csr_create_fd2d_dist"):
        assert must in names


def test_library_exports_all_symbols():
    from pysolvers_amd import _native as N
    lib = ctypes.CDLL(N.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes binding covers exactly the header
    assert sorted(N.SIGNATURES) == _declared()


def test_library_basic_calls_without_gpu():
    from pysolvers_amd import _native as N
    assert N.lib.psk_abi_version() == 2
    n = N.device_count()
    assert n >= 0
    assert isinstance(N.lib.psk_last_error(), bytes)


def test_struct_layout_matches_header():
    from pysolvers_amd import _native as N
    # psk_ctl: int64, double, 4 x int32, double ; psk_result: see include/psk.h
    assert ctypes.sizeof(N.PskCtl) == 40
    # psk_result: 2 x int32, int64, 5 x double, 2 x int64, char[256]
    assert N.PskResult.msg.offset == 4 + 4 + 8 + 5 * 8 + 2 * 8
    assert ctypes.sizeof(N.PskResult) == 72 + 256


def test_no_cpu_fallback_when_library_missing(tmp_path):
    """The product must fail loudly without the HIP library."""
    import subprocess
    import sys
    code = ("import os; os.environ['PSK_LIBRARY']='%s';\n"
            "try:\n    import pysolvers_amd\nexcept ImportError as e:\n    print('IMPORTERROR', e)\n"
            % str(tmp_path / "nope.so"))
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=120)
    assert "IMPORTERROR" in out.stdout
