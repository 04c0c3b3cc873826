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


def test_lab_entry_points_only_in_the_lab_library():
    """psk_lab_* (include/psk_lab.h) live in libpsk_lab.so, not in the product library or its header."""
    from pysolvers_amd import _native as N
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "psk_lab.h")).read(), flags=re.S)
    lab_names = sorted(set(re.findall(r"\b(psk_lab_[a-z0-9_]+)\s*\(", txt)))
    assert lab_names and sorted(N.LAB_SIGNATURES) == lab_names
    assert not [n for n in _declared() if n.startswith("psk_lab_")]
    prod = ctypes.CDLL(N.LIB_PATH)
    assert not [n for n in lab_names if hasattr(prod, n)]
    lab = N.load_lab()
    assert all(hasattr(lab, n) for n in lab_names)


def test_library_basic_calls_without_gpu():
    from pysolvers_amd import _native as N
    assert N.lib.psk_abi_version() == N.ABI_VERSION == 4
    n = N.device_count()
    assert n >= 0
    assert isinstance(N.lib.psk_last_error(), bytes)


def test_struct_layout_matches_header(tmp_path):
    """The ctypes structs against the C compiler's layout of include/psk.h (gcc, plain C)."""
    import subprocess
    from pysolvers_amd import _native as N
    prog = tmp_path / "layout.c"
    fields = {"psk_ctl": [f for f, _ in N.PskCtl._fields_], "psk_result": [f for f, _ in N.PskResult._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "psk.h"', 'int main(void) {']
    for st, fs in fields.items():
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (st, st))
        for f in fs:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (st, f, st, f))
    lines.append('return 0; }')
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), str(prog), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    for st, cls in (("psk_ctl", N.PskCtl), ("psk_result", N.PskResult)):
        assert int(got["%s sizeof" % st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(got["%s %s" % (st, f)]) == getattr(cls, f).offset, (st, f)


def test_no_cpu_fallback_when_library_missing(tmp_path):
    """The product must fail loudly without the HIP library."""
    import subprocess
    import sys
    code = ("import os; os.environ['PSK_LIBRARY']='%s';\n"
            "try:\n    import pysolvers_amd\nexcept ImportError as e:\n    print('IMPORTERROR', e)\n"
            % str(tmp_path / "nope.so"))
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=120)
    assert "IMPORTERROR" in out.stdout
