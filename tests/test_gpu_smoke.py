"""The driver's round-end smoke() (__graft_entry__.py) runs inside the GPU suite too, so a change of the
default layout or of the solve path cannot leave it failing unnoticed until the round ends."""
import pytest

pytestmark = pytest.mark.gpu


def test_graft_entry_smoke():
    import __graft_entry__ as g
    g.smoke()
