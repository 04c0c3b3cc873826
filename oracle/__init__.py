"""ORACLE — test infrastructure only, never the product.

CPU restatement of the reference (krlong014/PySolvers) Krylov path, used
solely as the checker: by ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py``.  The product (``pysolvers_amd``) never
imports anything from here.

Pinning: every function in this package was checked bit-for-bit against the
imported reference in this container by ``tests/golden/make_golden.py``; the
resulting golden vectors are committed under ``tests/golden/`` and
``tests/test_oracle_golden.py`` re-checks the oracle against them.
"""
