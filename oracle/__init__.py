"""CPU oracle for the GRiD steps 4-7 hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``grid_amd/`` imports this package; only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may use it, and only as the checker / CPU baseline, never as the
thing measured or shipped.

Every function is a from-scratch NumPy / pure-Python restatement of the
reference algorithm (caterer-z-t/GRiD, mounted read-only at /root/reference)
with the same IEEE-754 fp64 operation order, cited file:line per function.
It is pinned against golden vectors produced by importing the reference
itself (``tests/golden/make_golden.py``) and checked by
``tests/test_oracle_golden.py``.
"""
