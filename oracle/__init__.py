"""CPU oracle for the adversarial-patch hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (the HIP library behind the package) never imports it.

Parity pinning status: the reference repository has no
tests, fixtures or golden vectors, and executing the reference's Python in
this environment was denied.  This oracle is a PyTorch-CPU
fp32 restatement that follows the reference op for op (file:line citations on
every function).  It is pinned by the analytic known-answer tests of SURVEY.md
Appendix B (``tests/test_oracle_kat.py``) and by committed fixtures it
generated (``tests/golden/``).  It is NOT pinned by any output of the
reference itself: "parity unpinned" against the reference's own numbers.
"""
from .reference_path import *  # noqa: F401,F403
