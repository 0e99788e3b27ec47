"""Test infrastructure only: CPU oracle for the GP-kriging hot path.

Nothing in the product package (``2d-gp_amd/``) may import this package.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker / CPU baseline.
"""
