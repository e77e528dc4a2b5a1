"""CPU oracle for the record-batch hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this package, and only as the checker.  See rporacle.h for what it restates.
"""
from .oracle import *  # noqa: F401,F403
