"""CPU oracle for the AEAD hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, as the checker.  See aead_oracle.h.
"""
