"""CPU oracle for the trex Sankoff hot path -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg (as the checker / timed CPU baseline). Never shipped.
"""
