"""Oracle package -- TEST INFRASTRUCTURE ONLY (checker, never the measured or shipped path).

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
