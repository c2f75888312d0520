"""CPU restatement of the reference CBF hot path -- TEST INFRASTRUCTURE ONLY.

``pyoracle`` (pure Python, pinned to golden vectors captured from the
reference's cbf.py) and ``coracle`` (C, cross-checked bit-exactly against
``pyoracle``).  Only ``tests/``, ``__graft_entry__.smoke()`` and bench.py's
``cpu_baseline`` leg may import this package, and only as the checker.
"""
