"""Test infrastructure: CPU oracle of the reference renderer (see render_oracle.py header).

Never imported by the product package; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it.
"""
