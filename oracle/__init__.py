"""CPU oracle for the qppfuse hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything from here, and only as the checker.  The product (qpp-fusion-rag_amd/
qppfuse) never imports it and has no CPU fallback.
"""
