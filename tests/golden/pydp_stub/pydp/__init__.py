"""TEST-ONLY stand-in for the un-vendored PyDP package (python-dp==1.1.4).

Used exclusively by tests/golden/gen_golden.py, in the build container, to
import the read-only reference (/root/reference) and record golden
input/output vectors for the *noise-free* part of DPEngine.aggregate
(bounding, accumulation, merge, budget split).  It adds no noise and keeps
every partition, so the recorded outputs are exactly the pre-noise
aggregates.  Never imported by the product, smoke() or bench.py.
"""
