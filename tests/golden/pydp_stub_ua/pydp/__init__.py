"""TEST-ONLY stand-in for the un-vendored PyDP package (python-dp==1.1.4),
for tests/golden/gen_golden_ua.py (utility-analysis fixtures): noise
parameters and keep probabilities restated from oracle/mechanisms.py, no
noise drawn.  Never imported by the product, smoke() or bench.py."""
