"""PyDP partition-selection stand-in for utility-analysis fixtures: the
keep probabilities restated in oracle/mechanisms.py (truncated geometric
pinned by the reference's known answers; thresholding unpinned)."""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "..", "..", ".."))
from oracle import mechanisms  # noqa: E402


class _Strategy:

    def __init__(self, name, eps, delta, l0, pre):
        self.pre = pre or 0
        if name == "truncated_geometric":
            tab = mechanisms.truncated_geometric_table(eps, delta, l0)
            self.base = lambda n: tab[n] if n < len(tab) else 1.0
        elif name == "laplace":
            thr, b = mechanisms.laplace_threshold(eps, delta, l0)
            self.base = lambda n: (1 - 0.5 * math.exp(-(n - thr) / b) if n >= thr
                                   else 0.5 * math.exp((n - thr) / b))
        else:
            thr, s = mechanisms.gaussian_threshold(eps, delta, l0)
            self.base = lambda n: 0.5 * math.erfc(-(n - thr) / s / math.sqrt(2))

    def probability_of_keep(self, n):
        if n <= 0:
            return 0.0
        if self.pre:
            if n < self.pre:
                return 0.0
            n = n - self.pre + 1
        return self.base(n)

    def should_keep(self, n):
        return True


def create_partition_strategy(name, epsilon, delta, max_partitions, pre_threshold=None):
    return _Strategy(name, epsilon, delta, max_partitions, pre_threshold)
