"""PyDP stand-in for utility-analysis fixtures (fixture generation only):
noise parameters restated (oracle/mechanisms.py, pinned by the reference's
own known answers), no noise is ever drawn."""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "..", "..", ".."))
from oracle import mechanisms  # noqa: E402


class LaplaceMechanism:

    def __init__(self, epsilon, sensitivity):
        self.epsilon = epsilon
        self.sensitivity = sensitivity
        self.diversity = sensitivity / epsilon

    def add_noise(self, value):
        return value


class GaussianMechanism:

    def __init__(self, epsilon, delta, sensitivity):
        self.epsilon = epsilon
        self.delta = delta
        self.l2_sensitivity = sensitivity
        self.std = mechanisms.gaussian_sigma(epsilon, delta, sensitivity)

    def add_noise(self, value):
        return value
