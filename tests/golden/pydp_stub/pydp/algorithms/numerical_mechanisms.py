"""No-noise stand-ins for PyDP Laplace/Gaussian mechanisms (fixture generation only)."""
import math


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
        # std is not needed by the fixtures; keep a finite placeholder.
        self.std = float("nan")

    @classmethod
    def create_from_standard_deviation(cls, stddev):
        m = cls(0.0, 0.0, 1.0)
        m.std = stddev
        return m

    def add_noise(self, value):
        return value
