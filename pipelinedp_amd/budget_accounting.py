"""Privacy budget accounting (API mirror of pipeline_dp/budget_accounting.py).

`NaiveBudgetAccountant` keeps the reference's semantics exactly
(budget_accounting.py:301-408): mechanisms are requested lazily during graph
construction, scopes normalise the weights of the mechanisms requested inside
them (:289-298), and `compute_budgets()` splits epsilon by weight over every
mechanism and delta only over the non-Laplace ones (:393-408).  The device
path reads `spec.eps` / `spec.delta` only when the lazy result is
materialised, i.e. after `compute_budgets()`.

The PLD accountant (:411-619) needs the `dp_accounting` package, which is
not available; it is out of scope.
"""
import abc
import collections
import dataclasses
import logging
from typing import List, Optional

from pipelinedp_amd import aggregate_params as agg


@dataclasses.dataclass
class MechanismSpec:
    """A lazily-resolved mechanism budget (budget_accounting.py:40-111)."""
    mechanism_type: agg.MechanismType
    _noise_standard_deviation: Optional[float] = None
    _eps: Optional[float] = None
    _delta: Optional[float] = None
    _count: int = 1

    @property
    def noise_standard_deviation(self) -> float:
        if self._noise_standard_deviation is None:
            raise AssertionError("Noise standard deviation is not calculated yet.")
        return self._noise_standard_deviation

    @property
    def eps(self) -> float:
        if self._eps is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._eps

    @property
    def delta(self) -> float:
        if self._delta is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._delta

    @property
    def count(self) -> int:
        return self._count

    def set_eps_delta(self, eps: float, delta: Optional[float]) -> None:
        if eps is None:
            raise AssertionError("eps must not be None.")
        self._eps = eps
        self._delta = delta

    def set_noise_standard_deviation(self, stddev: float) -> None:
        self._noise_standard_deviation = stddev

    def use_delta(self) -> bool:
        return self.mechanism_type != agg.MechanismType.LAPLACE

    @property
    def standard_deviation_is_set(self) -> bool:
        return self._noise_standard_deviation is not None


@dataclasses.dataclass
class MechanismSpecInternal:
    sensitivity: float
    weight: float
    mechanism_spec: MechanismSpec


Budget = collections.namedtuple("Budget", ["epsilon", "delta"])


class BudgetAccountantScope:
    """`with accountant.scope(weight):` -- mechanisms requested inside share
    `weight` of the parent's budget."""

    def __init__(self, accountant: "BudgetAccountant", weight: float):
        self.accountant = accountant
        self.weight = weight
        self.mechanisms: List[MechanismSpecInternal] = []

    def __enter__(self):
        self.accountant._enter_scope(self)
        return self

    def __exit__(self, exc_type, exc, tb):
        self.accountant._exit_scope()
        if self.mechanisms:
            total = sum(m.weight for m in self.mechanisms)
            factor = self.weight / total
            for m in self.mechanisms:
                m.weight *= factor


class BudgetAccountant(abc.ABC):
    """Base accountant (budget_accounting.py:125-270)."""

    def __init__(self, total_epsilon: float, total_delta: float,
                 num_aggregations: Optional[int],
                 aggregation_weights: Optional[list]):
        agg.validate_epsilon_delta(total_epsilon, total_delta, "BudgetAccountant")
        if num_aggregations is not None and aggregation_weights is not None:
            raise ValueError(
                "'num_aggregations' and 'aggregation_weights' can not be set "
                "simultaneously.")
        if num_aggregations is not None and num_aggregations <= 0:
            raise ValueError(f"'num_aggregations'={num_aggregations}, but it has "
                             f"to be positive.")
        self._total_epsilon = total_epsilon
        self._total_delta = total_delta
        self._scopes_stack: List[BudgetAccountantScope] = []
        self._mechanisms: List[MechanismSpecInternal] = []
        self._finalized = False
        self._expected_num_aggregations = num_aggregations
        self._expected_aggregation_weights = aggregation_weights
        self._actual_aggregation_weights: List[float] = []

    @abc.abstractmethod
    def request_budget(self, mechanism_type: agg.MechanismType,
                       sensitivity: float = 1, weight: float = 1, count: int = 1,
                       noise_standard_deviation: Optional[float] = None
                       ) -> MechanismSpec:
        """Returns a lazy MechanismSpec."""

    @abc.abstractmethod
    def compute_budgets(self):
        """Resolves every requested MechanismSpec."""

    def scope(self, weight: float) -> BudgetAccountantScope:
        return BudgetAccountantScope(self, weight)

    def _compute_budget_for_aggregation(self, weight: float) -> Optional[Budget]:
        self._actual_aggregation_weights.append(weight)
        if self._expected_num_aggregations:
            k = self._expected_num_aggregations
            return Budget(self._total_epsilon / k, self._total_delta / k)
        if self._expected_aggregation_weights:
            share = weight / sum(self._expected_aggregation_weights)
            return Budget(self._total_epsilon * share, self._total_delta * share)
        return None

    def _check_aggregation_restrictions(self):
        actual = self._actual_aggregation_weights
        if self._expected_num_aggregations:
            if len(actual) != self._expected_num_aggregations:
                raise ValueError(
                    f"'num_aggregations'({self._expected_num_aggregations}) in "
                    f"the constructor of BudgetAccountant is different from the"
                    f" actual number of aggregations in the pipeline"
                    f"({len(actual)}).")
            if any(w != 1 for w in actual):
                raise ValueError(
                    f"Aggregation weights = {actual}. If 'num_aggregations' is "
                    f"set in the constructor of BudgetAccountant, all "
                    f"aggregation weights have to be 1.")
        expected = self._expected_aggregation_weights
        if expected:
            if len(actual) != len(expected):
                raise ValueError(
                    f"Length of 'aggregation_weights' in the constructor of "
                    f"BudgetAccountant is {len(expected)} != {len(actual)} the "
                    f"actual number of aggregations.")
            if any(a != e for a, e in zip(actual, expected)):
                raise ValueError(
                    f"'aggregation_weights' in the constructor ({expected}) is "
                    f"different from actual aggregation weights ({actual}).")

    def _register_mechanism(self, m: MechanismSpecInternal) -> MechanismSpecInternal:
        self._mechanisms.append(m)
        for scope in self._scopes_stack:
            scope.mechanisms.append(m)
        return m

    def _enter_scope(self, scope: BudgetAccountantScope):
        self._scopes_stack.append(scope)

    def _exit_scope(self):
        self._scopes_stack.pop()

    def _finalize(self):
        if self._finalized:
            raise Exception("compute_budgets can not be called twice.")
        self._finalized = True


class NaiveBudgetAccountant(BudgetAccountant):
    """Naive composition (budget_accounting.py:301-408)."""

    def __init__(self, total_epsilon: float, total_delta: float,
                 num_aggregations: Optional[int] = None,
                 aggregation_weights: Optional[list] = None):
        super().__init__(total_epsilon, total_delta, num_aggregations,
                         aggregation_weights)

    def request_budget(self, mechanism_type: agg.MechanismType,
                       sensitivity: float = 1, weight: float = 1, count: int = 1,
                       noise_standard_deviation: Optional[float] = None
                       ) -> MechanismSpec:
        if self._finalized:
            raise Exception(
                "request_budget() is called after compute_budgets(). Please "
                "ensure that compute_budgets() is called after DP aggregations.")
        if noise_standard_deviation is not None:
            raise NotImplementedError(
                "Count and noise standard deviation have not been implemented yet.")
        if (mechanism_type == agg.MechanismType.GAUSSIAN and
                self._total_delta == 0):
            raise ValueError("The Gaussian mechanism requires that the pipeline "
                             "delta is greater than 0")
        spec = MechanismSpec(mechanism_type=mechanism_type, _count=count)
        self._register_mechanism(
            MechanismSpecInternal(sensitivity=sensitivity, weight=weight,
                                  mechanism_spec=spec))
        return spec

    def compute_budgets(self):
        self._check_aggregation_restrictions()
        self._finalize()
        if not self._mechanisms:
            logging.warning("No budgets were requested.")
            return
        if self._scopes_stack:
            raise Exception("Cannot call compute_budgets from within a budget scope.")
        w_eps = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms)
        w_delta = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms
                      if m.mechanism_spec.use_delta())
        for m in self._mechanisms:
            eps = self._total_epsilon * m.weight / w_eps if w_eps else 0
            delta = 0
            if m.mechanism_spec.use_delta() and w_delta:
                delta = self._total_delta * m.weight / w_delta
            m.mechanism_spec.set_eps_delta(eps, delta)


class PLDBudgetAccountant(BudgetAccountant):
    """Out of scope: needs the unavailable `dp_accounting` package."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError(
            "PLDBudgetAccountant needs the dp_accounting package, which is not "
            "available in this build; use NaiveBudgetAccountant.")

    def request_budget(self, *a, **k):  # pragma: no cover
        raise NotImplementedError

    def compute_budgets(self):  # pragma: no cover
        raise NotImplementedError
