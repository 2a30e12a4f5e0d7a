"""Explain-computation report (API mirror of pipeline_dp/report_generator.py).

Stages may be strings or zero-argument callables; callables are evaluated
only when the report text is produced, i.e. after compute_budgets(), so a
stage can mention budgets that are unknown at graph-construction time
(report_generator.py:66-89).
"""
from typing import Callable, List, Optional, Union

from pipelinedp_amd import aggregate_params as agg

Stage = Union[str, Callable[[], str]]


class ReportGenerator:

    def __init__(self, params, method_name: str,
                 is_public_partition: Optional[bool] = None):
        self._params_str = (agg.parameters_to_readable_string(
            params, is_public_partition) if params else None)
        self._method_name = method_name
        self._stages: List[Stage] = []

    def add_stage(self, stage_description: Stage) -> None:
        self._stages.append(stage_description)

    def report(self) -> str:
        if not self._params_str:
            return ""
        out = [f"DPEngine method: {self._method_name}", self._params_str,
               "Computation graph:"]
        for i, stage in enumerate(self._stages, 1):
            text = stage() if callable(stage) else stage
            out.append(f" {i}. {text}")
        return "\n".join(out)


class ExplainComputationReport:
    """Output argument of DPEngine.aggregate."""

    def __init__(self):
        self._report_generator: Optional[ReportGenerator] = None

    def _set_report_generator(self, generator: ReportGenerator) -> None:
        self._report_generator = generator

    def text(self) -> str:
        if self._report_generator is None:
            raise ValueError("The report_generator is not set.\nWas this object "
                             "passed as an argument to DP aggregation method?")
        try:
            return self._report_generator.report()
        except Exception as e:  # e.g. budgets not computed yet
            raise ValueError("Explain computation report failed to be generated."
                             "\nWas BudgetAccountant.compute_budget() called?") from e
