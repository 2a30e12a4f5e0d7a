"""Data extractors (API mirror of pipeline_dp/data_extractors.py:5-15).

Row-wise callables behave as in the reference.  For columnar input (see
pipelinedp_amd/columnar.py) an extractor may also be a column name (str) or a
callable that maps the whole column container to one column.
"""
import dataclasses
from typing import Callable, Union

Extractor = Union[Callable, str, None]


@dataclasses.dataclass
class DataExtractors:
    privacy_id_extractor: Extractor = None
    partition_extractor: Extractor = None
    value_extractor: Extractor = None


@dataclasses.dataclass
class PreAggregateExtractors:
    partition_extractor: Callable
    preaggregate_extractor: Callable
