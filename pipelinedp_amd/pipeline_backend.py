"""Pipeline backends: the plug-in point (mirror of pipeline_dp/pipeline_backend.py).

`PipelineBackend` keeps the reference's abstract interface
(pipeline_backend.py:38-195) so code written against it type-checks here.
`MI355XBackend` is the only backend in this package.  `DPEngine.aggregate` /
`select_partitions` detect it and return a lazy `DeviceAggregation`
(device_aggregate.py) instead of building the reference's graph of generic
ops; the generic ops
are implemented with plain Python generators (LocalBackend semantics,
pipeline_backend.py:477-583) for user-side collection plumbing only -- the
DP aggregation never runs through them.
"""
import abc
import collections
import functools
import itertools
import os
import random
import typing
from typing import Any, Callable, Iterable, List, Optional

import numpy as np
import torch

from pipelinedp_amd import _native
from pipelinedp_amd import columnar


class PipelineBackend(abc.ABC):
    """Interface of PipelineDP's execution backends."""

    def to_collection(self, collection_or_iterable, col, stage_name: str):
        return collection_or_iterable

    def to_multi_transformable_collection(self, col):
        return col

    @abc.abstractmethod
    def map(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_with_side_inputs(self, col, fn, side_input_cols, stage_name: str):
        pass

    @abc.abstractmethod
    def flat_map(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_tuple(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def map_values(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def group_by_key(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def filter(self, col, fn, stage_name: str):
        pass

    @abc.abstractmethod
    def filter_by_key(self, col, keys_to_keep, stage_name: str):
        pass

    @abc.abstractmethod
    def keys(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def values(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def sample_fixed_per_key(self, col, n: int, stage_name: str):
        pass

    @abc.abstractmethod
    def count_per_element(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def sum_per_key(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def combine_accumulators_per_key(self, col, combiner, stage_name: str):
        pass

    @abc.abstractmethod
    def reduce_per_key(self, col, fn: Callable, stage_name: str):
        pass

    @abc.abstractmethod
    def flatten(self, cols: Iterable, stage_name: str):
        pass

    @abc.abstractmethod
    def distinct(self, col, stage_name: str):
        pass

    @abc.abstractmethod
    def to_list(self, col, stage_name: str):
        pass

    def annotate(self, col, stage_name: str, **kwargs):
        return col


class Annotator(abc.ABC):
    """pipeline_backend.py:826-851: user hooks called on every DP result."""

    @abc.abstractmethod
    def annotate(self, col, backend: PipelineBackend, stage_name: str, **kwargs):
        pass


_annotators: List[Annotator] = []


def register_annotator(annotator: Annotator):
    _annotators.append(annotator)


class _HostCollectionOps:
    """Generic collection operations (LocalBackend semantics), host only."""

    def to_multi_transformable_collection(self, col):
        return list(col)

    def map(self, col, fn, stage_name=None):
        return map(fn, col)

    def map_with_side_inputs(self, col, fn, side_input_cols, stage_name=None):
        side = [list(c) for c in side_input_cols]
        return (fn(x, *side) for x in col)

    def flat_map(self, col, fn, stage_name=None):
        return (y for x in col for y in fn(x))

    def map_tuple(self, col, fn, stage_name=None):
        return (fn(*x) for x in col)

    def map_values(self, col, fn, stage_name=None):
        return ((k, fn(v)) for k, v in col)

    def group_by_key(self, col, stage_name=None):
        def gen():
            groups = collections.defaultdict(list)
            for k, v in col:
                groups[k].append(v)
            yield from groups.items()
        return gen()

    def filter(self, col, fn, stage_name=None):
        return filter(fn, col)

    def filter_by_key(self, col, keys_to_keep, stage_name=None):
        keep = keys_to_keep if isinstance(keys_to_keep, (set, frozenset, dict)) else set(keys_to_keep)
        return (kv for kv in col if kv[0] in keep)

    def keys(self, col, stage_name=None):
        return (k for k, _ in col)

    def values(self, col, stage_name=None):
        return (v for _, v in col)

    def sample_fixed_per_key(self, col, n, stage_name=None):
        def gen():
            for k, vs in self.group_by_key(col):
                if len(vs) > n:
                    idx = np.random.choice(len(vs), n, replace=False)
                    vs = [vs[i] for i in idx]
                yield k, vs
        return gen()

    def count_per_element(self, col, stage_name=None):
        yield from collections.Counter(col).items()

    def sum_per_key(self, col, stage_name=None):
        return self.map_values(self.group_by_key(col), sum)

    def combine_accumulators_per_key(self, col, combiner, stage_name=None):
        return self.map_values(
            self.group_by_key(col),
            lambda accs: functools.reduce(combiner.merge_accumulators, accs))

    def reduce_per_key(self, col, fn, stage_name=None):
        return self.map_values(self.group_by_key(col),
                               lambda vs: functools.reduce(fn, vs))

    def flatten(self, cols, stage_name=None):
        return itertools.chain(*cols)

    def distinct(self, col, stage_name=None):
        return iter(set(col))

    def to_list(self, col, stage_name=None):
        return iter([list(col)])


class MI355XBackend(_HostCollectionOps, PipelineBackend):
    """Runs DPEngine.aggregate / select_partitions on one MI355X GPU.

    Args:
      device: GPU ordinal (defaults to LOCAL_RANK or 0).
      seed: 64-bit seed of every keyed random stream (sampling, selection,
        noise).  Default: fresh randomness from os.urandom -- a fixed seed
        makes the noise reproducible, which is only acceptable in tests.
      process_group: torch.distributed group for multi-GPU aggregation
        (records must be sharded by privacy id); None = single GPU.
      exchange: how the ranks merge their per-partition partials
        (distributed.py): 'auto' (from P, the accumulator arrays and the
        occupancy bound min(P, records, privacy ids x l0) -- no device
        data, no host synchronisation), 'reduce_scatter' (dense) or
        'all_to_all' (fixed blocks of the occupied partitions' rows).
        Partition pk is owned by rank pk mod world_size.
    """

    def __init__(self, device: Optional[int] = None, seed: Optional[int] = None,
                 process_group=None, exchange: str = "auto"):
        if exchange not in ("auto", "reduce_scatter", "all_to_all"):
            raise ValueError(f"unknown exchange {exchange!r}")
        self.exchange = exchange
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", 0))
        self.device_index = device
        self.device = torch.device("cuda", device)
        self.seed = int.from_bytes(os.urandom(8), "little") if seed is None else int(seed)
        self.process_group = process_group
        self._ctx = None

    @property
    def ctx(self) -> _native.Context:
        if self._ctx is None:
            if not torch.cuda.is_available():
                raise _native.NativeError(
                    "MI355XBackend needs a ROCm GPU; there is no CPU fallback.")
            self._ctx = _native.Context(self.device_index, self.seed)
        return self._ctx

    def annotate(self, col, stage_name: str, **kwargs):
        for a in _annotators:
            col = a.annotate(col, self, stage_name, **kwargs)
        return col

    @property
    def world_size(self) -> int:
        if self.process_group is None:
            return 1
        return torch.distributed.get_world_size(self.process_group)
