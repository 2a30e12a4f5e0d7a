"""Utility-analysis test helpers: the reference's own known-answer cases
(analysis/tests/utility_analysis_test.py, computed there with the real
PyDP), conversion of product results to plain dicts, and a nested-dict
comparator (the reference compares with an absolute delta of 1e-5,
analysis/tests/common.py:22-80)."""
import dataclasses
import enum
import math

import numpy as np

# utility_analysis_test.py:59-195, not pre-aggregated: 10 privacy ids, each
# contributing 3 times to each of 10 partitions; COUNT + PRIVACY_ID_COUNT,
# Gaussian, mpc 1, mcpp 2, eps 3, delta 0.9
WO_PUBLIC_ROWS = [(i, j) for i in range(10) for j in range(10)] * 3
WO_PUBLIC_EXPECTED = dict(
    configuration_index=0,
    partitions_info=dict(public_partitions=False, num_dataset_partitions=10,
                         strategy="TRUNCATED_GEOMETRIC",
                         kept_partitions=dict(mean=3.51622411, var=2.2798409)),
    metric_errors=[
        dict(metric="COUNT", noise_std=1.380859375,
             ratio_data_dropped=dict(l0=0.6, linf=0.333333333,
                                     partition_selection=0.04322517259988915),
             absolute_error=dict(bounding_errors=dict(l0=dict(mean=-18, var=3.6), linf_min=0.0,
                                                      linf_max=-10),
                                 mean=-28, variance=5.5067726, rmse=28.098163153, l1=0.0,
                                 rmse_with_dropped_partitions=29.331271542782087,
                                 l1_with_dropped_partitions=0.0),
             relative_error=dict(bounding_errors=dict(l0=dict(mean=-0.6, var=0.004),
                                                      linf_min=0.0, linf_max=-0.33333333),
                                 mean=-0.93333333, variance=0.006118636237250433,
                                 rmse=0.9366054384576044, l1=0.0,
                                 rmse_with_dropped_partitions=0.9777090514260699,
                                 l1_with_dropped_partitions=0.0)),
        dict(metric="PRIVACY_ID_COUNT", noise_std=0.6904296875,
             ratio_data_dropped=dict(l0=0.9, linf=0.0, partition_selection=0.06483775889983372),
             absolute_error=dict(bounding_errors=dict(l0=dict(mean=-9, var=0.9), linf_min=0.0,
                                                      linf_max=0.0),
                                 mean=-9, variance=1.37669315, rmse=9.07616070, l1=0.0,
                                 rmse_with_dropped_partitions=9.67515739991,
                                 l1_with_dropped_partitions=0.0),
             relative_error=dict(bounding_errors=dict(l0=dict(mean=-0.9, var=0.009),
                                                      linf_min=0.0, linf_max=0.0),
                                 mean=-0.9, variance=0.013766931533, rmse=0.90761607055726,
                                 l1=0.0, rmse_with_dropped_partitions=0.9675157399915,
                                 l1_with_dropped_partitions=0.0)),
    ])
WO_PUBLIC_BIN = (20, 50)

# utility_analysis_test.py:190-234: public partitions, noise std of COUNT and
# PRIVACY_ID_COUNT (eps 2, delta 1e-10, mpc 1, mcpp 1)
W_PUBLIC_STD = {"GAUSSIAN": 5.9765625, "LAPLACE": 1.4142135623730951}

# utility_analysis_test.py:236-292: two configurations
MULTI_STD = [3.02734375, 8.56262117843085]
MULTI_L0_MEAN = [-0.5, 0]

# utility_analysis_test.py:327-380: partition selection probability
SELECT_PROB = {None: 0.612579511, 3: 0.0644512636}


def to_plain(x):
    """dataclasses / enums / Metric -> nested dicts of plain values."""
    if dataclasses.is_dataclass(x) and type(x).__name__ == "Metric":
        return x.name
    if dataclasses.is_dataclass(x):
        return {f.name: to_plain(getattr(x, f.name)) for f in dataclasses.fields(x)}
    if isinstance(x, enum.Enum):
        return x.name
    if isinstance(x, (list, tuple)):
        return [to_plain(v) for v in x]
    if isinstance(x, dict):
        return {k: to_plain(v) for k, v in x.items()}
    return x


SKIP = {"noise_kind", "aggregation"}


def assert_close(want, got, path="", atol=1e-5, rtol=0.0, skip=SKIP):
    """Nested comparison: keys of `want` only; numbers within
    atol + rtol * |want|; None / strings exact."""
    if isinstance(want, dict):
        assert isinstance(got, dict), f"{path}: {got!r} is not a dict"
        for k, v in want.items():
            if k in skip:
                continue
            assert k in got, f"{path}.{k} missing"
            assert_close(v, got[k], f"{path}.{k}", atol, rtol, skip)
    elif isinstance(want, list):
        assert isinstance(got, list) and len(got) == len(want), f"{path}: length {got!r}"
        for i, (a, b) in enumerate(zip(want, got)):
            assert_close(a, b, f"{path}[{i}]", atol, rtol, skip)
    elif isinstance(want, bool) or want is None or isinstance(want, str):
        assert want == got, f"{path}: want {want!r} got {got!r}"
    else:
        assert got is not None and math.isfinite(float(got)) == math.isfinite(float(want)), \
            f"{path}: {got!r}"
        assert abs(float(got) - float(want)) <= atol + rtol * abs(float(want)), \
            f"{path}: want {want!r} got {got!r}"


def load_fixture():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                        "utility_analysis.json")
    with open(path) as f:
        return json.load(f)


def oracle_configs(case):
    """Configuration dicts of the oracle from a fixture case."""
    cfg = case["configs"]
    n = len(cfg["max_partitions_contributed"])
    out = []
    for i in range(n):
        def get(k, default):
            v = cfg.get(k)
            return v[i] if v else default
        out.append(dict(mpc=get("max_partitions_contributed", None),
                        mcpp=get("max_contributions_per_partition", None),
                        min_sum=get("min_sum_per_partition", -np.inf),
                        max_sum=get("max_sum_per_partition", np.inf),
                        noise_kind=case["noise"],
                        strategy=get("partition_selection_strategy", "TRUNCATED_GEOMETRIC"),
                        pre_threshold=case["pre_threshold"]))
    return out


def sampler(prob):
    """sampling_utils.ValueSampler (the reference's partition sampling)."""
    if prob >= 1:
        return None
    import hashlib
    bound = int(round(2**64 * prob))
    return lambda k: int(hashlib.sha1(repr(k).encode()).hexdigest()[:16], 16) < bound
