"""Loads the reference fixtures of tests/golden (see tests/golden/gen_golden.py)."""
import json
import os

import numpy as np

import pipelinedp_amd as pdp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_METRICS = {"COUNT": pdp.Metrics.COUNT, "SUM": pdp.Metrics.SUM,
            "PRIVACY_ID_COUNT": pdp.Metrics.PRIVACY_ID_COUNT, "MEAN": pdp.Metrics.MEAN,
            "VARIANCE": pdp.Metrics.VARIANCE}


def cases():
    with open(os.path.join(GOLDEN, "aggregate_cases.json")) as f:
        return json.load(f)


def params_of(meta):
    kw = dict(meta["params"])
    kw["metrics"] = [_METRICS[m] for m in kw["metrics"]]
    if "noise_kind" in kw:
        kw["noise_kind"] = pdp.NoiseKind[kw["noise_kind"]]
    return pdp.AggregateParams(**kw)


def load(meta):
    d = np.load(os.path.join(GOLDEN, f"agg_{meta['name']}.npz"))
    return {k: d[k] for k in d.files}


def tolerance_ok(field, got, want):
    """counts exact; float64 results within 1e-9 relative (north star)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    if field in ("count", "privacy_id_count"):
        return np.array_equal(got, want)
    return np.allclose(got, want, rtol=1e-9, atol=1e-9)
