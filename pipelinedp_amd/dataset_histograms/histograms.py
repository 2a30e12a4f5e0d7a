"""Histogram data types (API mirror of
pipeline_dp/dataset_histograms/histograms.py).

FrequencyBin :21-57, HistogramType :60-75, Histogram :78-158,
compute_ratio_dropped :161-200, DatasetHistograms :203-211.  These are host
containers for the few thousand bins the device histograms produce
(csrc/dpg_hist.h); nothing here touches per-record data.
"""
import dataclasses
import enum
from typing import List, Optional, Sequence, Tuple, Union

Number = Union[int, float]


@dataclasses.dataclass
class FrequencyBin:
    """Values in [lower, upper) (the last bin of a float histogram includes
    its upper): how many (`count`), their total (`sum`) and largest (`max`)."""
    lower: Number
    upper: Number
    count: int
    sum: Number
    max: Number

    def __add__(self, other: "FrequencyBin") -> "FrequencyBin":
        assert (self.lower, self.upper) == (other.lower, other.upper)
        return FrequencyBin(self.lower, self.upper, self.count + other.count,
                            self.sum + other.sum, max(self.max, other.max))

    def __eq__(self, other) -> bool:
        # the upper is implied by the lower (histograms.py:51-53)
        return (self.lower, self.count, self.sum, self.max) == (other.lower, other.count,
                                                                 other.sum, other.max)


class HistogramType(enum.Enum):
    L0_CONTRIBUTIONS = "l0_contributions"
    L1_CONTRIBUTIONS = "l1_contributions"
    LINF_CONTRIBUTIONS = "linf_contributions"
    LINF_SUM_CONTRIBUTIONS = "linf_sum_contributions"
    COUNT_PER_PARTITION = "count_per_partition"
    COUNT_PRIVACY_ID_PER_PARTITION = "privacy_id_per_partition_count"


@dataclasses.dataclass
class Histogram:
    """Bins sorted by lower.  Integer histograms (all but LINF_SUM) start at
    1 and have no upper; the float one spans [first lower, last upper]."""
    name: HistogramType
    bins: List[FrequencyBin]
    lower: Optional[Number] = dataclasses.field(init=False)
    upper: Optional[Number] = dataclasses.field(init=False)

    def __post_init__(self):
        if not self.bins:
            self.lower = self.upper = None
        elif self.is_integer:
            self.lower, self.upper = 1, None
        else:
            self.lower, self.upper = self.bins[0].lower, self.bins[-1].upper

    @property
    def is_integer(self) -> bool:
        return self.name != HistogramType.LINF_SUM_CONTRIBUTIONS

    def total_count(self):
        return sum(b.count for b in self.bins)

    def total_sum(self):
        return sum(b.sum for b in self.bins)

    def max_value(self):
        return self.bins[-1].max

    def quantiles(self, q: List[float]) -> List[Number]:
        """For each q (ascending), the lower of the first bin such that the
        bins left of it hold at most a q fraction of the elements."""
        assert sorted(q) == q, "Quantiles to compute must be sorted."
        total = self.total_count()
        if total == 0:
            raise ValueError("Cannot compute quantiles of an empty histogram")
        out = []
        smaller = total
        i = len(q) - 1
        for b in reversed(self.bins):
            smaller -= b.count
            while i >= 0 and q[i] >= smaller / total:
                out.append(b.lower)
                i -= 1
        while i >= 0:  # only reachable for q < 0
            out.append(self.bins[0].lower)
            i -= 1
        return out[::-1]


def compute_ratio_dropped(contribution_histogram: Histogram) -> Sequence[Tuple[Number, float]]:
    """(threshold, fraction of the histogram's total sum dropped by bounding
    at that threshold) for every bin lower and the max value, plus (0, 1);
    sorted by threshold."""
    bins = contribution_histogram.bins
    if not bins:
        return []
    total = contribution_histogram.total_sum()
    out = []
    prev = bins[-1].lower
    if contribution_histogram.max_value() != prev:
        out.append((contribution_histogram.max_value(), 0.0))
    dropped = larger = 0
    for b in reversed(bins):
        cur = b.lower
        dropped += larger * (prev - cur) + (b.sum - b.count * cur)
        out.append((cur, dropped / total))
        prev = cur
        larger += b.count
    out.append((0, 1))
    return out[::-1]


@dataclasses.dataclass
class DatasetHistograms:
    """The histograms parameter tuning works from."""
    l0_contributions_histogram: Histogram
    l1_contributions_histogram: Histogram
    linf_contributions_histogram: Histogram
    linf_sum_contributions_histogram: Histogram
    count_per_partition_histogram: Histogram
    count_privacy_id_per_partition: Histogram
