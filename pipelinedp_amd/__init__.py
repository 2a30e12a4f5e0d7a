"""pipelinedp_amd -- MI355X-native DPEngine.aggregate for PipelineDP users.

Drop-in names of the reference package (pipeline_dp/__init__.py) for the
hot path: AggregateParams & friends, NaiveBudgetAccountant, DataExtractors,
DPEngine and ExplainComputationReport, plus `MI355XBackend` (the execution
backend) and `ColumnarData` (columnar input).  Device compute lives in the
HIP library pipelinedp_amd/lib/libdpg.so (C ABI: include/dpg.h).
"""
from pipelinedp_amd.aggregate_params import AggregateParams
from pipelinedp_amd.aggregate_params import CalculatePrivateContributionBoundsParams
from pipelinedp_amd.aggregate_params import CountParams
from pipelinedp_amd.aggregate_params import MechanismType
from pipelinedp_amd.aggregate_params import Metric
from pipelinedp_amd.aggregate_params import Metrics
from pipelinedp_amd.aggregate_params import NoiseKind
from pipelinedp_amd.aggregate_params import NormKind
from pipelinedp_amd.aggregate_params import PartitionSelectionStrategy
from pipelinedp_amd.aggregate_params import PrivacyIdCountParams
from pipelinedp_amd.aggregate_params import PrivateContributionBounds
from pipelinedp_amd.aggregate_params import SelectPartitionsParams
from pipelinedp_amd.aggregate_params import SumParams
from pipelinedp_amd.budget_accounting import BudgetAccountant
from pipelinedp_amd.budget_accounting import MechanismSpec
from pipelinedp_amd.budget_accounting import NaiveBudgetAccountant
from pipelinedp_amd.budget_accounting import PLDBudgetAccountant
from pipelinedp_amd.columnar import ColumnarData
from pipelinedp_amd.data_extractors import DataExtractors
from pipelinedp_amd.data_extractors import PreAggregateExtractors
from pipelinedp_amd.dp_engine import DPEngine
from pipelinedp_amd.pipeline_backend import Annotator
from pipelinedp_amd.pipeline_backend import MI355XBackend
from pipelinedp_amd.pipeline_backend import PipelineBackend
from pipelinedp_amd.pipeline_backend import register_annotator
from pipelinedp_amd.report_generator import ExplainComputationReport
from pipelinedp_amd import dataset_histograms

__version__ = "0.1.0"
