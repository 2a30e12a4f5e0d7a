"""Utility analysis on MI355X (API mirror of the reference's `analysis`
package, analysis/__init__.py): perform_utility_analysis evaluates many
contribution-bound configurations in one device pass over the
per-(privacy id, partition) pre-aggregate."""
from pipelinedp_amd.analysis.data_structures import MultiParameterConfiguration
from pipelinedp_amd.analysis.data_structures import UtilityAnalysisOptions
from pipelinedp_amd.analysis import metrics
from pipelinedp_amd.analysis.utility_analysis import perform_utility_analysis
from pipelinedp_amd.analysis.utility_analysis import UtilityAnalysis
from pipelinedp_amd.analysis import parameter_tuning
