"""Dataset contribution histograms (pipeline_dp/dataset_histograms)."""
from pipelinedp_amd.dataset_histograms import computing_histograms
from pipelinedp_amd.dataset_histograms import histograms
