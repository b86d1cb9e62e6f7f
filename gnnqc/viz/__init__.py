"""Visualisation: evaluation plots and integrated-gradients figures (matplotlib, Agg)."""
from .results import extract_target_info, plot_classified_samples, plot_results, plot_roc_curves, timeseries_figure

__all__ = ["plot_roc_curves", "extract_target_info", "timeseries_figure", "plot_classified_samples",
           "plot_results"]
