"""Visualisation: evaluation plots and integrated-gradients figures (matplotlib, Agg)."""
from .results import (classified_timeseries_figure, classified_timeseries_figure_with_neighbours, extract_target_info,
                      plot_classified_samples, plot_classified_timeseries, plot_classified_timeseries_with_neighbours,
                      plot_results, plot_roc_curves, timeseries_figure)

__all__ = ["plot_roc_curves", "extract_target_info", "timeseries_figure", "plot_classified_samples",
           "plot_results", "classified_timeseries_figure", "plot_classified_timeseries",
           "classified_timeseries_figure_with_neighbours", "plot_classified_timeseries_with_neighbours"]
