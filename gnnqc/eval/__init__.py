"""Evaluation: metrics + the ``test_model`` API."""
from . import metrics
from .test_model import anomaly_index, calculate_metrics, calculate_threshold, select_threshold

__all__ = ["metrics", "select_threshold", "calculate_threshold", "calculate_metrics", "anomaly_index"]
