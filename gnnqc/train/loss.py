"""Weighted binary cross-entropy.

Keras ``binary_crossentropy`` on a sigmoid output recovers the logits in graph
mode, i.e. it is the stable BCE-with-logits; ``class_weight`` turns into per-sample
weights ``w_y`` and the reduction is SUM_OVER_BATCH_SIZE (``sum(w*l) / n``), with
``n`` the number of (valid) samples, not ``sum(w)`` (``libs/fit_model.py:104-111``).
Class weights: ``calculate_weights`` (``libs/fit_model.py:8-25``).
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F


def weighted_bce_with_logits(logits: torch.Tensor, y: torch.Tensor, mask: torch.Tensor,
                             w0: float = 1.0, w1: float = 1.0) -> torch.Tensor:
    per = F.binary_cross_entropy_with_logits(logits, y, reduction="none")
    w = torch.where(y > 0.5, torch.full_like(y, w1), torch.full_like(y, w0)) * mask
    return (per * w).sum() / mask.sum().clamp(min=1.0)


def calculate_weights(model_config, labels: Optional[np.ndarray] = None) -> Optional[Dict[int, float]]:
    wc = model_config.get("weight_classes") if hasattr(model_config, "get") else None
    if not wc or not wc.get("use", False):
        return None
    if wc.get("calculate", False):
        if labels is None:
            raise ValueError("calculate=True needs the training labels")
        y = np.asarray(labels).ravel()
        n, a = float(y.size), float(y.sum())
        return {0: n / (n - a), 1: 2 * n / a}
    c0, c1 = wc.get("class_0"), wc.get("class_1")
    if c0 is not None and c1 is not None:
        return {0: float(c0), 1: float(c1)}
    return {0: 1.0, 1: 5.0}


__all__ = ["weighted_bce_with_logits", "calculate_weights"]
