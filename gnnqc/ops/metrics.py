"""Score histograms for threshold sweeps / AUC."""
from __future__ import annotations

import torch


def score_histogram(scores: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor | None = None,
                    bins: int = 1001) -> torch.Tensor:
    """[2, bins] counts (row 0 negatives, row 1 positives); bin = rint(p*(bins-1))."""
    from . import use_hip
    s = scores.reshape(-1).float().contiguous()
    y = labels.reshape(-1).float().contiguous()
    m = mask.reshape(-1).float().contiguous() if mask is not None else None
    if use_hip(s):
        from ..utils.native import hip_ops
        return hip_ops().score_histogram(s, y, m if m is not None else s.new_zeros(0), int(bins))
    b = torch.round(s.clamp(0, 1) * (bins - 1)).long().clamp(0, bins - 1)
    w = m if m is not None else torch.ones_like(s)
    pos = (y > 0.5).long()
    out = torch.zeros(2 * bins, dtype=torch.float32, device=s.device)
    out.index_add_(0, pos * bins + b, w)
    return out.view(2, bins)


__all__ = ["score_histogram"]
