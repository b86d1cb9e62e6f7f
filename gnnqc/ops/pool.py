"""MaxPooling1D (valid padding, stride = pool size) - TimeLayer pooling.

GPU: ``maxpool1d_fwd`` keeps a byte argmax per output, ``maxpool1d_bwd`` routes
the gradient to it (one pass each). Elsewhere ``max(dim)``, whose gradient also
goes to a single position per window like TF's ``MaxPoolGrad``.
"""
from __future__ import annotations

import torch


class _HipMaxPool1d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p: int):
        from ..utils.native import hip_ops
        y, idx = hip_ops().maxpool1d_fwd(x, p)
        ctx.save_for_backward(idx)
        ctx.T, ctx.p = x.shape[1], p
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..utils.native import hip_ops
        (idx,) = ctx.saved_tensors
        return hip_ops().maxpool1d_bwd(dy.contiguous(), idx, ctx.T, ctx.p), None


def max_pool1d(x: torch.Tensor, p: int) -> torch.Tensor:
    from . import use_hip
    M, T, C = x.shape
    if use_hip(x) and x.dtype == torch.float32 and C % 4 == 0 and 1 <= p <= 255:
        return _HipMaxPool1d.apply(x.contiguous(), int(p))
    To = T // p
    return x[:, :To * p].reshape(M, To, p, C).max(2).values


def max_pool1d_tm(x_tm: torch.Tensor, p: int) -> torch.Tensor:
    """Time-major pooling: [T, Mp, C] -> [T // p, Mp, C] (pool along the leading time axis)."""
    T, Mp, C = x_tm.shape
    y = max_pool1d(x_tm.contiguous().view(1, T, Mp * C), p)
    return y.view(T // p, Mp, C)


__all__ = ["max_pool1d", "max_pool1d_tm"]
