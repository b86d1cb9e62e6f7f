"""Fused classifier head + weighted BCE (+ metric accumulation).

``Dense(F,64) -> LeakyReLU -> Dense(64,64) -> LeakyReLU -> Dense(64,1)`` followed by
the class-weighted, SUM_OVER_BATCH_SIZE binary cross-entropy of
:func:`gnnqc.train.loss.weighted_bce_with_logits`. On the GPU this is one HIP
forward kernel (which also adds the step's loss sum, confusion counts and score
histogram into the device metric accumulators) and one backward kernel that
writes every head gradient straight into the optimiser's flat gradient buffer
(:func:`gnnqc.ops.lstm.direct_grad_accumulation`). Elsewhere it is plain PyTorch.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .lstm import _grad_sink


def head_eager(feat, W1, b1, W2, b2, W3, b3, alpha1: float, alpha2: float) -> torch.Tensor:
    a1 = F.leaky_relu(feat @ W1 + b1, alpha1)
    a2 = F.leaky_relu(a1 @ W2 + b2, alpha2)
    return (a2 @ W3 + b3).squeeze(-1)


class _HipHeadLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, W1, b1, W2, b2, W3, b3, y, mask, alpha1, alpha2, w0, w1, sums, hist):
        from ..utils.native import hip_ops
        ops = hip_ops()
        empty = feat.new_zeros(0)
        z1, z2, logits, aux = ops.head_fwd(feat, W1.contiguous(), b1.contiguous(), W2.contiguous(), b2.contiguous(),
                                           W3.contiguous(), b3.contiguous(), y, mask, alpha1, alpha2, w0, w1,
                                           sums if sums is not None else empty.double(),
                                           hist if hist is not None else empty)
        ctx.save_for_backward(feat, W1, W2, W3, z1, z2, logits, y, mask, aux)
        ctx.params = (W1, b1, W2, b2, W3, b3)
        ctx.consts = (alpha1, alpha2, w0, w1)
        ctx.mark_non_differentiable(logits)
        return aux[0], logits

    @staticmethod
    def backward(ctx, gloss, _glogits):
        from ..utils.native import hip_ops
        ops = hip_ops()
        feat, W1, W2, W3, z1, z2, logits, y, mask, aux = ctx.saved_tensors
        a1, a2, w0, w1 = ctx.consts
        sinks = [_grad_sink(p) for p in ctx.params]
        g = gloss.reshape(1).float().contiguous()
        need_dfeat = bool(ctx.needs_input_grad[0])
        dfeat = ops.head_bwd(feat, W1.contiguous(), W2.contiguous(), W3.contiguous(), z1, z2, logits, y, mask,
                             a1, a2, w0, w1, g, aux, *[s[0] for s in sinks], need_dfeat)
        grads = []
        for (buf, direct), need in zip(sinks, ctx.needs_input_grad[1:7]):
            grads.append(None if direct or not need else buf)
        return (dfeat if need_dfeat else None, *grads, None, None, None, None, None, None, None, None)


def fused_head_loss(feat: torch.Tensor, dense, dense2, dense_out, alpha1: float, alpha2: float, y: torch.Tensor,
                    mask: torch.Tensor, w0: float, w1: float, sums: Optional[torch.Tensor] = None,
                    hist: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(loss, logits) for rows ``feat`` [R, F]; ``sums``/``hist`` (optional) are the
    :class:`~gnnqc.train.engine.MetricAccumulator` buffers, updated in place on GPU."""
    from . import use_hip
    R, Fdim = feat.shape
    y = y.reshape(-1).float().contiguous()
    mask = mask.reshape(-1).float().contiguous()
    ok = (use_hip(feat) and Fdim in (32, 64, 128) and dense.kernel.shape[1] == 64 and dense2.kernel.shape == (64, 64)
          and dense_out.kernel.shape == (64, 1))
    if ok:
        f = feat.float()
        if not (f.stride(1) == 1 and f.stride(0) % 4 == 0 and f.data_ptr() % 16 == 0):
            f = f.contiguous()
        return _HipHeadLoss.apply(f, dense.kernel, dense.bias, dense2.kernel, dense2.bias, dense_out.kernel,
                                  dense_out.bias, y, mask, float(alpha1), float(alpha2), float(w0), float(w1), sums,
                                  hist)
    from ..train.loss import weighted_bce_with_logits
    z = head_eager(feat.float(), dense.kernel, dense.bias, dense2.kernel, dense2.bias, dense_out.kernel,
                   dense_out.bias, alpha1, alpha2)
    loss = weighted_bce_with_logits(z, y, mask, w0, w1)
    if sums is not None:
        from ..train.engine import MetricAccumulator
        MetricAccumulator.update_buffers(sums, hist, loss, z, y, mask)
    return loss, z


__all__ = ["fused_head_loss", "head_eager"]
