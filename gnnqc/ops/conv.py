"""Conv1D(padding='same') + LeakyReLU (+ GlobalAveragePooling1D) - the CNN TimeLayer branch
(reference ``libs/create_model.py:80-101``).

GPU: ``conv1d.hip`` - implicit-GEMM MFMA forward with bias, LeakyReLU and (for the last
layer) the time mean fused into the epilogue; the backward forms ``dz = dy * leaky'(y)``
inside its loads, accumulates dW/db straight into the optimiser's flat gradient
buffer (direct mode) and computes dx with the same forward kernel on flipped weights.
Elsewhere: ``F.conv1d`` + ``leaky_relu`` (+ ``mean``), the fp32 numerics oracle.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .lstm import _grad_sink


def conv1d_act_eager(x, W, b, alpha: float, gap: bool = False):
    """x [M,T,Cin], W [k,Cin,Cout] (Keras layout), b [Cout] -> leaky(conv_same(x)) [M,T,Cout] (or its time mean)."""
    k = W.shape[0]
    left = (k - 1) // 2
    xt = F.pad(x.transpose(1, 2), (left, k - 1 - left))
    y = F.conv1d(xt, W.permute(2, 1, 0), b).transpose(1, 2)
    if alpha != 1.0:
        y = F.leaky_relu(y, alpha)
    return y.mean(1) if gap else y


class _HipConv1dAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, alpha: float, gap: bool):
        from ..utils.native import hip_ops
        x = x.contiguous()
        need = any(ctx.needs_input_grad[:3])
        y, g = hip_ops().conv1d_fwd(x, W.contiguous(), b.contiguous(), float(alpha), bool(gap), need or not gap)
        ctx.alpha, ctx.gap, ctx.params = float(alpha), bool(gap), (W, b)
        if need:
            ctx.save_for_backward(x, W, y)
        return g if gap else y

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        x, W, y = ctx.saved_tensors
        need = ctx.needs_input_grad
        wgrad = any(need[1:3])
        if wgrad:
            sinks = [_grad_sink(p) for p in ctx.params]
        else:
            e = x.new_zeros(0)
            sinks = [(e, True)] * 2
        dx = hip_ops().conv1d_bwd(dout.contiguous(), y, x, W.contiguous(), ctx.alpha, ctx.gap,
                                  sinks[0][0], sinks[1][0], bool(need[0]))
        grads = [None if (direct or not n) else buf for (buf, direct), n in zip(sinks, need[1:3])]
        return (dx if need[0] else None, *grads, None, None)


def hip_conv_supported(k: int, cin: int, cout: int) -> bool:
    """Shapes the HIP kernels take (``conv1d_supported`` in conv1d.hip): channels <= 128 and
    the weight-gradient im2col tile k*Cin + 1 within 24 column tiles of 16."""
    return 1 <= k and 1 <= cin <= 128 and 1 <= cout <= 128 and (k * cin + 1 + 15) // 16 <= 24


def conv1d_act(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, alpha: float = 1.0, gap: bool = False):
    """Fused Conv1D(same) + LeakyReLU(alpha) (+ GAP). ``alpha=1`` is the identity."""
    from . import use_hip
    k, cin, cout = W.shape
    if use_hip(x) and x.dtype == torch.float32 and hip_conv_supported(k, cin, cout) and x.shape[1] > 0:
        return _HipConv1dAct.apply(x, W, b, float(alpha), bool(gap))
    return conv1d_act_eager(x, W, b, alpha, gap)


__all__ = ["conv1d_act", "conv1d_act_eager", "hip_conv_supported"]
