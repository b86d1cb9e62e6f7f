"""Keras-semantics LSTM layer.

Gate order i, f, c(g), o; ``z_t = x_t W + h_{t-1} U + b``; recurrent activation
sigmoid; ``activation`` (tanh by default) for g and the cell output; zero initial
state (Keras ``LSTM`` as built by ``libs/create_model.py:61-79``).

GPU path: one library GEMM for the input projection of all T steps, then the
persistent HIP recurrence (``lstm_fwd``); backward = persistent BPTT kernel
(``lstm_bwd``) producing dz for all steps, then the weight/input gradients as
plain GEMMs over all (sequence, step) rows.
"""
from __future__ import annotations

import torch

_ACT = {
    "tanh": torch.tanh,
    "relu": torch.relu,
    "sigmoid": torch.sigmoid,
    "linear": lambda x: x,
    None: lambda x: x,
}


def lstm_eager(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor,
               return_sequences: bool = True, activation: str = "tanh") -> torch.Tensor:
    """Reference implementation: x [M,T,Din], W [Din,4H], U [H,4H], b [4H]."""
    act = _ACT[activation]
    M, T, _ = x.shape
    H = U.shape[0]
    xp = torch.matmul(x, W) + b
    h = x.new_zeros(M, H)
    c = x.new_zeros(M, H)
    outs = []
    for t in range(T):
        z = xp[:, t] + h @ U
        i, f, g, o = z.split(H, dim=-1)
        i, f, o = torch.sigmoid(i), torch.sigmoid(f), torch.sigmoid(o)
        c = f * c + i * act(g)
        h = o * act(c)
        if return_sequences:
            outs.append(h)
    return torch.stack(outs, 1) if return_sequences else h


class _HipLSTM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, U, b, bf16: bool, return_sequences: bool):
        from ..utils.native import hip_ops
        ops = hip_ops()
        M, T, Din = x.shape
        H = U.shape[0]
        x = x.contiguous()
        xp = torch.addmm(b, x.reshape(M * T, Din), W).view(M, T, 4 * H)
        need = any(ctx.needs_input_grad[:4])
        h, c, g = ops.lstm_fwd(xp, U.contiguous(), need, bf16)
        ctx.bf16 = bf16
        ctx.return_sequences = return_sequences
        if need:
            ctx.save_for_backward(x, W, U, h, c, g)
        return h if return_sequences else h[:, -1]

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        x, W, U, h, c, g = ctx.saved_tensors
        M, T, Din = x.shape
        H = U.shape[0]
        if ctx.return_sequences:
            dh = dout.contiguous()
        else:
            dh = dout.new_zeros(M, T, H)
            dh[:, -1] = dout
        dz = ops.lstm_bwd(dh, g, c, U.contiguous(), ctx.bf16)
        dz2 = dz.view(M * T, 4 * H)
        dx = dW = dU = db = None
        if ctx.needs_input_grad[0]:
            dx = (dz2 @ W.t()).view(M, T, Din)
        if ctx.needs_input_grad[1]:
            dW = x.reshape(M * T, Din).t() @ dz2
        if ctx.needs_input_grad[2]:
            # dU = sum_t h_{t-1}^T dz_t  (h_{-1} = 0)
            if T > 1:
                dU = torch.einsum("mth,mtg->hg", h[:, :-1], dz[:, 1:])
            else:
                dU = U.new_zeros(U.shape)
        if ctx.needs_input_grad[3]:
            db = dz2.sum(0)
        return dx, dW, dU, db, None, None


def lstm_layer(x: torch.Tensor, W: torch.Tensor, U: torch.Tensor, b: torch.Tensor,
               return_sequences: bool = True, activation: str = "tanh", bf16: bool = True) -> torch.Tensor:
    """Dispatch: HIP persistent kernel on GPU (tanh, H multiple of 16), eager otherwise."""
    from . import use_hip
    H = U.shape[0]
    if use_hip(x) and activation == "tanh" and H % 16 == 0 and 16 <= H <= (256 if bf16 else 128):
        return _HipLSTM.apply(x, W, U, b, bool(bf16), bool(return_sequences))
    return lstm_eager(x, W, U, b, return_sequences, activation)


__all__ = ["lstm_layer", "lstm_eager"]
