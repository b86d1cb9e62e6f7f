"""Reference LSTM with the HIP kernels' rounding points, for numerics tests.

The recurrences run on bf16 MFMA (``lstm_chain.hip``, ``lstm_tm.hip``, ``time4_head.hip``,
``lstm_grads.hip``), so comparing them with a plain float64 model needs tolerances of several
percent (bf16 has 8 significand bits), loose enough to hide a real bug. This reference keeps
float64 arithmetic everywhere EXCEPT where the kernels round, and rounds there exactly like
them (round-to-nearest-even to bf16):

forward   z_t = bf16(x_t) bf16(W) + bf16(h_{t-1}) bf16(U) + b; gates / c / h in full precision;
          the gates saved for the backward are bf16 for H <= 64 (the time-major kernels pack
          them, ``lstm_tm_common.h gates_pack``) and full precision for H = 128 (the training
          chain's time4; the standalone time4 layer and lstm_fwd<128> save bf16 gates as well -
          a difference well inside the tests' tolerances); the recompute-gates layers (lstm_tm.hip RG)
          save c_t in bf16 (TM_RG_BF16C), likewise not modelled here;
backward  dz_t (the four gate pre-activation gradients, from the saved gates) is rounded to
          bf16 - the value the kernels store and feed to every MFMA; dh_{t-1} = dz_t bf16(U)^T,
          dx = dz bf16(W)^T, dW = bf16(x)^T dz, dU = bf16(h_{t-1})^T dz, db = sum dz.

Everything else (the GCN, pooling, the head, the loss) is the ordinary float64 eager model. With
:func:`kernel_rounding` active, :func:`gnnqc.ops.lstm.lstm_eager` runs this instead of its
autograd recurrence (tanh activation only, as the kernels). ``rounding=False`` gives the exact
float64 gradient of the same recurrence (tested against autograd).
"""
from __future__ import annotations

import contextlib

import torch


class _State:
    on = False


@contextlib.contextmanager
def kernel_rounding(flag: bool = True):
    """Within this context the eager LSTM (CPU / float64 reference models) rounds like the kernels."""
    prev = _State.on
    _State.on = bool(flag)
    try:
        yield
    finally:
        _State.on = prev


def kernel_rounding_on() -> bool:
    return _State.on


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(t.dtype)


def _same(t: torch.Tensor) -> torch.Tensor:
    return t


class KernelLSTM(torch.autograd.Function):
    """x [M, T, Din], W [Din, 4H], U [H, 4H], b [4H] -> h [M, T, H] (or the last step [M, H])."""

    @staticmethod
    def forward(ctx, x, W, U, b, return_sequences: bool, rounding: bool = True):
        r = _bf if rounding else _same
        M, T, _ = x.shape
        H = U.shape[0]
        Wr, Ur = r(W), r(U)
        xr = r(x)
        xp = xr @ Wr + b
        h = x.new_zeros(M, H)
        c = x.new_zeros(M, H)
        hs, cs, gs = [], [], []
        for t in range(T):
            z = xp[:, t] + r(h) @ Ur
            i, f, g, o = z.split(H, dim=-1)
            i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
            c = f * c + i * g
            h = o * torch.tanh(c)
            hs.append(h)
            cs.append(c)
            gs.append(torch.cat([i, f, g, o], -1))
        hseq = torch.stack(hs, 1)
        gates = torch.stack(gs, 1)
        if rounding and H <= 64:
            gates = _bf(gates)                      # the time-major kernels save bf16 gates
        ctx.save_for_backward(xr, Wr, Ur, hseq, torch.stack(cs, 1), gates)
        ctx.return_sequences = return_sequences
        ctx.rounding = rounding
        return hseq if return_sequences else hseq[:, -1]

    @staticmethod
    def backward(ctx, dout):
        xr, Wr, Ur, hseq, cseq, gates = ctx.saved_tensors
        r = _bf if ctx.rounding else _same
        M, T, H = hseq.shape
        if ctx.return_sequences:
            dh_out = dout
        else:
            dh_out = dout.new_zeros(M, T, H)
            dh_out[:, -1] = dout
        dz = hseq.new_zeros(M, T, 4 * H)
        dh_rec = hseq.new_zeros(M, H)
        dc = hseq.new_zeros(M, H)
        for t in reversed(range(T)):
            dh = dh_out[:, t] + dh_rec
            i, f, g, o = gates[:, t].split(H, dim=-1)
            tc = torch.tanh(cseq[:, t])
            cprev = cseq[:, t - 1] if t > 0 else torch.zeros_like(dc)
            dct = dc + dh * o * (1 - tc * tc)
            dc = dct * f
            z = r(torch.cat([dct * g * i * (1 - i), dct * cprev * f * (1 - f), dct * i * (1 - g * g),
                             dh * tc * o * (1 - o)], -1))
            dz[:, t] = z
            dh_rec = z @ Ur.t()
        dx = dz @ Wr.t()
        hprev = torch.cat([hseq.new_zeros(M, 1, H), hseq[:, :-1]], 1)
        dW = torch.einsum("mtd,mtg->dg", xr, dz)
        dU = torch.einsum("mth,mtg->hg", r(hprev), dz)
        db = dz.sum((0, 1))
        return dx, dW, dU, db, None, None


__all__ = ["KernelLSTM", "kernel_rounding", "kernel_rounding_on"]
