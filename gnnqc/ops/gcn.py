"""GeneralConv (+ BatchNorm + PReLU) with fused node pooling.

Semantics of spektral 1.3 ``GeneralConv(channels, batch_norm=True, dropout,
aggregate, activation='prelu')`` as built at ``libs/create_model.py:184-189``:
``x@W+b -> BatchNorm(momentum .99, eps 1e-3) -> Dropout -> PReLU -> aggregate
messages x_j over edges (i <- j)``, followed for CML by ``timeseries_pooling``
(mean/sum/max over the nodes of a sample, or ``selection`` of the flagged node,
``:8-41``).

Graphs here are dense per-sample adjacencies ``[B, N, N]`` shared by all time
steps, with a node mask for padding. BatchNorm statistics run over the valid
node rows only (exactly the rows the reference's ragged batch contains).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def normalized_adjacency(adj: torch.Tensor, aggregate: str = "mean") -> torch.Tensor:
    """Row-normalised (mean) or raw (sum) aggregation matrix. Row i aggregates j."""
    if aggregate == "mean":
        deg = adj.sum(-1, keepdim=True)
        return adj / deg.clamp(min=1.0)
    if aggregate == "sum":
        return adj
    raise ValueError(f"linear aggregation expected, got {aggregate}")


def node_pool_weights(adj: torch.Tensor, mask: torch.Tensor, anom_pos: torch.Tensor | None,
                      aggregate: str = "mean", pooling: str = "mean") -> torch.Tensor:
    """w[b, j] such that pool(aggregate(a))[b, t] = sum_j w[b, j] a[b, t, j]."""
    A = normalized_adjacency(adj, aggregate)
    if pooling == "mean":
        p = mask / mask.sum(-1, keepdim=True).clamp(min=1.0)
    elif pooling == "sum":
        p = mask
    elif pooling == "selection":
        p = F.one_hot(anom_pos.clamp(min=0), adj.shape[-1]).to(adj.dtype)
    else:
        raise ValueError(f"linear pooling expected, got {pooling}")
    return torch.bmm(p.unsqueeze(1), A).squeeze(1).contiguous()


def masked_batchnorm(z: torch.Tensor, mask: torch.Tensor, gamma, beta, running_mean, running_var,
                     training: bool, momentum: float = 0.99, eps: float = 1e-3) -> torch.Tensor:
    """BatchNorm over the last axis using only rows where ``mask`` (broadcast) is 1.

    ``z``: [B, T, N, F]; ``mask``: [B, N]. Keras semantics: biased batch variance,
    ``moving = moving * momentum + batch * (1 - momentum)``.
    """
    m = mask[:, None, :, None].to(z.dtype)
    if training:
        cnt = (mask.sum() * z.shape[1]).clamp(min=1.0)
        mu = (z * m).sum(dim=(0, 1, 2)) / cnt
        var = (((z - mu) ** 2) * m).sum(dim=(0, 1, 2)) / cnt
        with torch.no_grad():
            running_mean.mul_(momentum).add_(mu.detach() * (1 - momentum))
            running_var.mul_(momentum).add_(var.detach() * (1 - momentum))
    else:
        mu, var = running_mean, running_var
    return (z - mu) * torch.rsqrt(var + eps) * gamma + beta


def prelu(x, alpha):
    return torch.where(x > 0, x, alpha * x)


def general_conv_eager(x, adj, mask, W, b, gamma, beta, running_mean, running_var, alpha, training,
                       aggregate="mean", dropout=0.0, momentum=0.99, eps=1e-3, use_batch_norm=True,
                       activation="prelu"):
    """Per-node GeneralConv output [B, T, N, F] (reference oracle, any aggregation)."""
    z = torch.matmul(x, W) + b
    if use_batch_norm:
        z = masked_batchnorm(z, mask, gamma, beta, running_mean, running_var, training, momentum, eps)
    if dropout and training:
        z = F.dropout(z, dropout, training=True)
    if activation == "prelu":
        a = prelu(z, alpha)
    elif activation in (None, "linear"):
        a = z
    else:
        a = getattr(torch, activation)(z) if hasattr(torch, activation) else getattr(F, activation)(z)
    a = a * mask[:, None, :, None]
    if aggregate == "max":
        # max over neighbours j of a[j] (messages only along edges)
        big = torch.finfo(a.dtype).max
        msg = a.unsqueeze(2).expand(-1, -1, a.shape[2], -1, -1)          # [B,T,N(i),N(j),F]
        edge = adj[:, None, :, :, None] > 0
        out = torch.where(edge, msg, torch.full_like(msg, -big)).amax(3)
        out = torch.where(edge.any(3), out, torch.zeros_like(out))
        return out * mask[:, None, :, None]
    A = normalized_adjacency(adj, aggregate)
    return torch.einsum("bij,btjf->btif", A, a)


class _HipGCNPool(torch.autograd.Function):
    """Fused stats -> affine/BN/PReLU -> weighted node sum -> concat (HIP)."""

    @staticmethod
    def forward(ctx, x, w, mask, anom, W, b, gamma, beta, alpha, running_mean, running_var, training: bool,
                momentum: float, eps: float):
        from ..utils.native import hip_ops
        ops = hip_ops()
        Cin = x.shape[-1]
        if training:
            S = ops.gcn_stats(x, mask)
            cnt = S[-1].clamp(min=1.0)
            S1 = S[:Cin]
            S2 = S[Cin:Cin + Cin * Cin].view(Cin, Cin)
            ex = S1 / cnt
            cov = S2 / cnt - torch.outer(ex, ex)
            Wd = W.double()
            mu = (ex @ Wd + b.double()).float()
            var = torch.einsum("kf,kl,lf->f", Wd, cov, Wd).clamp(min=0).float()
            with torch.no_grad():
                running_mean.mul_(momentum).add_(mu * (1 - momentum))
                running_var.mul_(momentum).add_(var * (1 - momentum))
        else:
            mu, var = running_mean, running_var
            S1 = S2 = cnt = None
        invstd = torch.rsqrt(var + eps)
        scale = (gamma * invstd).contiguous()
        shift = (beta - mu * scale).contiguous()
        anom_t = anom.contiguous() if anom is not None else x.new_zeros(0)
        out = ops.gcn_pool_fwd(x, w, anom_t, W.contiguous(), b.contiguous(), scale, shift, alpha.contiguous())
        ctx.training = training
        ctx.ca = 0 if anom is None else anom.shape[-1]
        ctx.has_anom = anom is not None
        stats = (S1.float(), S2.float(), cnt.float().reshape(1)) if training else (x.new_zeros(0),) * 3
        ctx.save_for_backward(x, w, mask, W, b, gamma, alpha, mu, invstd, scale, shift, *stats)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        ops = hip_ops()
        (x, w, mask, W, b, gamma, alpha, mu, invstd, scale, shift, S1, S2, cnt) = ctx.saved_tensors
        dout = dout.contiguous()
        Cin = x.shape[-1]
        need_w = any(ctx.needs_input_grad[4:9])
        dW = db = dgamma = dbeta = dalpha = None
        if ctx.training or need_w:
            acc = ops.gcn_pool_bwd(x, w, dout, W.contiguous(), b.contiguous(), scale, shift, alpha.contiguous(),
                                   ctx.ca)
            A, Z, P, Q = acc[0], acc[1], acc[2], acc[3:3 + Cin]
            dbeta = A
            dgamma = invstd * (Z - mu * A)
            dalpha = P
        if ctx.training:
            n = cnt[0]
            sxx = invstd * (S2 @ W + torch.outer(S1, b - mu))       # sum_rows x_k * xhat_f
            dW = scale * (Q - torch.outer(S1, A / n) - sxx * (dgamma / n))
            db = torch.zeros_like(b)
            c0 = scale * (-A / n + mu * invstd * dgamma / n)
            c2 = -scale * invstd * dgamma / n
        else:
            # inference-mode BN is a fixed affine map (e.g. integrated gradients: frozen weights,
            # input gradients only -> no weight-gradient reduction at all)
            if need_w:
                dW = scale * Q
                db = scale * A
            c0 = torch.zeros_like(scale)
            c2 = torch.zeros_like(scale)
        dx = None
        if ctx.needs_input_grad[0]:
            coef = torch.stack([c0, scale, c2]).contiguous()
            dx = ops.gcn_pool_bwd_input(x, w, mask, dout, W.contiguous(), b.contiguous(), scale, shift,
                                        alpha.contiguous(), coef, ctx.ca)
        danom = dout[..., : ctx.ca] if (ctx.has_anom and ctx.needs_input_grad[3]) else None
        return dx, None, None, danom, dW, db, dgamma, dbeta, dalpha, None, None, None, None, None


def gcn_pool(x, adj, mask, anom, anom_pos, W, b, gamma, beta, alpha, running_mean, running_var,
             training: bool, aggregate: str = "mean", pooling: str = "mean", momentum: float = 0.99,
             eps: float = 1e-3, dropout: float = 0.0):
    """GeneralConv + node pooling + concat -> LSTM input ``[B, T, Ca + F]``.

    Uses the fused HIP kernels for linear aggregation/pooling on GPU; otherwise the
    eager per-node path.
    """
    from . import use_hip
    linear = aggregate in ("mean", "sum") and pooling in ("mean", "sum", "selection")
    if use_hip(x) and linear and not (dropout and training) and x.shape[-1] <= 8 and 256 % W.shape[1] == 0:
        w = node_pool_weights(adj, mask, anom_pos, aggregate, pooling)
        return _HipGCNPool.apply(x.contiguous(), w, mask.contiguous().float(), anom, W, b, gamma, beta, alpha,
                                 running_mean, running_var, bool(training), float(momentum), float(eps))
    h = general_conv_eager(x, adj, mask, W, b, gamma, beta, running_mean, running_var, alpha, training,
                           aggregate, dropout, momentum, eps)
    pooled = pool_nodes(h, mask, anom_pos, pooling)
    return pooled if anom is None else torch.cat([anom, pooled], dim=-1)


def pool_nodes(h: torch.Tensor, mask: torch.Tensor, anom_pos, pooling: str = "mean") -> torch.Tensor:
    """``timeseries_pooling`` over valid nodes: [B,T,N,F] -> [B,T,F]."""
    m = mask[:, None, :, None].to(h.dtype)
    if pooling == "mean":
        return (h * m).sum(2) / m.sum(2).clamp(min=1.0)
    if pooling == "sum":
        return (h * m).sum(2)
    if pooling == "max":
        big = torch.finfo(h.dtype).max
        return torch.where(m > 0, h, torch.full_like(h, -big)).amax(2) * (m.sum(2) > 0)
    if pooling == "selection":
        idx = anom_pos.clamp(min=0)[:, None, None, None].expand(-1, h.shape[1], 1, h.shape[3])
        return h.gather(2, idx).squeeze(2)
    raise ValueError(pooling)


__all__ = ["gcn_pool", "node_pool_weights", "masked_batchnorm", "general_conv_eager", "pool_nodes",
           "normalized_adjacency", "prelu"]
