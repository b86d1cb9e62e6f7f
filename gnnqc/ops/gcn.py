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
    """Fused stats -> affine/BN/PReLU -> weighted node sum -> concat (HIP).

    Launches per training step: gcn_prep (pool weights + batch moments + BN prep) and
    gcn_pool_fwd forward; gcn_pool_bwd and gcn_bwd_finalize (+ gcn_pool_bwd_input when dx is
    needed) backward. Weight gradients go straight into the optimiser's flat buffer when
    direct accumulation is on (see ``gnnqc.ops.lstm.direct_grad_accumulation``)."""

    @staticmethod
    def forward(ctx, x, adj, mask, anom, anom_pos, agg_mean: bool, pool: int, W, b, gamma, beta, alpha,
                running_mean, running_var, training: bool, momentum: float, eps: float, Mp: int = 0, Cp: int = 0):
        from ..utils.native import hip_ops
        ops = hip_ops()
        w, S, st = ops.gcn_prep(x, adj, mask, anom_pos, bool(agg_mean), int(pool), W.contiguous(), b.contiguous(),
                                gamma.contiguous(), beta.contiguous(), running_mean, running_var, bool(training),
                                float(momentum), float(eps))
        anom_t = anom.contiguous() if anom is not None else x.new_zeros(0)
        out = ops.gcn_pool_fwd(x, w, anom_t, W.contiguous(), b.contiguous(), st[2], st[3], alpha.contiguous(),
                               int(Mp), int(Cp))
        ctx.tm = Mp > 0
        ctx.training = training
        ctx.ca = 0 if anom is None else anom.shape[-1]
        ctx.has_anom = anom is not None
        ctx.params = (W, b, gamma, beta, alpha)
        ctx.save_for_backward(x, w, mask, W, b, alpha, st, S)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        from .lstm import _grad_sink
        ops = hip_ops()
        x, w, mask, W, b, alpha, st, S = ctx.saved_tensors
        dout = dout.contiguous()
        need = ctx.needs_input_grad
        need_w = any(need[7:12])
        empty = x.new_zeros(0)
        acc = empty
        if ctx.training or need_w:
            acc = ops.gcn_pool_bwd(x, w, dout, W.contiguous(), b.contiguous(), st[2], st[3], alpha.contiguous(),
                                   ctx.ca, ctx.tm)
        sinks = [(_grad_sink(p) if n else (empty, True)) for p, n in zip(ctx.params, need[7:12])]
        coef = ops.gcn_bwd_finalize(acc, S, W.contiguous(), b.contiguous(), st, bool(ctx.training),
                                    *[s[0] for s in sinks])
        dx = None
        if need[0]:
            dx = ops.gcn_pool_bwd_input(x, w, mask, dout, W.contiguous(), b.contiguous(), st[2], st[3],
                                        alpha.contiguous(), coef, ctx.ca, ctx.tm)
        danom = None
        if ctx.has_anom and need[3]:
            danom = dout[:, : x.shape[0], : ctx.ca].transpose(0, 1) if ctx.tm else dout[..., : ctx.ca]
        grads = [None if direct or not n else buf for (buf, direct), n in zip(sinks, need[7:12])]
        return (dx, None, None, danom, None, None, None, *grads, None, None, None, None, None, None, None)


def gcn_pool_hip_ok(x, W, aggregate: str, pooling: str, dropout: float, training: bool) -> bool:
    from . import use_hip
    linear = aggregate in ("mean", "sum") and pooling in ("mean", "sum", "selection")
    return bool(use_hip(x) and linear and not (dropout and training) and x.shape[-1] <= 8
                and W.shape[1] in (8, 16, 32))


def gcn_pool(x, adj, mask, anom, anom_pos, W, b, gamma, beta, alpha, running_mean, running_var,
             training: bool, aggregate: str = "mean", pooling: str = "mean", momentum: float = 0.99,
             eps: float = 1e-3, dropout: float = 0.0, time_major: bool = False):
    """GeneralConv + node pooling + concat -> LSTM input ``[B, T, Ca + F]``.

    Uses the fused HIP kernels for linear aggregation/pooling on GPU; otherwise the
    eager per-node path. ``time_major=True`` (HIP path only) returns ``(h [T, Mp, Cp], B)``:
    the time-major, row- and channel-padded input of
    :meth:`gnnqc.models.timelayer.TimeLayer.forward_time_major`, written by the kernel itself.
    """
    if gcn_pool_hip_ok(x, W, aggregate, pooling, dropout, training):
        ap = anom_pos.long().contiguous() if (pooling == "selection" and anom_pos is not None) else x.new_zeros(0)
        Mp = Cp = 0
        if time_major:
            B = x.shape[0]
            Mp = (B + 15) // 16 * 16
            Cp = W.shape[1] + (anom.shape[-1] if anom is not None else 0)
            Cp += (-Cp) % 4
        out = _HipGCNPool.apply(x.contiguous(), adj.float().contiguous(), mask.contiguous().float(), anom, ap,
                                aggregate == "mean", {"mean": 0, "sum": 1, "selection": 2}[pooling], W, b, gamma,
                                beta, alpha, running_mean, running_var, bool(training), float(momentum), float(eps),
                                Mp, Cp)
        return (out, x.shape[0]) if time_major else out
    if time_major:
        raise ValueError("gcn_pool(time_major=True) needs the HIP path")
    h = general_conv_eager(x, adj, mask, W, b, gamma, beta, running_mean, running_var, alpha, training,
                           aggregate, dropout, momentum, eps)
    pooled = pool_nodes(h, mask, anom_pos, pooling)
    return pooled if anom is None else torch.cat([anom, pooled], dim=-1)


class _HipGCNNodeTM(torch.autograd.Function):
    """Per-node GeneralConv -> time-major LSTM input ``[T, Mp, Cp]`` (``gcn_node.hip``).

    Forward: gcn_stats, gcn_bn_prep, gcn_node_fwd; backward: gcn_node_bwd,
    gcn_bwd_finalize (+ gcn_node_bwd_input when dx is needed, e.g. integrated gradients)."""

    @staticmethod
    def forward(ctx, x, bits, bitsT, rs, mask, W, b, gamma, beta, alpha, running_mean, running_var,
                training: bool, momentum: float, eps: float, Mp: int, Cp: int):
        from ..utils.native import hip_ops
        ops = hip_ops()
        S = ops.gcn_stats(x, mask) if training else x.new_zeros(0, dtype=torch.float64)
        st = ops.gcn_bn_prep(S, W.contiguous(), b.contiguous(), gamma.contiguous(), beta.contiguous(),
                             running_mean, running_var, bool(training), float(momentum), float(eps))
        out = ops.gcn_node_fwd(x, bits, rs, mask, W.contiguous(), b.contiguous(), st[2], st[3], alpha.contiguous(),
                               int(Mp), int(Cp))
        ctx.training = training
        ctx.params = (W, b, gamma, beta, alpha)
        ctx.save_for_backward(x, bitsT, rs, mask, W, b, alpha, st, S)
        return out

    @staticmethod
    def backward(ctx, dout):
        from ..utils.native import hip_ops
        from .lstm import _grad_sink
        ops = hip_ops()
        x, bitsT, rs, mask, W, b, alpha, st, S = ctx.saved_tensors
        dout = dout.contiguous()
        need = ctx.needs_input_grad
        empty = x.new_zeros(0)
        acc = empty
        if ctx.training or any(need[5:10]):
            acc = ops.gcn_node_bwd(x, bitsT, rs, mask, dout, W.contiguous(), b.contiguous(), st[2], st[3],
                                   alpha.contiguous())
        sinks = [(_grad_sink(p) if n else (empty, True)) for p, n in zip(ctx.params, need[5:10])]
        coef = ops.gcn_bwd_finalize(acc, S, W.contiguous(), b.contiguous(), st, bool(ctx.training),
                                    *[s[0] for s in sinks])
        dx = None
        if need[0]:
            dx = ops.gcn_node_bwd_input(x, bitsT, rs, mask, dout, W.contiguous(), b.contiguous(), st[2], st[3],
                                        alpha.contiguous(), coef)
        grads = [None if direct or not n else buf for (buf, direct), n in zip(sinks, need[5:10])]
        return (dx, None, None, None, None, *grads, None, None, None, None, None, None, None)


def gcn_node_tm_ok(x: torch.Tensor, W: torch.Tensor, aggregate: str, dropout: float, training: bool) -> bool:
    """Whether :func:`gcn_node_tm` runs the HIP kernels for this input."""
    from . import use_hip
    F_ = W.shape[1]
    N = x.shape[2]
    lds = (N * ((N + 31) // 32) + 3) // 4 * 16 + N * F_ * 4 + N * 8     # gcn_node.hip node_smem_bytes
    return (use_hip(x) and aggregate in ("mean", "sum") and not (dropout and training) and x.shape[-1] <= 4
            and F_ <= 64 and 64 % F_ == 0 and lds <= 150 * 1024)


def gcn_node_tm(x, adj, mask, W, b, gamma, beta, alpha, running_mean, running_var, training: bool,
                aggregate: str = "mean", momentum: float = 0.99, eps: float = 1e-3, cpad_to: int = 4):
    """SoilNet GeneralConv + ``Concatenate([gcn, x])`` + ``graph_reshape`` as ONE time-major tensor.

    Returns ``(h [T, Mp, Cp], M)`` with row ``m = b*N + i`` (the reference's
    per-node sequence order), channels ``[F gcn | Cin raw | 0 pad]`` (Cp a multiple
    of ``cpad_to``) and zero rows past ``M = B*N`` - the input layout of
    :meth:`gnnqc.models.timelayer.TimeLayer.forward_time_major`.
    """
    from ..utils.native import hip_ops
    B, T, N, Cin = x.shape
    M = B * N
    Mp = (M + 15) // 16 * 16
    Cp = W.shape[1] + Cin
    Cp += (-Cp) % cpad_to
    bits, bitsT, rs = hip_ops().gcn_adj_bits(adj.float().contiguous(), aggregate == "mean")
    h = _HipGCNNodeTM.apply(x.float().contiguous(), bits, bitsT, rs, mask.float().contiguous(), W, b, gamma, beta,
                            alpha, running_mean, running_var, bool(training), float(momentum), float(eps), Mp, Cp)
    return h, M


def gcn_node_tm_eager(x, adj, mask, W, b, gamma, beta, alpha, running_mean, running_var, training: bool,
                      aggregate: str = "mean", momentum: float = 0.99, eps: float = 1e-3, cpad_to: int = 4):
    """Eager oracle of :func:`gcn_node_tm` (same output layout)."""
    B, T, N, Cin = x.shape
    M = B * N
    Mp = (M + 15) // 16 * 16
    h = general_conv_eager(x, adj, mask, W, b, gamma, beta, running_mean, running_var, alpha, training, aggregate,
                           0.0, momentum, eps)
    seq = torch.cat([h, x], -1).permute(1, 0, 2, 3).reshape(T, M, -1)
    C = seq.shape[-1]
    return F.pad(seq, (0, (-C) % cpad_to, 0, Mp - M)), M


class _HipStoreGCN(torch.autograd.Function):
    """Window gather + GeneralConv + BatchNorm + PReLU + node pooling + concat in ONE launch,
    straight from the resident window store (``gcn_fused.hip``): ``(h [T, Mp, Cp], y, y_mask,
    wid)``. Backward: ONE launch adding the parameter gradients with float atomics (training mode
    only; not bitwise reproducible, so the deterministic mode keeps :class:`_HipGCNPool`). In the
    CML configuration the forward also emits the backward's coefficients and the backward is the
    dot product of dh with them (``gcn_coef_bwd``), usually run inside the batched weight-gradient
    launch."""

    @staticmethod
    def forward(ctx, data, ids, W, b, gamma, beta, alpha, running_mean, running_var, training: bool,
                momentum: float, eps: float, Mp: int, Cp: int, coef: bool = False, defer: bool = False):
        from ..utils.native import hip_ops
        wids, table, cursor = ids
        h, S, st, y, ym, wid, cf = hip_ops().gcn_fused_fwd(
            *data["fwd"], wids, table, cursor, *data["dims"], W.contiguous(), b.contiguous(), gamma.contiguous(),
            beta.contiguous(), alpha.contiguous(), running_mean, running_var, bool(training), float(momentum),
            float(eps), int(Mp), int(Cp), coef, defer)
        ctx.data, ctx.ids, ctx.training = data, ids, bool(training)
        ctx.params = (W, b, gamma, beta, alpha)
        ctx.save_for_backward(W, b, alpha, S, st, cf)
        ctx.mark_non_differentiable(y, ym, wid)
        ctx.set_materialize_grads(False)
        return h, y, ym, wid

    @staticmethod
    def backward(ctx, dh, _dy, _dym, _dwid):
        from ..utils.native import hip_ops
        from .lstm import _grad_sink
        W, b, alpha, S, st, cf = ctx.saved_tensors
        need = ctx.needs_input_grad[2:7]
        if dh is None or not any(need):
            return (None,) * 15
        if not ctx.training:
            raise RuntimeError("gcn_fused backward: parameter gradients in eval mode take the generic path")
        sinks = [(_grad_sink(p) if n else (torch.zeros_like(p), False)) for p, n in zip(ctx.params, need)]
        from .lstm import defer_to_grads_launch
        direct = all(direct for (_, direct), n in zip(sinks, need) if n)
        if cf.numel() > 0:
            # coefficient form: dh x coef, deferred onto the batched LSTM weight-gradient launch when
            # every gradient goes straight into .grad
            ca = int(ctx.data["ca"])
            # (the coefficients are normally written by spare workgroups of the chain forward launch;
            # if no chain launch took the job, run it now)
            hip_ops().gcn_coef_flush(cf)
            jt = [dh.contiguous(), cf, S, st, W.contiguous(), b.contiguous(), sinks[0][0], sinks[2][0], sinks[3][0],
                  sinks[4][0]]
            if not (direct and defer_to_grads_launch((jt, [ca]))):
                hip_ops().gcn_coef_bwd(jt[0], ca, *jt[1:])
            grads = [None if direct or not n else buf for (buf, direct), n in zip(sinks, need)]
            return (None, None, *grads, None, None, None, None, None, None, None, None, None)
        wids, table, cursor = ctx.ids
        args = (dh.contiguous(), int(ctx.data["ca"]), *ctx.data["bwd"], wids, table, cursor, *ctx.data["dims"], S, st,
                W.contiguous(), b.contiguous(), alpha.contiguous(), sinks[0][0], sinks[2][0], sinks[3][0], sinks[4][0])
        # (deferred onto the batched LSTM weight-gradient launch when every gradient goes straight
        # into .grad and the configuration is the one that launch instantiates)
        if not (direct and tuple(W.shape) == (2, 16) and defer_to_grads_launch(_gcn_job_lists(args))):
            hip_ops().gcn_fused_bwd(*args)
        grads = [None if direct or not n else buf for (buf, direct), n in zip(sinks, need)]
        return (None, None, *grads, None, None, None, None, None, None, None, None, None)


def _gcn_job_lists(args):
    """gcn_fused_bwd's arguments as lstm_grads_multi's (gcn_t, gcn_i) job lists."""
    (dh, c_off, series, shift, scale, wg, wc, wv, gap, pw, wids, table, cursor, tb, seq_len, time_norm, S, st, W, b,
     alpha, dW, dgamma, dbeta, dalpha) = args
    cur = cursor if cursor is not None else series.new_zeros(0, dtype=torch.long)
    return ([dh, series, shift, scale, wg, wc, wv, gap, pw, wids, table, cur, S, st, W, b, alpha, dW, dgamma, dbeta,
             dalpha], [int(c_off), int(tb), int(seq_len), int(bool(time_norm))])


def store_gcn_ok(store, layer, training: bool, pooling: str) -> bool:
    """Whether :func:`gcn_pool_from_store` runs for this store / GeneralConv configuration."""
    from . import deterministic, use_hip
    if not (use_hip(store.series) and getattr(store, "per_sensor", False) and store.series.dtype == torch.float32
            and store.win_label.dim() == 1):
        return False
    if training and deterministic():
        return False
    W = layer.kernel
    C, N = store.n_feat, store.n_nodes
    return (layer.aggregate in ("mean", "sum") and pooling in ("mean", "sum", "selection")
            and not (layer.dropout and training) and W.shape[0] == C and 1 <= C <= 4 and N * C <= 128
            and W.shape[1] in (8, 16, 32) and store.seq_len >= 1)


def gcn_pool_from_store(store, ids, layer, training: bool, pooling: str = "mean", defer: bool = False):
    """The CML GCN front end of a training / evaluation step straight from ``store``:
    ``(h [T, Mp, Cp], B, y [B], y_mask [B], wid [B])`` with ``h`` the time-major LSTM input
    (``[flagged series | pooled GCN | 0 pad]``) of :meth:`gnnqc.models.timelayer.TimeLayer.forward_time_major`.
    ``ids``: window ids [B] (-1 = padding) or a :class:`gnnqc.data.store.CursorIds`.

    ``defer`` (training with the coefficient-form backward only): no launch here; the next headed
    LSTM chain forward launch whose input is ``h`` runs this forward as producer workgroups and its
    first stage streams their output (``gcn_fused.h`` ``gcn_prod_body``). Every other consumer of the
    outputs must call ``hip_ops().gcn_prod_flush(h)`` first (the backward does)."""
    from ..data.store import CursorIds
    agg_mean = layer.aggregate == "mean"
    pool = {"mean": 0, "sum": 1, "selection": 2}[pooling]
    data = store.gcn_fused_data(agg_mean, pool)
    e = store.series.new_zeros(0, dtype=torch.long)
    if isinstance(ids, CursorIds):
        idt = (e, ids.table, ids.cursor)
        B = int(ids.table.shape[1])
    else:
        idt = (ids.to(store.device).long().contiguous(), e, None)
        B = int(idt[0].shape[0])
    F_ = layer.kernel.shape[1]
    C = store.n_feat
    Mp = (B + 15) // 16 * 16
    Cp = C + F_
    Cp += (-Cp) % 4
    # training with gradients: the forward also writes the backward's per-(t, sample, feature)
    # coefficients, so the backward is a streaming dot product against dh (gcn_coef_bwd). (Decided
    # here: inside an autograd Function's forward grad mode is always off.)
    import os
    coef = (bool(training) and torch.is_grad_enabled() and tuple(layer.kernel.shape) == (2, 16)
            and any(p.requires_grad for p in (layer.kernel, layer.bn_gamma, layer.bn_beta, layer.prelu_alpha))
            and os.environ.get("GNNQC_GCN_COEF", "1") == "1")
    # (off by default: measured slower - the producers' id -> window -> series load chain and
    # per-row compute take ~13 us inside the chain launch vs 11.4 us for the forward's own launch;
    # profiles/r5_gcn_producer_ab.txt)
    defer = bool(defer and coef and os.environ.get("GNNQC_GCN_PROD", "0") == "1")
    h, y, ym, wid = _HipStoreGCN.apply(data, idt, layer.kernel, layer.bias, layer.bn_gamma, layer.bn_beta,
                                       layer.prelu_alpha, layer.bn_moving_mean, layer.bn_moving_variance,
                                       bool(training), float(layer.momentum), float(layer.eps), Mp, Cp, coef, defer)
    return h, B, y, ym, wid


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


__all__ = ["gcn_pool", "gcn_pool_hip_ok", "gcn_node_tm", "gcn_node_tm_eager", "gcn_node_tm_ok", "node_pool_weights", "masked_batchnorm", "general_conv_eager", "pool_nodes",
           "normalized_adjacency", "prelu"]
