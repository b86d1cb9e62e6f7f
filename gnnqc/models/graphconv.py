"""Graph convolution layers on dense per-sample graphs.

Input convention: ``x [B, T, N, F]`` node features for every time step,
``adj [B, N, N]`` 0/1 adjacency (row i aggregates from column j; self loops come
from the data like the reference, whose distance-0 diagonal is below the radius),
``mask [B, N]`` valid nodes. One adjacency per sample is shared by all T steps
instead of the reference's per-(sample, step) block-diagonal SparseTensor
(``libs/preprocessing_functions.py:637-666``).

* :class:`GeneralConv` - spektral GeneralConv (the reference default); its fused
  HIP path (``gnnqc.ops.gcn``) is used by the CML classifier.
* :class:`AGNNConv`, :class:`GATConv`, :class:`GatedGraphConv` (``libs/create_model.py:173-194``)
  and :class:`EdgeConv` (``xai/libs/create_model.py:147-153``): eager PyTorch,
  chunked over time to bound the ``[B, t, N, N, .]`` edge tensors.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.gcn import general_conv_eager, normalized_adjacency
from .layers import Dense, apply_activation, glorot_uniform_


def _time_chunks(T: int, B: int, N: int, budget: int = 1 << 26):
    step = max(1, budget // max(1, B * N * N * 16))
    for t0 in range(0, T, step):
        yield t0, min(T, t0 + step)


def _masked_edge_softmax(scores: torch.Tensor, adj: torch.Tensor) -> torch.Tensor:
    """Softmax over neighbours j of node i. scores [..., N, N, H], adj [B, 1, N, N, 1]-broadcastable."""
    neg = torch.finfo(scores.dtype).min
    s = torch.where(adj > 0, scores, torch.full_like(scores, neg))
    s = s - s.amax(dim=-2, keepdim=True)
    e = torch.exp(s) * (adj > 0)
    return e / e.sum(dim=-2, keepdim=True).clamp(min=1e-30)


class GeneralConv(nn.Module):
    """spektral GeneralConv(channels, batch_norm=True, dropout, aggregate, activation)."""

    def __init__(self, in_features: int, channels: int = 256, dropout: float = 0.0, aggregate: str = "sum",
                 activation: str = "prelu", use_batch_norm: bool = True, regularizer: Optional[float] = None):
        super().__init__()
        self.channels = channels
        self.dropout = float(dropout or 0.0)
        self.aggregate = aggregate
        self.activation = activation
        self.use_batch_norm = use_batch_norm
        self.regularizer = regularizer
        self.kernel = nn.Parameter(torch.empty(in_features, channels))
        self.bias = nn.Parameter(torch.zeros(channels))
        glorot_uniform_(self.kernel, in_features, channels)
        self.prelu_alpha = nn.Parameter(torch.zeros(channels))
        self.bn_gamma = nn.Parameter(torch.ones(channels))
        self.bn_beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("bn_moving_mean", torch.zeros(channels))
        self.register_buffer("bn_moving_variance", torch.ones(channels))
        self.momentum, self.eps = 0.99, 1e-3

    @property
    def out_features(self):
        return self.channels

    def forward(self, x, adj, mask):
        return general_conv_eager(x, adj, mask, self.kernel, self.bias, self.bn_gamma, self.bn_beta,
                                  self.bn_moving_mean, self.bn_moving_variance, self.prelu_alpha, self.training,
                                  self.aggregate, self.dropout, self.momentum, self.eps, self.use_batch_norm,
                                  self.activation)

    def reg_loss(self):
        return self.regularizer * (self.kernel ** 2).sum() if self.regularizer else None


class AGNNConv(nn.Module):
    """spektral AGNNConv: cosine-attention propagation, output dim = input dim."""

    def __init__(self, in_features: int, aggregate: str = "sum", activation: Optional[str] = None,
                 trainable: bool = True):
        super().__init__()
        self.in_features = in_features
        self.aggregate = aggregate
        self.activation = activation
        self.beta = nn.Parameter(torch.ones(1), requires_grad=trainable)
        self.prelu_alpha = nn.Parameter(torch.zeros(in_features)) if activation == "prelu" else None

    @property
    def out_features(self):
        return self.in_features

    def forward(self, x, adj, mask):
        B, T, N, Fdim = x.shape
        xn = F.normalize(x, dim=-1)
        outs = []
        a = adj[:, None, :, :, None]
        for t0, t1 in _time_chunks(T, B, N):
            cos = torch.einsum("btif,btjf->btij", xn[:, t0:t1], xn[:, t0:t1]).unsqueeze(-1) * self.beta
            att = _masked_edge_softmax(cos, a)[..., 0]                     # [B,t,N,N]
            o = torch.einsum("btij,btjf->btif", att, x[:, t0:t1])
            if self.aggregate == "mean":
                o = o / adj.sum(-1).clamp(min=1)[:, None, :, None]
            outs.append(o)
        out = torch.cat(outs, 1)
        if self.activation == "prelu":
            out = torch.where(out > 0, out, self.prelu_alpha * out)
        else:
            out = apply_activation(out, self.activation)
        return out * mask[:, None, :, None]


class GATConv(nn.Module):
    """spektral GATConv(channels, attn_heads, concat_heads=True, dropout_rate, add_self_loops=True)."""

    def __init__(self, in_features: int, channels: int, attn_heads: int = 1, concat_heads: bool = True,
                 dropout_rate: float = 0.5, activation: Optional[str] = None, regularizer: Optional[float] = None):
        super().__init__()
        self.channels, self.heads, self.concat = channels, attn_heads, concat_heads
        self.dropout_rate = float(dropout_rate or 0.0)
        self.activation = activation
        self.regularizer = regularizer
        self.kernel = nn.Parameter(torch.empty(in_features, attn_heads, channels))
        self.attn_kernel_self = nn.Parameter(torch.empty(channels, attn_heads, 1))
        self.attn_kernel_neighs = nn.Parameter(torch.empty(channels, attn_heads, 1))
        out = channels * attn_heads if concat_heads else channels
        self.bias = nn.Parameter(torch.zeros(out))
        glorot_uniform_(self.kernel, in_features, attn_heads * channels)
        glorot_uniform_(self.attn_kernel_self, channels, attn_heads)
        glorot_uniform_(self.attn_kernel_neighs, channels, attn_heads)
        self.prelu_alpha = nn.Parameter(torch.zeros(out)) if activation == "prelu" else None

    @property
    def out_features(self):
        return self.channels * self.heads if self.concat else self.channels

    def forward(self, x, adj, mask):
        B, T, N, _ = x.shape
        eye = torch.eye(N, device=adj.device, dtype=adj.dtype)
        a = ((adj + eye * mask[:, :, None]) > 0).to(x.dtype)[:, None, :, :, None]   # add self loops
        h = torch.einsum("btnf,fhc->btnhc", x, self.kernel)
        s_self = torch.einsum("btnhc,chk->btnh", h, self.attn_kernel_self)
        s_nb = torch.einsum("btnhc,chk->btnh", h, self.attn_kernel_neighs)
        outs = []
        for t0, t1 in _time_chunks(T, B, N):
            e = F.leaky_relu(s_self[:, t0:t1, :, None, :] + s_nb[:, t0:t1, None, :, :], 0.2)   # [B,t,i,j,H]
            att = _masked_edge_softmax(e, a)
            if self.training and self.dropout_rate > 0:
                att = F.dropout(att, self.dropout_rate)
            outs.append(torch.einsum("btijh,btjhc->btihc", att, h[:, t0:t1]))
        o = torch.cat(outs, 1)
        o = o.reshape(B, T, N, -1) if self.concat else o.mean(3)
        o = o + self.bias
        if self.activation == "prelu":
            o = torch.where(o > 0, o, self.prelu_alpha * o)
        else:
            o = apply_activation(o, self.activation)
        return o * mask[:, None, :, None]

    def reg_loss(self):
        return self.regularizer * (self.kernel ** 2).sum() if self.regularizer else None


class _KerasGRUCell(nn.Module):
    """Keras GRUCell(units, reset_after=True): gate order z, r, h."""

    def __init__(self, in_features: int, units: int):
        super().__init__()
        self.units = units
        self.kernel = nn.Parameter(torch.empty(in_features, 3 * units))
        self.recurrent_kernel = nn.Parameter(torch.empty(units, 3 * units))
        self.bias = nn.Parameter(torch.zeros(2, 3 * units))
        glorot_uniform_(self.kernel, in_features, 3 * units)
        from .layers import orthogonal_
        orthogonal_(self.recurrent_kernel)

    def forward(self, x, h):
        H = self.units
        xm = x @ self.kernel + self.bias[0]
        hm = h @ self.recurrent_kernel + self.bias[1]
        z = torch.sigmoid(xm[..., :H] + hm[..., :H])
        r = torch.sigmoid(xm[..., H:2 * H] + hm[..., H:2 * H])
        hh = torch.tanh(xm[..., 2 * H:] + r * hm[..., 2 * H:])
        return z * h + (1 - z) * hh


class GatedGraphConv(nn.Module):
    """spektral GatedGraphConv(channels, n_layers): GRU over ``n_layers`` message rounds."""

    def __init__(self, in_features: int, channels: int, n_layers: int, activation: Optional[str] = None,
                 regularizer: Optional[float] = None):
        super().__init__()
        if in_features > channels:
            raise ValueError("GatedGraphConv needs channels >= input features")
        self.in_features, self.channels, self.n_layers = in_features, channels, int(n_layers)
        self.activation = activation
        self.regularizer = regularizer
        self.kernel = nn.Parameter(torch.empty(self.n_layers, channels, channels))
        for i in range(self.n_layers):
            glorot_uniform_(self.kernel.data[i], channels, channels)
        self.rnn = _KerasGRUCell(channels, channels)
        self.prelu_alpha = nn.Parameter(torch.zeros(channels)) if activation == "prelu" else None

    @property
    def out_features(self):
        return self.channels

    def forward(self, x, adj, mask):
        h = F.pad(x, (0, self.channels - x.shape[-1]))
        for i in range(self.n_layers):
            m = torch.einsum("bij,btjf->btif", adj, h @ self.kernel[i])
            h = self.rnn(m, h)
        if self.activation == "prelu":
            h = torch.where(h > 0, h, self.prelu_alpha * h)
        else:
            h = apply_activation(h, self.activation)
        return h * mask[:, None, :, None]

    def reg_loss(self):
        return self.regularizer * (self.kernel ** 2).sum() if self.regularizer else None


class EdgeConv(nn.Module):
    """spektral EdgeConv(channels, mlp_hidden, mlp_activation='relu', aggregate)."""

    def __init__(self, in_features: int, channels: int, mlp_hidden: Optional[Sequence[int]] = None,
                 mlp_activation: str = "relu", aggregate: str = "sum", activation: Optional[str] = None,
                 regularizer: Optional[float] = None):
        super().__init__()
        self.channels, self.aggregate = channels, aggregate
        dims = [2 * in_features] + list(mlp_hidden or [])
        self.hidden = nn.ModuleList([Dense(dims[i], dims[i + 1], mlp_activation, regularizer=regularizer)
                                     for i in range(len(dims) - 1)])
        self.out = Dense(dims[-1], channels, None, regularizer=regularizer)
        self.activation = activation
        self.prelu_alpha = nn.Parameter(torch.zeros(channels)) if activation == "prelu" else None

    @property
    def out_features(self):
        return self.channels

    def forward(self, x, adj, mask):
        B, T, N, Fdim = x.shape
        outs = []
        a = adj[:, None, :, :, None]
        for t0, t1 in _time_chunks(T, B, N):
            xi = x[:, t0:t1, :, None, :].expand(-1, -1, N, N, Fdim)
            xj = x[:, t0:t1, None, :, :].expand(-1, -1, N, N, Fdim)
            m = torch.cat([xi, xj - xi], -1)
            for layer in self.hidden:
                m = layer(m)
            m = self.out(m)
            if self.activation == "prelu":
                m = torch.where(m > 0, m, self.prelu_alpha * m)
            else:
                m = apply_activation(m, self.activation)
            m = m * a
            o = m.sum(3) if self.aggregate != "max" else m.amax(3)
            if self.aggregate == "mean":
                o = o / adj.sum(-1).clamp(min=1)[:, None, :, None]
            outs.append(o)
        return torch.cat(outs, 1) * mask[:, None, :, None]

    def reg_loss(self):
        terms = [l.reg_loss() for l in list(self.hidden) + [self.out]]
        terms = [t for t in terms if t is not None]
        return sum(terms) if terms else None


def make_graph_layer(cfg_gc, in_features: int) -> nn.Module:
    name = cfg_gc.get("layer", "GeneralConv")
    act = cfg_gc.get("activation", "prelu")
    reg = cfg_gc.get("regularizer")
    if name == "GeneralConv":
        return GeneralConv(in_features, cfg_gc.get("units", 16), cfg_gc.get("dropout_rate", 0.0),
                           cfg_gc.get("aggregation_type", "mean"), act, regularizer=reg)
    if name == "AGNNConv":
        return AGNNConv(in_features, cfg_gc.get("aggregation_type", "sum"), act)
    if name == "GATConv":
        return GATConv(in_features, cfg_gc.get("units", 16), cfg_gc.get("attention_heads") or 1,
                       dropout_rate=cfg_gc.get("dropout_rate", 0.5), activation=act, regularizer=reg)
    if name == "GatedGraphConv":
        return GatedGraphConv(in_features, cfg_gc.get("units", 16), cfg_gc.get("n_layers") or 1, act, reg)
    if name == "EdgeConv":
        return EdgeConv(in_features, cfg_gc.get("units", 16), cfg_gc.get("mlp_hidden"), "relu",
                        cfg_gc.get("aggregation_type", "sum"), act, reg)
    raise ValueError(f"unknown graph layer {name}")


__all__ = ["GeneralConv", "AGNNConv", "GATConv", "GatedGraphConv", "EdgeConv", "make_graph_layer"]
