"""GCNClassifier (``libs/create_model.py:140-258``).

CML: graph conv over each sample's neighbourhood -> node pooling per time step ->
concat ``[flagged series, pooled]`` -> TimeLayer -> Dense(64) LeakyReLU Dense(64)
LeakyReLU Dense(1, sigmoid). One prediction per window.

SoilNet: graph conv -> concat ``[gcn out, raw features]`` -> one sequence per node
(``graph_reshape``) -> TimeLayer -> head. One prediction per node and window.

XAI-snapshot options (``xai/libs/create_model.py:105-239``): ``spatial_transformer``,
``nodes_sequence_layer`` (SensorsTimeLayer), ``dropout`` after the TimeLayer and the
first dense layer, ``pooling.type = selection``.

Inputs (dense padded batches, see :class:`gnnqc.data.store.Batch`):
CML ``(x [B,T,N,2], anom [B,T,2], adj [B,N,N], node_mask [B,N], anom_pos [B][, coords])``;
SoilNet ``(x [B,T,N,3], adj, node_mask[, coords])``.
``forward`` returns probabilities (Keras ``sigmoid`` output); ``logits`` the
pre-sigmoid values used by the numerically stable loss.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from ..config import freq_minutes
from ..ops.gcn import (gcn_node_tm, gcn_node_tm_ok, gcn_pool, gcn_pool_from_store, gcn_pool_hip_ok, pool_nodes,
                       store_gcn_ok)
from .graphconv import GeneralConv, make_graph_layer
from .layers import Dense, Dropout, LeakyReLU
from .spatial import SensorsTimeLayer, SpatialTransformer
from .timelayer import TimeLayer


def _get(cfg, dotted, default=None):
    node = cfg
    for p in dotted.split("."):
        if node is None or not hasattr(node, "get"):
            return default
        node = node.get(p)
    return default if node is None else node


def compute_bf16(model_config) -> bool:
    return str(_get(model_config, "runtime.compute_dtype", "bf16")).lower() != "fp32"


def timeseries_pooling(h: torch.Tensor, mask: torch.Tensor, anom_pos: torch.Tensor,
                       aggregation_type: str = "mean", type: str = "pool") -> torch.Tensor:
    """Node pooling per time step, [B,T,N,F] -> [B,T,F] (``libs/create_model.py:8-41``)."""
    return pool_nodes(h, mask, anom_pos, "selection" if type == "selection" else aggregation_type)


def graph_reshape(h: torch.Tensor) -> torch.Tensor:
    """Every node becomes its own sequence: [B,T,N,F] -> [B*N, T, F] (``:242-258``)."""
    B, T, N, Fdim = h.shape
    return h.permute(0, 2, 1, 3).reshape(B * N, T, Fdim)


class GCNClassifier(nn.Module):
    def __init__(self, model_config, preprocessing_config):
        super().__init__()
        mc, pc = model_config, preprocessing_config
        self.model_config = mc
        self.ds_type = pc["ds_type"]
        # flagged-sensor neighbourhoods (CML; SoilNet of the XAI generation) vs network-wide SoilNet
        self.per_sensor = bool(pc.get("per_sensor", self.ds_type == "cml"))
        self.freq = freq_minutes(self.ds_type)
        self.timestep_before, self.timestep_after = int(pc["timestep_before"]), int(pc["timestep_after"])
        self.batch_size = int(pc["batch_size"])
        in_feat = 2 if self.ds_type == "cml" else 3
        self.input_feature_numb = in_feat
        self.register_buffer("model_info", torch.tensor([self.timestep_before, self.timestep_after,
                                                         self.batch_size, self.freq], dtype=torch.int32))
        self.model_type = self.ds_type
        self.model_normalization = pc.get("normalization") or ("rolling_median" if self.ds_type == "cml"
                                                               else "scale_range")
        bf16 = compute_bf16(mc)
        gc = mc["graph_convolution"]
        self.aggregation_type = _get(mc, "pooling.aggregation_type", "mean")
        self.pooling_type = _get(mc, "pooling.type", "pool")
        node_feat = in_feat
        self.sensors_time_layer = None
        if _get(mc, "nodes_sequence_layer.use", False):
            nsl = mc["nodes_sequence_layer"]
            self.sensors_time_layer = SensorsTimeLayer(in_feat, nsl.get("units", 16), nsl.get("layer_type", "lstm"),
                                                       kernel_size=nsl.get("kernel_size", 5), compute_bf16=bf16)
            node_feat = nsl.get("units", 16)
        self.spatial_transformer = None
        if _get(mc, "spatial_transformer.use", False):
            st = mc["spatial_transformer"]
            self.spatial_transformer = SpatialTransformer(st["min_scale"], st["max_scale"], st["scale_numb"],
                                                          st.get("units", 32))
            node_feat += st.get("units", 32) * (2 if self.ds_type == "cml" else 1)
        self.gcn_layer = make_graph_layer(gc, node_feat)
        self.features_gcn_out = self.gcn_layer.out_features
        time_in = in_feat + self.features_gcn_out
        sl = mc["sequence_layer"]
        self.time_layer = TimeLayer(time_in, sl.get("filter_1_size", 16), sl.get("n_stacks", 2),
                                    sl.get("algorithm", "lstm"), sl.get("activation", "tanh"), sl.get("kernel_size"),
                                    sl.get("regularizer"), sl.get("pool_size", 3), sl.get("alpha", 0.3),
                                    compute_bf16=bf16)
        rates = _get(mc, "dropout.rates", [0.0, 0.0]) if _get(mc, "dropout.use", False) else [0.0, 0.0]
        self.dropout1, self.dropout2 = Dropout(rates[0]), Dropout(rates[1])
        d = mc["dense"]
        self.dense = Dense(self.time_layer.out_features, d.get("units", 64), regularizer=d.get("regularizer"))
        self.leakyrelu4 = LeakyReLU(d.get("alpha", 0.3))
        self.dense2 = Dense(d.get("units", 64), d.get("units", 64), regularizer=d.get("regularizer"))
        self.leakyrelu5 = LeakyReLU(d.get("alpha", 0.3))
        self.dense_out = Dense(d.get("units", 64), 1)

    # ----------------------------------------------------------------- parts
    def _node_features(self, x, mask, coords):
        feats = x
        if self.sensors_time_layer is not None:
            feats = self.sensors_time_layer(x) * mask[:, None, :, None]
        if self.spatial_transformer is not None:
            if coords is None:
                raise ValueError("spatial_transformer needs node coordinates in the inputs")
            T = x.shape[1]
            if self.ds_type == "cml":
                enc = torch.cat([self.spatial_transformer(coords[..., 0], coords[..., 1]),
                                 self.spatial_transformer(coords[..., 2], coords[..., 3])], -1)
            else:
                enc = self.spatial_transformer(coords[..., 0], coords[..., 1])
            feats = torch.cat([feats, enc[:, None].expand(-1, T, -1, -1) * mask[:, None, :, None]], -1)
        return feats

    def _fused_ok(self) -> bool:
        g = self.gcn_layer
        return (isinstance(g, GeneralConv) and g.activation == "prelu" and g.use_batch_norm
                and g.aggregate in ("mean", "sum")
                and (self.pooling_type == "selection" or self.aggregation_type in ("mean", "sum")))

    def temporal_input(self, inputs) -> torch.Tensor:
        """Everything before the TimeLayer: per-sensor (CML, XAI SoilNet) [B,T,Ca+F]; network-wide
        SoilNet [B*N,T,F+C]."""
        if self.per_sensor:
            x, anom, adj, mask, anom_pos = inputs[:5]
            coords = inputs[5] if len(inputs) > 5 else None
            feats = self._node_features(x, mask, coords)
            pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
            if self._fused_ok():
                g = self.gcn_layer
                return gcn_pool(feats, adj, mask, anom, anom_pos, g.kernel, g.bias, g.bn_gamma, g.bn_beta,
                                g.prelu_alpha, g.bn_moving_mean, g.bn_moving_variance, self.training, g.aggregate,
                                pooling, g.momentum, g.eps, g.dropout)
            h = self.gcn_layer(feats, adj, mask)
            return torch.cat([anom, pool_nodes(h, mask, anom_pos, pooling)], -1)
        x, adj, mask = inputs[:3]
        coords = inputs[3] if len(inputs) > 3 else None
        feats = self._node_features(x, mask, coords)
        h = self.gcn_layer(feats, adj, mask)
        return graph_reshape(torch.cat([h, x], -1))

    def _soil_fused(self, inputs) -> bool:
        """SoilNet fast path: fused per-node GCN kernel writing the time-major LSTM input."""
        if self.per_sensor or not self._fused_ok():
            return False
        if self.sensors_time_layer is not None or self.spatial_transformer is not None:
            return False
        x = inputs[0]
        g = self.gcn_layer
        return (gcn_node_tm_ok(x, g.kernel, g.aggregate, g.dropout, self.training)
                and self.time_layer.time_major_ok(x, g.out_features + x.shape[-1]))

    def head(self, ts: torch.Tensor) -> torch.Tensor:
        d = self.dropout1(ts)
        d = self.leakyrelu4(self.dense(d))
        d = self.dropout2(d)
        d = self.leakyrelu5(self.dense2(d))
        return self.dense_out(d).squeeze(-1)

    def _cml_time_major(self, inputs) -> bool:
        """CML fast path: the fused GCN + pooling kernel writes the time-major LSTM input."""
        if not self.per_sensor or not self._fused_ok() or self.sensors_time_layer is not None:
            return False
        if self.spatial_transformer is not None or len(inputs) > 5:
            return False
        x, anom = inputs[0], inputs[1]
        g = self.gcn_layer
        pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
        return (gcn_pool_hip_ok(x, g.kernel, g.aggregate, pooling, g.dropout, self.training)
                and self.time_layer.time_major_ok(x, g.out_features + anom.shape[-1]))

    def features(self, inputs) -> torch.Tensor:
        """TimeLayer output rows [R, F] (CML: R = B; SoilNet: R = B*N) - the head's input."""
        if self._cml_time_major(inputs):
            x, anom, adj, mask, anom_pos = inputs[:5]
            g = self.gcn_layer
            pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
            h, M = gcn_pool(x, adj, mask, anom, anom_pos, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha,
                            g.bn_moving_mean, g.bn_moving_variance, self.training, g.aggregate, pooling, g.momentum,
                            g.eps, g.dropout, time_major=True)
            return self.time_layer.forward_time_major(h, M)
        if self._soil_fused(inputs):
            x, adj, mask = inputs[:3]
            g = self.gcn_layer
            h, M = gcn_node_tm(x, adj, mask, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha,
                               g.bn_moving_mean, g.bn_moving_variance, self.training, g.aggregate, g.momentum, g.eps)
            return self.time_layer.forward_time_major(h, M)
        return self.time_layer(self.temporal_input(inputs))

    def head_spec(self):
        """(dense, dense2, dense_out, alpha1, alpha2) when the head is the plain
        Dense-LeakyReLU-Dense-LeakyReLU-Dense stack the fused HIP kernel implements."""
        if self.training and (self.dropout1.rate > 0 or self.dropout2.rate > 0):
            return None
        if any(d.activation not in (None, "linear") for d in (self.dense, self.dense2, self.dense_out)):
            return None
        return self.dense, self.dense2, self.dense_out, self.leakyrelu4.alpha, self.leakyrelu5.alpha

    def fused_loss(self, inputs, y: torch.Tensor, mask: torch.Tensor, w0: float, w1: float, sums=None, hist=None):
        """(loss, logits) through the headed-chain fast path (CML, GPU): the fused GCN kernel
        writes the time-major LSTM input, then ONE kernel runs the whole TimeLayer, the head, the
        weighted BCE and the metric accumulation (``gnnqc.ops.lstm.lstm_chain_head_tm``).
        None when the configuration is not the one those kernels implement."""
        spec = self.head_spec()
        if spec is None or not self.per_sensor or not self._cml_time_major(inputs):
            return None
        if any(d.kernel.shape[1] != 64 for d in spec[:2]) or spec[2].kernel.shape != (64, 1):
            return None
        if not (self.training is False or (self.dropout1.rate == 0 and self.dropout2.rate == 0)):
            return None
        x, anom, adj, mask_n, anom_pos = inputs[:5]
        g = self.gcn_layer
        pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
        h, M = gcn_pool(x, adj, mask_n, anom, anom_pos, g.kernel, g.bias, g.bn_gamma, g.bn_beta, g.prelu_alpha,
                        g.bn_moving_mean, g.bn_moving_variance, self.training, g.aggregate, pooling, g.momentum,
                        g.eps, g.dropout, time_major=True)
        if not self.time_layer.head_chain_ok(h) or spec[0].kernel.shape[0] != 128:
            # (the GCN already ran: finish on the separate-kernel path from its output)
            from ..ops.head import fused_head_loss
            return fused_head_loss(self.time_layer.forward_time_major(h, M), *spec, y, mask, w0, w1, sums, hist)
        yf = y.reshape(-1).float().contiguous()
        mf = mask.reshape(-1).float().contiguous()
        return self.time_layer.forward_time_major_head(h, M, spec[:3], spec[3:], yf, mf, w0, w1, sums, hist)

    def store_fused_ok(self, store) -> bool:
        """Whether :meth:`fused_store_loss` applies: the CML headed-chain configuration, on the GPU,
        with the window store as the input (gather, GCN and pooling fused into one launch)."""
        spec = self.head_spec()
        if spec is None or not self.per_sensor or not self._fused_ok() or self.sensors_time_layer is not None:
            return False
        if self.spatial_transformer is not None:
            return False
        if any(d.kernel.shape[1] != 64 for d in spec[:2]) or spec[2].kernel.shape != (64, 1):
            return False
        if spec[0].kernel.shape[0] != 128 or (self.training and (self.dropout1.rate or self.dropout2.rate)):
            return False
        pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
        return store_gcn_ok(store, self.gcn_layer, self.training, pooling)

    def fused_store_loss(self, store, ids, w0: float, w1: float, sums=None, hist=None):
        """(loss, logits) of a batch given by window ids (or a device cursor into an id table)
        straight from the resident store: ONE launch for the window gather + GeneralConv +
        BatchNorm + PReLU + node pooling + concat (``gcn_fused.hip``), then the headed LSTM chain
        of :meth:`fused_loss`. Check :meth:`store_fused_ok` first."""
        spec = self.head_spec()
        g = self.gcn_layer
        pooling = "selection" if self.pooling_type == "selection" else self.aggregation_type
        # (defer: the GCN forward runs inside the chain forward launch, as its input's producer)
        h, M, y, ym, _ = gcn_pool_from_store(store, ids, g, self.training, pooling, defer=True)
        if not self.time_layer.head_chain_ok(h):
            from ..ops.head import fused_head_loss
            from ..utils.native import hip_ops
            hip_ops().gcn_prod_flush(h)
            return fused_head_loss(self.time_layer.forward_time_major(h, M), *spec, y, ym, w0, w1, sums, hist)
        return self.time_layer.forward_time_major_head(h, M, spec[:3], spec[3:], y, ym, w0, w1, sums, hist)

    def logits(self, inputs) -> torch.Tensor:
        z = self.head(self.features(inputs))
        if not self.per_sensor:
            B, N = inputs[0].shape[0], inputs[0].shape[2]
            z = z.view(B, N)
        return z

    def forward(self, inputs) -> torch.Tensor:
        return torch.sigmoid(self.logits(inputs))

    def regularization_loss(self) -> Optional[torch.Tensor]:
        terms = [m.reg_loss() for m in self.modules() if m is not self and hasattr(m, "reg_loss")]
        terms = [t for t in terms if t is not None]
        return sum(terms) if terms else None


__all__ = ["GCNClassifier", "timeseries_pooling", "graph_reshape", "compute_bf16"]
