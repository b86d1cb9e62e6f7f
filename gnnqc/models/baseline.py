"""Graph-less baseline (``libs/create_model.py:261-377``).

The same temporal stack + dense head, fed only with the flagged sensor (CML,
input ``[B, T, 2]``) or with every SoilNet node as its own sequence. Config comes
from ``model_config.baseline_model`` (type lstm|cnn, n_stacks, filter_1_size,
pool_size, kernel_size, alpha, dense_layer_units, activation, regularizer,
XAI ``dropout``).

Reference quirk kept visible: a non-null
``baseline_model.regularizer`` raises NameError in the reference; here it works
and applies an L2 penalty.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from ..config import freq_minutes
from .gcn import compute_bf16, graph_reshape
from .layers import Dense, Dropout, LeakyReLU
from .timelayer import TimeLayer


class BaselineClassifier(nn.Module):
    def __init__(self, model_config, preprocessing_config):
        super().__init__()
        mc, pc = model_config, preprocessing_config
        self.model_config = mc
        self.ds_type = pc["ds_type"]
        # per-sensor data (CML; XAI SoilNet, xai/libs/preprocessing_functions.py:791-802): the model
        # sees the flagged sensor's series only; network-wide SoilNet: every node's series
        self.per_sensor = bool(pc.get("per_sensor", self.ds_type == "cml"))
        self.freq = freq_minutes(self.ds_type)
        self.input_feature_numb = 2 if self.ds_type == "cml" else 3
        self.timestep_before, self.timestep_after = int(pc["timestep_before"]), int(pc["timestep_after"])
        self.batch_size = int(pc["batch_size"])
        self.normalization = pc.get("normalization") or ("rolling_median" if self.ds_type == "cml" else "scale_range")
        self.register_buffer("model_info", torch.tensor([self.timestep_before, self.timestep_after,
                                                         self.batch_size, self.freq], dtype=torch.int32))
        bm = mc["baseline_model"]
        self.layer_type = bm.get("type", "lstm")
        self.time_layer = TimeLayer(self.input_feature_numb, bm.get("filter_1_size", 16), bm.get("n_stacks", 2),
                                    "cnn" if self.layer_type == "cnn" else "lstm", bm.get("activation", "tanh"),
                                    bm.get("kernel_size"), bm.get("regularizer"), bm.get("pool_size", 3),
                                    bm.get("alpha", 0.3), cnn_stack_pool=bm.get("pool_size", 3),
                                    compute_bf16=compute_bf16(mc))
        units = bm.get("dense_layer_units", 64)
        rate = bm.get("dropout") or 0.0
        self.dense1 = Dense(self.time_layer.out_features, units)
        self.leakyrelu4 = LeakyReLU(bm.get("alpha", 0.3))
        self.dropout1 = Dropout(rate)
        self.dense2 = Dense(units, units)
        self.leakyrelu5 = LeakyReLU(bm.get("alpha", 0.3))
        self.dropout2 = Dropout(rate)
        self.dense_out = Dense(units, 1)

    def temporal_input(self, inputs) -> torch.Tensor:
        if self.per_sensor:
            return inputs[0]
        x = inputs[0]
        return graph_reshape(x)

    def head(self, ts):
        d = self.dropout1(self.leakyrelu4(self.dense1(ts)))
        d = self.dropout2(self.leakyrelu5(self.dense2(d)))
        return self.dense_out(d).squeeze(-1)

    def features(self, inputs) -> torch.Tensor:
        return self.time_layer(self.temporal_input(inputs))

    def head_spec(self):
        if self.training and (self.dropout1.rate > 0 or self.dropout2.rate > 0):
            return None
        if any(d.activation not in (None, "linear") for d in (self.dense1, self.dense2, self.dense_out)):
            return None
        return self.dense1, self.dense2, self.dense_out, self.leakyrelu4.alpha, self.leakyrelu5.alpha

    def logits(self, inputs) -> torch.Tensor:
        z = self.head(self.time_layer(self.temporal_input(inputs)))
        if not self.per_sensor:
            x = inputs[0]
            z = z.view(x.shape[0], x.shape[2])
        return z

    def forward(self, inputs) -> torch.Tensor:
        return torch.sigmoid(self.logits(inputs))

    def regularization_loss(self) -> Optional[torch.Tensor]:
        terms = [m.reg_loss() for m in self.modules() if m is not self and hasattr(m, "reg_loss")]
        terms = [t for t in terms if t is not None]
        return sum(terms) if terms else None


__all__ = ["BaselineClassifier"]
