"""Keras-semantics building blocks in PyTorch (weights stored in Keras layout).

Weights keep the Keras shapes so checkpoints map 1:1 onto the reference's
TensorBundle variables: Dense kernel ``[in, out]``, LSTM kernel
``[in, 4H]`` / recurrent kernel ``[H, 4H]`` / bias ``[4H]`` (gate order i,f,c,o),
Conv1D kernel ``[k, in, out]``. Initialisers follow the decoded Keras configs
(SURVEY §5.10): GlorotUniform kernels, Orthogonal recurrent kernels, zero biases
with unit forget bias, zero PReLU alpha.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.lstm import lstm_layer


def glorot_uniform_(t: torch.Tensor, fan_in: int, fan_out: int, gen: Optional[torch.Generator] = None):
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-limit, limit, generator=gen)
    return t


def orthogonal_(t: torch.Tensor, gain: float = 1.0, gen: Optional[torch.Generator] = None):
    """Keras Orthogonal for a 2-D [rows, cols] kernel."""
    rows, cols = t.shape
    a = torch.randn(max(rows, cols), min(rows, cols), generator=gen, dtype=torch.float64)
    q, r = torch.linalg.qr(a)
    q = q * torch.sign(torch.diagonal(r))
    if rows < cols:
        q = q.t()
    with torch.no_grad():
        t.copy_((gain * q[:rows, :cols]).to(t.dtype))
    return t


class Dense(nn.Module):
    def __init__(self, in_features: int, units: int, activation: Optional[str] = None, use_bias: bool = True,
                 regularizer: Optional[float] = None):
        super().__init__()
        self.kernel = nn.Parameter(torch.empty(in_features, units))
        self.bias = nn.Parameter(torch.zeros(units)) if use_bias else None
        self.activation = activation
        self.regularizer = regularizer
        glorot_uniform_(self.kernel, in_features, units)

    def forward(self, x):
        y = x @ self.kernel
        if self.bias is not None:
            y = y + self.bias
        return apply_activation(y, self.activation)

    def reg_loss(self):
        return self.regularizer * (self.kernel ** 2).sum() if self.regularizer else None


def apply_activation(x, name, alpha: float = 0.3):
    if name in (None, "linear"):
        return x
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "tanh":
        return torch.tanh(x)
    if name == "relu":
        return torch.relu(x)
    if name == "leaky_relu":
        return F.leaky_relu(x, alpha)
    if name == "elu":
        return F.elu(x)
    if name == "softmax":
        return torch.softmax(x, -1)
    raise ValueError(f"unknown activation {name}")


class PReLU(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.alpha = nn.Parameter(torch.zeros(channels))

    def forward(self, x):
        return torch.where(x > 0, x, self.alpha * x)


class LeakyReLU(nn.Module):
    def __init__(self, alpha: float = 0.3):
        super().__init__()
        self.alpha = float(alpha)

    def forward(self, x):
        return F.leaky_relu(x, self.alpha)


class LSTM(nn.Module):
    """Keras ``layers.LSTM(units, activation, return_sequences)`` on [M, T, in]."""

    def __init__(self, in_features: int, units: int, activation: str = "tanh", return_sequences: bool = True,
                 regularizer: Optional[float] = None, compute_bf16: bool = True):
        super().__init__()
        self.units = units
        self.activation = activation
        self.return_sequences = return_sequences
        self.regularizer = regularizer
        self.compute_bf16 = compute_bf16
        self.kernel = nn.Parameter(torch.empty(in_features, 4 * units))
        self.recurrent_kernel = nn.Parameter(torch.empty(units, 4 * units))
        self.bias = nn.Parameter(torch.zeros(4 * units))
        glorot_uniform_(self.kernel, in_features, 4 * units)
        orthogonal_(self.recurrent_kernel)
        with torch.no_grad():
            self.bias[units:2 * units] = 1.0   # unit_forget_bias

    def forward(self, x):
        return lstm_layer(x, self.kernel, self.recurrent_kernel, self.bias, self.return_sequences, self.activation,
                          bf16=self.compute_bf16)

    def reg_loss(self):
        if not self.regularizer:
            return None
        return self.regularizer * ((self.kernel ** 2).sum() + (self.recurrent_kernel ** 2).sum())


class Conv1D(nn.Module):
    """Keras Conv1D(filters, kernel_size, padding='same') on [M, T, in] (channels last).

    ``forward_act`` fuses the following LeakyReLU (and optionally the
    GlobalAveragePooling1D) into one HIP kernel on the GPU (``gnnqc.ops.conv``)."""

    def __init__(self, in_features: int, filters: int, kernel_size: int, padding: str = "same",
                 regularizer: Optional[float] = None, compute_bf16: bool = True):
        super().__init__()
        self.kernel_size = int(kernel_size)
        self.padding = padding
        self.regularizer = regularizer
        self.compute_bf16 = compute_bf16
        self.kernel = nn.Parameter(torch.empty(self.kernel_size, in_features, filters))
        self.bias = nn.Parameter(torch.zeros(filters))
        glorot_uniform_(self.kernel, self.kernel_size * in_features, self.kernel_size * filters)

    def forward(self, x):
        return self.forward_act(x, 1.0)

    def forward_act(self, x, alpha: float = 1.0, gap: bool = False):
        from ..ops.conv import conv1d_act, conv1d_act_eager
        if self.padding == "same" and self.compute_bf16:
            return conv1d_act(x, self.kernel, self.bias, alpha, gap)
        if self.padding == "same":
            return conv1d_act_eager(x, self.kernel, self.bias, alpha, gap)
        y = F.conv1d(x.transpose(1, 2), self.kernel.permute(2, 1, 0), self.bias).transpose(1, 2)  # 'valid'
        if alpha != 1.0:
            y = F.leaky_relu(y, alpha)
        return y.mean(1) if gap else y

    def reg_loss(self):
        return self.regularizer * (self.kernel ** 2).sum() if self.regularizer else None


class MaxPooling1D(nn.Module):
    def __init__(self, pool_size: int = 3):
        super().__init__()
        self.pool_size = int(pool_size)

    def forward(self, x):                           # [M, T, C], valid padding, stride = pool
        from ..ops.pool import max_pool1d
        return max_pool1d(x, self.pool_size)


class GlobalAveragePooling1D(nn.Module):
    def forward(self, x):
        return x.mean(1)


class BatchNormalization(nn.Module):
    """Keras BatchNormalization(axis=-1, momentum=.99, epsilon=1e-3) state."""

    def __init__(self, channels: int, momentum: float = 0.99, eps: float = 1e-3):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))
        self.momentum, self.eps = momentum, eps


class Dropout(nn.Module):
    def __init__(self, rate: float):
        super().__init__()
        self.rate = float(rate or 0.0)

    def forward(self, x):
        return F.dropout(x, self.rate, self.training) if self.rate > 0 else x


__all__ = ["Dense", "PReLU", "LeakyReLU", "LSTM", "Conv1D", "MaxPooling1D", "GlobalAveragePooling1D",
           "BatchNormalization", "Dropout", "glorot_uniform_", "orthogonal_", "apply_activation"]
