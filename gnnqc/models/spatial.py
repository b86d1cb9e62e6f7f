"""XAI-snapshot model extras.

* :class:`SpatialTransformer` - multi-scale sin/cos positional encoding of
  lat/lon followed by ``Dense(units, sigmoid)`` (``xai/libs/create_model.py:415-456``).
  The reference's lon branch reuses ``lat_rad``;
  ``reference_bug=True`` (default) reproduces that so trained behaviour matches,
  ``False`` uses the longitude as intended.
* :class:`SensorsTimeLayer` - a per-node LSTM (or Conv1D + PReLU) over time applied
  before the graph convolution (``:242-293``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .layers import LSTM, Conv1D, Dense, PReLU


class SpatialTransformer(nn.Module):
    def __init__(self, min_scale: float, max_scale: float, grid_scales_number: int, units: int = 32,
                 reference_bug: bool = True):
        super().__init__()
        self.min_scale, self.max_scale, self.n = float(min_scale), float(max_scale), int(grid_scales_number)
        self.g = self.max_scale / self.min_scale
        self.units = units
        self.reference_bug = reference_bug
        self.dense = Dense(4 * self.n, units, activation="sigmoid")

    def encode(self, lat: torch.Tensor, lon: torch.Tensor) -> torch.Tensor:
        lat_rad = lat.reshape(-1, 1) * math.pi / 180.0
        lon_rad = lon.reshape(-1, 1) * math.pi / 180.0
        second = lat_rad if self.reference_bug else lon_rad
        pes = []
        for s in range(self.n):
            denom = self.min_scale * self.g ** (s / max(self.n - 1, 1))
            pe_lat = torch.cat([torch.cos(lat_rad / denom), torch.sin(lat_rad / denom)], 1)
            pe_lon = torch.cat([torch.cos(second / denom), torch.sin(second / denom)], 1)
            pes.append(torch.cat([pe_lon, pe_lat], 1))
        return torch.cat(pes, 1)

    def forward(self, lat: torch.Tensor, lon: torch.Tensor) -> torch.Tensor:
        shape = lat.shape
        return self.dense(self.encode(lat, lon)).reshape(*shape, self.units)


class SensorsTimeLayer(nn.Module):
    """Per-node temporal encoder: [B, T, N, F] -> [B, T, N, units]."""

    def __init__(self, in_features: int, units: int = 16, layer_type: str = "lstm", activation: str = "tanh",
                 kernel_size: int = 5, regularizer=None, compute_bf16: bool = True):
        super().__init__()
        self.units, self.layer_type = units, layer_type
        if layer_type == "lstm":
            self.time_layer = LSTM(in_features, units, activation, True, regularizer, compute_bf16)
        else:
            self.time_layer = Conv1D(in_features, units, kernel_size, regularizer=regularizer, compute_bf16=compute_bf16)
            self.activation = PReLU(units)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, N, Fdim = x.shape
        seq = x.permute(0, 2, 1, 3).reshape(B * N, T, Fdim)
        out = self.time_layer(seq)
        if self.layer_type != "lstm":
            out = self.activation(out)
        return out.reshape(B, N, T, self.units).permute(0, 2, 1, 3)


__all__ = ["SpatialTransformer", "SensorsTimeLayer"]
