"""Sensor neighbourhoods and window indices.

Where the reference materialises one serialized ``SequenceExample`` per minute and
flagged sensor (``libs/preprocessing_functions.py:343-482``), this framework keeps
the (interpolated) raw series of every neighbourhood resident in memory / HBM and
describes a window by an **index** (group, centre time) plus per-window node
validity. Windows are cut on the fly on the GPU (:mod:`gnnqc.data.store`).

Window rules reproduced exactly:

* window = ``[t - timestep_before, t + timestep_after]`` inclusive, skipped if it
  leaves the time axis (``:396-400``);
* CML: skipped if the flagged sensor has a NaN in TL_1 or TL_2 (``:401-403``);
  neighbours with any NaN are dropped (``:404-407``); label = flagged sensor's
  target at ``t``;
* SoilNet: sensors whose target at ``t`` is NaN are dropped (``:459-464``), then
  sensors with any NaN in moisture/temp/battv (``:465-472``); skipped when empty;
  labels are per node.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import numpy as np


@dataclasses.dataclass
class SensorGroup:
    """One graph neighbourhood: CML = flagged link + neighbours, SoilNet = network."""

    group_id: str
    ds_type: str
    sensor_ids: np.ndarray            # [N]
    anomalous_pos: int                # position of the flagged sensor (-1 for SoilNet)
    feature_names: List[str]
    features: np.ndarray              # [N, C, Ttot] float32
    time: np.ndarray                  # [Ttot] datetime64[m]
    target: np.ndarray                # CML [Ttot] bool; SoilNet [N, Ttot] float (NaN = unlabelled)
    distances: np.ndarray             # [N, N]
    depths: Optional[np.ndarray] = None  # [N, N] |depth_i - depth_j| (SoilNet)
    lat: Optional[np.ndarray] = None     # [N] (CML: mid-point)
    lon: Optional[np.ndarray] = None
    coords: Dict[str, np.ndarray] = dataclasses.field(default_factory=dict)
    stats: Dict[str, np.ndarray] = dataclasses.field(default_factory=dict)

    @property
    def n_nodes(self) -> int:
        return int(self.sensor_ids.shape[0])

    @property
    def n_time(self) -> int:
        return int(self.time.shape[0])

    @property
    def per_sensor(self) -> bool:
        """One flagged sensor + its neighbours with that sensor's target series (CML, and the XAI
        generation's SoilNet neighbourhoods) vs a network-wide graph with per-node targets."""
        return self.anomalous_pos >= 0 and np.ndim(self.target) == 1


@dataclasses.dataclass
class WindowIndex:
    """Windows of one group."""

    group: int                      # index into the group list
    center: np.ndarray              # [W] int64 centre time index
    node_valid: np.ndarray          # [W, N] bool
    labels: np.ndarray              # CML [W] int8 ; SoilNet [W, N] int8 (valid where label_valid)
    label_valid: Optional[np.ndarray] = None  # SoilNet [W, N] bool

    @property
    def size(self) -> int:
        return int(self.center.shape[0])


def _nan_window_any(nan_mask: np.ndarray, lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    """For [N, Ttot] bool mask: any NaN in [lo, hi] (inclusive) per window -> [W, N]."""
    csum = np.concatenate([np.zeros((nan_mask.shape[0], 1), np.int64),
                           np.cumsum(nan_mask, axis=1, dtype=np.int64)], axis=1)
    return (csum[:, hi + 1] - csum[:, lo]).T > 0


def build_window_index(group: SensorGroup, group_pos: int, timestep_before: int, timestep_after: int,
                       freq: int, min_date=None, max_date=None) -> WindowIndex:
    tb = int(round(timestep_before / freq))
    ta = int(round(timestep_after / freq))
    T = group.n_time
    t = group.time
    sel = np.ones(T, dtype=bool)
    if min_date is not None:
        sel &= t >= np.datetime64(min_date)
    if max_date is not None:
        sel &= t <= np.datetime64(max_date)
    centers = np.nonzero(sel)[0]
    centers = centers[(centers - tb >= 0) & (centers + ta < T)]
    lo, hi = centers - tb, centers + ta
    nan_any = np.isnan(group.features).any(axis=1)          # [N, Ttot]
    bad = _nan_window_any(nan_any, lo, hi)                   # [W, N]
    if group.per_sensor:
        keep = ~bad[:, group.anomalous_pos]
        tgt = np.asarray(group.target)
        if tgt.dtype.kind == "f":                           # SoilNet (XAI): unlabelled steps are NaN
            keep &= np.isfinite(tgt[centers])
        centers, bad = centers[keep], bad[keep]
        labels = (np.nan_to_num(tgt[centers].astype(np.float64)) > 0.5).astype(np.int8)
        return WindowIndex(group_pos, centers.astype(np.int64), ~bad, labels)
    # SoilNet
    tgt = group.target[:, centers].T                         # [W, N]
    has_target = ~np.isnan(tgt)
    valid = has_target & ~bad
    keep = valid.any(axis=1)
    valid, tgt, centers = valid[keep], tgt[keep], centers[keep]
    labels = np.where(valid, np.nan_to_num(tgt), 0).astype(np.int8)
    return WindowIndex(group_pos, centers.astype(np.int64), valid, labels, valid.copy())


@dataclasses.dataclass
class WindowSet:
    """All windows of a dataset: concatenation of per-group window indices.

    ``keys`` identify the reference's record files: CML ``<sensor>_<YYYY-MM-DD>``
    (one per flagged sensor and day, ``:392-393``), SoilNet ``<YYYY-MM-DD>`` (``:452``).
    """

    groups: List[SensorGroup]
    indices: List[WindowIndex]
    ds_type: str
    timestep_before: int
    timestep_after: int
    freq: int

    @property
    def per_sensor(self) -> bool:
        return bool(self.groups) and all(g.per_sensor for g in self.groups)

    @property
    def seq_len(self) -> int:
        return int((self.timestep_before + self.timestep_after) / self.freq + 1)

    @property
    def n_windows(self) -> int:
        return int(sum(ix.size for ix in self.indices))

    @property
    def max_nodes(self) -> int:
        return int(max(g.n_nodes for g in self.groups))

    def flat(self):
        """(group_of_window [W], local_window [W]) for the concatenated index."""
        g = np.concatenate([np.full(ix.size, i, np.int64) for i, ix in enumerate(self.indices)])
        l = np.concatenate([np.arange(ix.size, dtype=np.int64) for ix in self.indices])
        return g, l

    def window_dates(self) -> np.ndarray:
        """Centre datetime of every window (concatenated order)."""
        return np.concatenate([self.groups[ix.group].time[ix.center] for ix in self.indices])

    def window_days(self) -> np.ndarray:
        return self.window_dates().astype("datetime64[D]")

    def window_keys(self) -> np.ndarray:
        days = self.window_days().astype(str)
        if self.per_sensor:
            gid = np.concatenate([np.full(ix.size, self.groups[ix.group].group_id, dtype=object)
                                  for ix in self.indices])
            return np.array([f"{a}_{b}" for a, b in zip(gid, days)])
        return days

    def labels_flat(self) -> np.ndarray:
        if self.per_sensor:
            return np.concatenate([ix.labels for ix in self.indices])
        return np.concatenate([ix.labels for ix in self.indices], axis=0)

    def group_of(self) -> np.ndarray:
        return self.flat()[0]


__all__ = ["SensorGroup", "WindowIndex", "WindowSet", "build_window_index"]
