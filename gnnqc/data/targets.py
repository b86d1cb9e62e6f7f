"""Per-minute anomaly targets.

* CML: a minute is anomalous if at least ``min_experts`` of the 4 experts flagged
  it under any flag variable (``libs/preprocessing_functions.py:11-17``).
* SoilNet: 0 where ``moisture_flag_OK`` and 0 < moisture < 100, 1 where
  ``moisture_flag_Manual`` and in range, NaN otherwise
  (``libs/preprocessing_functions.py:18-21``). The XAI snapshot's "all flags"
  mode (``xai/libs/preprocessing_functions.py:1035-1043``) is ``flags_type='all'``.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from .raw_io import SensorData

CML_FLAG_VARS = ("Jump", "Dew", "Fluctuation", "Unknown anomaly")


def create_target(ds: SensorData, flag_vars: Sequence[str] = CML_FLAG_VARS, min_experts: int = 3,
                  ds_type: str = "cml", flags_type: str = "manual", sensors=None) -> np.ndarray:
    """``sensors`` (CML): positions along ``sensor_id`` to evaluate (rows of the result, in that
    order); None = every sensor."""
    if ds_type == "cml":
        per_var = []
        for name in flag_vars:
            v = ds[name]
            ax = v.dims.index("expert")
            d = np.asarray(v.data)
            if sensors is not None:
                d = np.take(d, np.asarray(sensors, dtype=np.int64), axis=v.dims.index("sensor_id"))
            per_var.append(d.astype(np.int32).sum(axis=ax) >= min_experts)
        return np.any(np.stack(per_var, axis=0), axis=0)
    if ds_type == "soilnet":
        m = np.asarray(ds["moisture"].data, dtype=np.float64)
        if flags_type == "manual":
            in_range = (m > 0) & (m < 100)
            target = np.where(np.asarray(ds["moisture_flag_OK"].data, bool) & in_range, 0.0, np.nan)
            target[np.asarray(ds["moisture_flag_Manual"].data, bool) & in_range] = 1.0
            return target
        # 'all' flags: labelled points are 0 unless not OK
        no_label = np.asarray(ds["moisture_flag_no_label"].data, bool)
        ok = np.asarray(ds["moisture_flag_OK"].data, bool)
        target = np.where(no_label, np.nan, 0.0)
        target[(~no_label) & (~ok)] = 1.0
        return target
    raise ValueError(f"unknown ds_type {ds_type}")


__all__ = ["create_target", "CML_FLAG_VARS"]
