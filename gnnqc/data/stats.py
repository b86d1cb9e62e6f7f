"""Normalisation statistics.

``calculate_statistics`` of the reference (``libs/preprocessing_functions.py:123-173``)
computes, per sensor and feature, global mean/std/min/max/median over time and
**trailing** rolling mean/std/median over ``window_length`` samples with
``min_periods=1`` (xarray ``rolling(time=w, min_periods=1)``; NaNs skipped, std with
ddof=0). The rolling median dominates preprocessing cost, so it runs in the native
host library (multithreaded C++, ``csrc/host/gnnqc_host.cpp``); pandas' rolling
implementation is the fallback and the test oracle.
"""
from __future__ import annotations

import os
from typing import Dict, Sequence

import numpy as np

from ..utils.native import host_lib


def rolling_stats(x: np.ndarray, window: int, min_periods: int = 1, which=("mean", "std", "median"),
                  nthreads: int | None = None, backend: str = "auto") -> Dict[str, np.ndarray]:
    """Trailing rolling statistics along the last axis of ``x`` ([..., T])."""
    x = np.asarray(x)
    shape = x.shape
    flat = np.ascontiguousarray(x.reshape(-1, shape[-1]), dtype=np.float32)
    rows, n = flat.shape
    out = {k: np.empty((rows, n), dtype=np.float32) for k in which}
    lib = host_lib() if backend in ("auto", "native") else None
    if backend == "native" and lib is None:
        raise RuntimeError("native host library not built")
    if lib is not None:
        ptr = lambda k: out[k].ctypes.data if k in out else None  # noqa: E731
        lib.gq_rolling_stats(flat, rows, n, int(window), int(min_periods), ptr("mean"), ptr("std"),
                             ptr("median"), int(nthreads or min(os.cpu_count() or 1, 16)))
    else:
        import pandas as pd
        df = pd.DataFrame(flat.T.astype(np.float64))
        r = df.rolling(window=int(window), min_periods=int(min_periods))
        if "mean" in out:
            out["mean"] = r.mean().to_numpy().T.astype(np.float32)
        if "std" in out:
            out["std"] = r.std(ddof=0).to_numpy().T.astype(np.float32)
        if "median" in out:
            out["median"] = r.median().to_numpy().T.astype(np.float32)
    return {k: v.reshape(shape) for k, v in out.items()}


def global_stats(x: np.ndarray) -> Dict[str, np.ndarray]:
    """NaN-skipping mean/std(ddof=0)/min/max/median over the last axis."""
    with np.errstate(all="ignore"):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            return {
                "mean": np.nanmean(x, axis=-1).astype(np.float32),
                "std": np.nanstd(x, axis=-1).astype(np.float32),
                "min": np.nanmin(x, axis=-1).astype(np.float32),
                "max": np.nanmax(x, axis=-1).astype(np.float32),
                "median": np.nanmedian(x, axis=-1).astype(np.float32),
            }


def calculate_statistics(features: Dict[str, np.ndarray], window_length: int,
                         which_rolling: Sequence[str] = ("mean", "std", "median")) -> Dict[str, np.ndarray]:
    """Reference-named statistics for each feature array ``[sensor, time]``.

    Returns keys like ``TL_1_mean``, ``TL_1_rolling_median`` (same names the reference
    stores on the xarray Dataset).
    """
    out: Dict[str, np.ndarray] = {}
    for name, arr in features.items():
        g = global_stats(arr)
        for k, v in g.items():
            out[f"{name}_{k}"] = v
        r = rolling_stats(arr, window_length, 1, which=tuple(which_rolling))
        for k, v in r.items():
            out[f"{name}_rolling_{k}"] = v
    return out


__all__ = ["rolling_stats", "global_stats", "calculate_statistics"]
