"""Gap-limited linear interpolation along time.

Matches ``xarray.DataArray.interpolate_na(dim="time", max_gap=..., method="linear")``
as used by ``libs/preprocessing_functions.py:67-76``: a run of NaNs is filled only if
the distance between the valid samples bounding it is ``<= max_gap``; leading and
trailing NaNs are never filled. Vectorised over all sensors at once.
"""
from __future__ import annotations

import numpy as np


def interpolate_gaps(values: np.ndarray, times: np.ndarray, max_gap) -> np.ndarray:
    """values: [..., T] float; times: [T] datetime64 or numeric; max_gap: timedelta/number."""
    x = np.array(values, dtype=np.float64, copy=True)
    shape = x.shape
    x = x.reshape(-1, shape[-1])
    if np.issubdtype(np.asarray(times).dtype, np.datetime64):
        t = np.asarray(times).astype("datetime64[s]").astype(np.int64).astype(np.float64)
        if isinstance(max_gap, str):
            max_gap = np.timedelta64(int(max_gap.rstrip("min")), "m") if max_gap.endswith("min") else np.timedelta64(max_gap)
        gap = np.asarray(max_gap).astype("timedelta64[s]").astype(np.int64).astype(np.float64)
    else:
        t = np.asarray(times, dtype=np.float64)
        gap = float(max_gap)
    T = x.shape[1]
    idx = np.arange(T)
    valid = ~np.isnan(x)
    # previous valid index (or -1) and next valid index (or T) for every position
    prev = np.where(valid, idx[None, :], -1)
    prev = np.maximum.accumulate(prev, axis=1)
    nxt = np.where(valid, idx[None, :], T)
    nxt = np.minimum.accumulate(nxt[:, ::-1], axis=1)[:, ::-1]
    fill = (~valid) & (prev >= 0) & (nxt < T)
    r, c = np.nonzero(fill)
    if r.size:
        p = prev[r, c]
        n = nxt[r, c]
        tp, tn, tc = t[p], t[n], t[c]
        ok = (tn - tp) <= gap
        r, c, p, n, tp, tn, tc = r[ok], c[ok], p[ok], n[ok], tp[ok], tn[ok], tc[ok]
        w = (tc - tp) / (tn - tp)
        x[r, c] = x[r, p] * (1 - w) + x[r, n] * w
    return x.reshape(shape)


__all__ = ["interpolate_gaps"]
