"""Train/val/test splits and k-fold CV.

Splits operate on window "files" exactly like the reference operates on TFRecord
file names:

* CML (``libs/preprocessing_functions.py:485-563``): chronological by unique day.
  ``n_train = round(days * train_fraction)``; train = days before
  ``day[n_train - ceil((tb+ta)/1440)]``; val = ``[day[n_train], day[n_train+n_val - gap])``;
  test = days from ``day[n_train + n_val]`` on (the gap keeps windows from
  straddling two splits).
* SoilNet: random months for train/val/test; within a month that is not followed
  by an adjacent month of the same split, days too close to the month end are
  trimmed (``:525-553``). Seeded (the reference's ``random.sample`` is unseeded
  unless an earlier call seeded the module RNG - SURVEY §5.11 item 5).
* k-fold (``xai/libs/preprocessing_functions.py:804-836``): the ordered file
  numbers are cut into ``split_numb`` contiguous chunks (``np.array_split``); chunk
  ``k`` is the test fold, the rest trains. ``gap_days`` optionally drops days of the
  training folds that touch the test fold (off = reference behaviour).
"""
from __future__ import annotations

import math
import random as _random
from typing import Tuple

import numpy as np


def _gap_days(timestep_before: int, timestep_after: int) -> int:
    return int(np.ceil((timestep_before + timestep_after) / (60 * 24)))


def chronological_split(days: np.ndarray, train_fraction: float, val_fraction: float,
                        timestep_before: int, timestep_after: int):
    """Boolean masks (train, val, test) over windows from their day stamps."""
    days = np.asarray(days).astype("datetime64[D]")
    u = np.unique(days)
    n = len(u)
    gap = _gap_days(timestep_before, timestep_after)
    n_tr = int(np.round(n * train_fraction))
    n_va = int(np.round(n * val_fraction))
    if n_tr + n_va >= n or n_tr - gap < 0:
        raise ValueError(f"not enough days ({n}) for the requested split")
    train_max = u[n_tr]
    train_max_removed = u[n_tr - gap]
    val_max = u[n_tr + n_va]
    val_max_removed = u[n_tr + n_va - gap]
    tr = days < train_max_removed
    va = (days >= train_max) & (days < val_max_removed)
    te = days >= val_max
    return tr, va, te


def monthly_random_split(days: np.ndarray, train_fraction: float, val_fraction: float,
                         timestep_before: int, timestep_after: int, seed: int = 44):
    days = np.asarray(days).astype("datetime64[D]")
    months = days.astype("datetime64[M]")
    um = np.unique(months)
    n = len(um)
    rng = _random.Random(seed)
    n_tr = int(np.round(n * train_fraction))
    n_va = int(np.round(n * val_fraction))
    idx = list(range(n))
    tr_i = sorted(rng.sample(idx, n_tr))
    rest = sorted(set(idx) - set(tr_i))
    va_i = sorted(rng.sample(rest, min(n_va, len(rest))))
    te_i = sorted(set(rest) - set(va_i))
    gap = _gap_days(timestep_before, timestep_after)
    month_end = (months + np.timedelta64(1, "M")).astype("datetime64[D]") - np.timedelta64(1, "D")
    keep = np.ones(days.shape, bool)
    for sel in (tr_i, te_i, va_i):
        ms = um[sel]
        for j, m in enumerate(ms):
            nxt_adjacent = j + 1 < len(ms) and (ms[j + 1] - m) == np.timedelta64(1, "M")
            if not nxt_adjacent:
                in_m = months == m
                keep &= ~(in_m & (days > month_end - np.timedelta64(gap, "D")))
    tr = np.isin(months, um[tr_i]) & keep
    va = np.isin(months, um[va_i]) & keep
    te = np.isin(months, um[te_i]) & keep
    return tr, va, te


def kfold_split(file_numbers: np.ndarray, split_numb: int, test_split: int, gap: int = 0):
    """Contiguous k-fold over ordered file numbers -> (train_mask, test_mask)."""
    fn = np.asarray(file_numbers)
    u = np.arange(fn.min(), fn.max() + 1)
    chunks = np.array_split(u, split_numb)
    test_ids = chunks[test_split]
    te = np.isin(fn, test_ids)
    tr = ~te
    if gap > 0 and test_ids.size:
        lo, hi = test_ids.min(), test_ids.max()
        near = ((fn >= lo - gap) & (fn < lo)) | ((fn > hi) & (fn <= hi + gap))
        tr &= ~near
    return tr, te


def day_numbers(days: np.ndarray) -> np.ndarray:
    d = np.asarray(days).astype("datetime64[D]")
    return (d - d.min()).astype(np.int64)


__all__ = ["chronological_split", "monthly_random_split", "kfold_split", "day_numbers"]
