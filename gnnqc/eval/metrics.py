"""Classification metrics.

numpy implementations with sklearn semantics (``roc_curve`` / ``auc`` /
``matthews_corrcoef`` / ``precision_score`` / ``recall_score`` / ``accuracy_score``,
used by ``libs/test_model.py``), the hand-rolled helpers of ``libs/metrics.py``
(batch MCC, tp/tn/fp/fn rates, ROC/PR points, MSE), and histogram-based streaming
versions that run on the device (``score_histogram`` kernel) for the 3-decimal MCC
threshold sweep and the Keras ``AUC(num_thresholds=200)`` metric.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np


def confusion(y_true, y_pred) -> Tuple[int, int, int, int]:
    y = np.asarray(y_true).astype(bool).ravel()
    p = np.asarray(y_pred).astype(bool).ravel()
    tp = int(np.sum(y & p))
    tn = int(np.sum(~y & ~p))
    fp = int(np.sum(~y & p))
    fn = int(np.sum(y & ~p))
    return tp, tn, fp, fn


def mcc_from_counts(tp, tn, fp, fn) -> float:
    num = tp * tn - fp * fn
    den = math.sqrt(float(tp + fp) * float(tp + fn) * float(tn + fp) * float(tn + fn))
    return float(num / den) if den > 0 else 0.0


def matthews_corrcoef(y_true, y_pred) -> float:
    return mcc_from_counts(*confusion(y_true, y_pred))


def precision_score(y_true, y_pred) -> float:
    tp, tn, fp, fn = confusion(y_true, y_pred)
    return tp / (tp + fp) if tp + fp > 0 else 0.0


def recall_score(y_true, y_pred) -> float:
    tp, tn, fp, fn = confusion(y_true, y_pred)
    return tp / (tp + fn) if tp + fn > 0 else 0.0


def accuracy_score(y_true, y_pred) -> float:
    tp, tn, fp, fn = confusion(y_true, y_pred)
    n = tp + tn + fp + fn
    return (tp + tn) / n if n else 0.0


def roc_curve(y_true, scores):
    """sklearn.metrics.roc_curve(drop_intermediate=True) semantics."""
    y = np.asarray(y_true).astype(np.float64).ravel()
    s = np.asarray(scores).astype(np.float64).ravel()
    order = np.argsort(s, kind="mergesort")[::-1]
    s, y = s[order], y[order]
    distinct = np.where(np.diff(s))[0]
    idx = np.r_[distinct, y.size - 1]
    tps = np.cumsum(y)[idx]
    fps = 1 + idx - tps
    thr = s[idx]
    # drop collinear points (sklearn drop_intermediate)
    if tps.size > 2:
        opt = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps, thr = fps[opt], tps[opt], thr[opt]
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    thr = np.r_[np.inf, thr]
    fpr = fps / fps[-1] if fps[-1] > 0 else np.full(fps.shape, np.nan)
    tpr = tps / tps[-1] if tps[-1] > 0 else np.full(tps.shape, np.nan)
    return fpr, tpr, thr


def auc(x, y) -> float:
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    d = np.diff(x)
    direction = -1.0 if np.all(d <= 0) and np.any(d < 0) else 1.0
    return float(direction * np.trapezoid(y, x))


def roc_auc_score(y_true, scores) -> float:
    """Exact ROC-AUC (Mann-Whitney with tie correction)."""
    y = np.asarray(y_true).astype(bool).ravel()
    s = np.asarray(scores, dtype=np.float64).ravel()
    n1, n0 = int(y.sum()), int((~y).sum())
    if n1 == 0 or n0 == 0:
        return float("nan")
    from scipy.stats import rankdata
    r = rankdata(s)
    return float((r[y].sum() - n1 * (n1 + 1) / 2) / (n1 * n0))


def select_threshold(predictions, labels, verbose: bool = True):
    """argmax-MCC threshold over ``np.unique(np.round(p, 3))`` (``libs/test_model.py:9-17``).

    Vectorised: one sort + cumulative counts instead of one sklearn call per
    candidate threshold. Ties resolve to the first (smallest) threshold like
    ``np.argmax``.
    """
    p = np.asarray(predictions, dtype=np.float64).ravel()
    y = np.asarray(labels).astype(bool).ravel()
    cands = np.unique(np.round(p, 3))
    order = np.argsort(p)
    ps, ys = p[order], y[order]
    # number of samples with p <= c (predicted negative at threshold c since rule is p > c)
    k = np.searchsorted(ps, cands, side="right")
    pos_le = np.r_[0, np.cumsum(ys)][k]
    neg_le = k - pos_le
    P, N = int(y.sum()), int((~y).sum())
    fn = pos_le
    tn = neg_le
    tp = P - fn
    fp = N - tn
    num = tp * tn - fp * fn
    den = np.sqrt((tp + fp).astype(np.float64) * (tp + fn) * (tn + fp) * (tn + fn))
    mcc = np.where(den > 0, num / np.where(den > 0, den, 1), 0.0)
    i = int(np.argmax(mcc))
    if verbose:
        print("Max MCC: {:.3f} for threshold: {:.3f}".format(mcc[i], cands[i]))
    return float(cands[i])


# ------------------------------------------------------------ histogram based
def threshold_sweep_from_hist(hist: np.ndarray):
    """From [2, bins] (neg, pos) counts with bin = rint(p*(bins-1)): per-threshold
    confusion counts for thresholds c_k = k/(bins-1) and rule ``p > c_k``."""
    neg, pos = np.asarray(hist[0], np.float64), np.asarray(hist[1], np.float64)
    P, N = pos.sum(), neg.sum()
    fn = np.cumsum(pos)      # p-bin <= k -> negative
    tn = np.cumsum(neg)
    return P - fn, tn, N - tn, fn          # tp, tn, fp, fn


def mcc_threshold_from_hist(hist: np.ndarray):
    tp, tn, fp, fn = threshold_sweep_from_hist(hist)
    present = (np.asarray(hist[0]) + np.asarray(hist[1])) > 0
    num = tp * tn - fp * fn
    den = np.sqrt((tp + fp) * (tp + fn) * (tn + fp) * (tn + fn))
    mcc = np.where(den > 0, num / np.where(den > 0, den, 1), 0.0)
    mcc = np.where(present, mcc, -np.inf)
    i = int(np.argmax(mcc))
    return i / (hist.shape[1] - 1), float(mcc[i])


def auc_from_hist(hist: np.ndarray) -> float:
    """ROC-AUC treating scores inside a bin as tied (trapezoid rule)."""
    neg, pos = np.asarray(hist[0], np.float64)[::-1], np.asarray(hist[1], np.float64)[::-1]
    P, N = pos.sum(), neg.sum()
    if P == 0 or N == 0:
        return float("nan")
    tpr = np.r_[0, np.cumsum(pos)] / P
    fpr = np.r_[0, np.cumsum(neg)] / N
    return float(np.trapezoid(tpr, fpr))


def keras_metrics_from_counts(tp, tn, fp, fn) -> Dict[str, float]:
    return {
        "recall": tp / (tp + fn) if tp + fn else 0.0,
        "precision": tp / (tp + fp) if tp + fp else 0.0,
        "binary_accuracy": (tp + tn) / max(tp + tn + fp + fn, 1),
        "tp": float(tp), "fp": float(fp), "tn": float(tn), "fn": float(fn),
    }


# ----------------------------------------------- libs/metrics.py helpers (numpy)
def matthews_correlation(y_true, y_pred, eps: float = 1e-7) -> float:
    """Batch-wise MCC with rounding (``libs/metrics.py:7-31``)."""
    yp = np.round(np.clip(y_pred, 0, 1))
    yt = np.round(np.clip(y_true, 0, 1))
    tp = np.sum(yt * yp)
    tn = np.sum((1 - yt) * (1 - yp))
    fp = np.sum((1 - yt) * yp)
    fn = np.sum(yt * (1 - yp))
    return float((tp * tn - fp * fn) / (np.sqrt((tp + fp) * (tp + fn) * (tn + fp) * (tn + fn)) + eps))


def tp_rate(y_true, y_pred):
    yp, yt = np.round(y_pred), np.round(y_true)
    return float(np.sum(yt * yp) / max(np.sum(yt), 1e-12))


def tn_rate(y_true, y_pred):
    yp, yt = np.round(y_pred), np.round(y_true)
    return float(np.sum((1 - yt) * (1 - yp)) / max(np.sum(1 - yt), 1e-12))


def fp_rate(y_true, y_pred):
    yp, yt = np.round(y_pred), np.round(y_true)
    return float(np.sum((1 - yt) * yp) / max(np.sum(1 - yt), 1e-12))


def fn_rate(y_true, y_pred):
    yp, yt = np.round(y_pred), np.round(y_true)
    return float(np.sum(yt * (1 - yp)) / max(np.sum(yt), 1e-12))


def precision_recall_curve(y_true, scores):
    y = np.asarray(y_true).astype(np.float64).ravel()
    s = np.asarray(scores, np.float64).ravel()
    order = np.argsort(s, kind="mergesort")[::-1]
    s, y = s[order], y[order]
    idx = np.r_[np.where(np.diff(s))[0], y.size - 1]
    tps = np.cumsum(y)[idx]
    fps = 1 + idx - tps
    prec = tps / np.maximum(tps + fps, 1)
    rec = tps / max(tps[-1], 1)
    return np.r_[prec[::-1], 1.0], np.r_[rec[::-1], 0.0], s[idx][::-1]


def mse(y_true, y_pred) -> float:
    return float(np.mean((np.asarray(y_true, np.float64) - np.asarray(y_pred, np.float64)) ** 2))


def mcc_metric(y_true, y_pred, threshold: float = 0.5) -> float:
    """``libs/metrics.py:194-211``: MCC of thresholded predictions."""
    return matthews_corrcoef(np.asarray(y_true).ravel() > 0.5, np.asarray(y_pred).ravel() > threshold)


__all__ = [
    "confusion", "mcc_from_counts", "matthews_corrcoef", "precision_score", "recall_score", "accuracy_score",
    "roc_curve", "auc", "roc_auc_score", "select_threshold", "threshold_sweep_from_hist",
    "mcc_threshold_from_hist", "auc_from_hist", "keras_metrics_from_counts", "matthews_correlation", "tp_rate",
    "tn_rate", "fp_rate", "fn_rate", "precision_recall_curve", "mse", "mcc_metric",
]
