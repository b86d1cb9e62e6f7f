"""Evaluation API of ``libs/test_model.py``.

* :func:`select_threshold` - argmax-MCC over ``np.unique(round(p, 3))``;
* :func:`calculate_threshold` - predict the validation split and pick the threshold
  (or 0.5 when ``calculate_threshold`` is off); also returns the anomaly index
  (``tb`` for CML, ``tb/freq`` for SoilNet) from ``model.model_info``;
* :func:`calculate_metrics` - MCC, precision, recall, accuracy, ROC curve + AUC,
  with the ROC figure written to ``plotting.outdir``.
"""
from __future__ import annotations

import os

import numpy as np

from .metrics import (accuracy_score, auc, matthews_corrcoef, precision_score, recall_score, roc_curve,
                      select_threshold)


def anomaly_index(model, ds_type: str) -> int:
    info = [int(x) for x in model.model_info.tolist()]
    return int(info[0] / info[-1]) if ds_type == "soilnet" else int(info[0])


def calculate_threshold(model_config, preproc_config, val_loader, model, baseline: bool = False, store=None):
    from ..train.engine import flatten_predictions, predict
    ds_type = preproc_config["ds_type"]
    idx = anomaly_index(model, ds_type)
    if model_config.get("calculate_threshold", True):
        store = store or val_loader.store
        r = flatten_predictions(predict(model, store, val_loader, baseline))
        thr = select_threshold(r["p"], r["y"])
    else:
        thr = 0.5
    return thr, idx


def calculate_metrics(anomaly_flags_true, anomaly_flags_pred, predictions, model_config=None, threshold=0.5,
                      baseline: bool = False, outpath=None, verbose: bool = True):
    y = np.asarray(anomaly_flags_true).ravel()
    yp = np.asarray(anomaly_flags_pred).ravel()
    mcc = matthews_corrcoef(y, yp)
    precision = precision_score(y, yp)
    recall = recall_score(y, yp)
    accuracy = accuracy_score(y, yp)
    fpr, tpr, thr = roc_curve(y, predictions)
    auc_score = auc(fpr, tpr)
    if verbose:
        print("MCC: {:.3f}\nPrecision: {:.3f}\nRecall: {:.3f}\nAccuracy: {:.3f}\nAUC: {:.3f} ".format(
            mcc, precision, recall, accuracy, auc_score))
    if model_config is not None and outpath is not False:
        try:
            from ..viz import plot_roc_curves
            if outpath is None:
                outdir = (model_config.get("plotting") or {}).get("outdir", "plots")
                outpath = os.path.join(outdir, "ROC_curve_baseline.png" if baseline else "ROC_curve.png")
            plot_roc_curves([fpr], [tpr], model_config, [thr], [threshold], outpath,
                            ["baseline" if baseline else "GCN"])
        except Exception as e:   # plotting must never break evaluation
            if verbose:
                print(f"ROC plot skipped: {e}")
    return mcc, precision, recall, accuracy, auc_score, fpr, tpr, thr


__all__ = ["select_threshold", "calculate_threshold", "calculate_metrics", "anomaly_index"]
