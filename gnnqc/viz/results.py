"""Evaluation plots (reference ``libs/visualize.py``).

* :func:`plot_roc_curves` - several ROC curves + the chosen-threshold markers
  (``:17-47``);
* :func:`extract_target_info` - sensor ids, centre dates, true flags (and series) of
  a window-id list (``:50-92``) straight from the window index - no dataset replay;
* :func:`timeseries_figure` - one classified window (``:95-149``);
* :func:`plot_classified_samples` - predict + plot validation windows (``:152-177``);
* :func:`plot_results` - per-sensor strips of TP/TN/FP/FN along time, optional
  GCN-vs-baseline comparison (``:180-417``).

All figures are written with the non-interactive Agg backend.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np

import matplotlib

matplotlib.use("Agg")
import matplotlib.dates as mdates  # noqa: E402
import matplotlib.patches as mpatches  # noqa: E402
import matplotlib.pyplot as plt  # noqa: E402

from ..eval.metrics import auc as _auc  # noqa: E402

COLOR_TAB = ["indianred", "teal", "darkorange", "slateblue"]
LINE_COLORS = ["teal", "deepskyblue"]
OUTCOME_COLORS = {(1, 1): "green", (0, 0): "blue", (1, 0): "orange", (0, 1): "red"}   # (pred, true)


def _outdir(model_config, default="plots"):
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    d = pl.get("outdir", default)
    os.makedirs(d, exist_ok=True)
    return d


def plot_roc_curves(fpr, tpr, model_config=None, thresholds=None, choosen_thresholds=None, outpath=None,
                    labels: Sequence[str] = ("GCN", "baseline")):
    """ROC curves with AUC in the legend; the chosen threshold is marked by
    interpolating (fpr, tpr) at it along the threshold axis."""
    if outpath is None:
        outpath = os.path.join(_outdir(model_config), "ROC_curve.png")
    os.makedirs(os.path.dirname(outpath) or ".", exist_ok=True)
    fig, ax = plt.subplots(figsize=(6, 5))
    for i in range(len(fpr)):
        f, t = np.asarray(fpr[i]), np.asarray(tpr[i])
        ax.plot(f, t, color=COLOR_TAB[i % len(COLOR_TAB)],
                label="ROC curve (area = {:.3f}) {:s}".format(_auc(f, t), labels[i] if i < len(labels) else str(i)))
        if thresholds is not None and choosen_thresholds is not None:
            th = np.asarray(thresholds[i], np.float64)
            order = np.argsort(th)
            th_s = th[order]
            fin = np.isfinite(th_s)
            x = float(choosen_thresholds[i])
            ft = np.interp(x, th_s[fin], f[order][fin])
            tt = np.interp(x, th_s[fin], t[order][fin])
            ax.plot(ft, tt, "o", color=COLOR_TAB[i % len(COLOR_TAB)])
    ax.plot([0, 1], [0, 1], "k--")
    ax.set_xlim([0.0, 1.0])
    ax.set_ylim([0.0, 1.05])
    ax.set_xlabel("False Positive Rate")
    ax.set_ylabel("True Positive Rate")
    ax.set_title("Receiver Operating Characteristic")
    ax.legend(loc="lower right")
    ax.margins(x=0.001)
    fig.savefig(outpath, bbox_inches="tight")
    plt.close(fig)
    return outpath


def extract_target_info(windows, window_ids, timeseries_out: bool = False, store=None):
    """(sensor_ids, anomaly_dates, flags_true[, series, dates]) of the given windows.

    CML: one entry per window (flagged sensor). SoilNet: one entry per valid node of
    each window (the reference repeats per node, ``:62-71``)."""
    window_ids = np.asarray(window_ids, np.int64)
    g_of, l_of = windows.flat()
    T = windows.seq_len
    tb = int(round(windows.timestep_before / windows.freq))
    sensor_ids, dates, flags, series, sdates = [], [], [], [], []
    for w in window_ids:
        gi, li = int(g_of[w]), int(l_of[w])
        g, ix = windows.groups[gi], windows.indices[gi]
        c = int(ix.center[li])
        t = g.time[c - tb:c - tb + T]
        if windows.ds_type == "cml":
            sensor_ids.append(str(g.group_id))
            dates.append(g.time[c])
            flags.append(int(ix.labels[li]))
            if timeseries_out:
                series.append(g.features[g.anomalous_pos][:, c - tb:c - tb + T].T)
                sdates.append(t)
        else:
            nodes = np.nonzero(ix.node_valid[li])[0]
            for n in nodes:
                sensor_ids.append(g.sensor_ids[n])
                dates.append(g.time[c])
                flags.append(int(ix.labels[li][n]))
                if timeseries_out:
                    series.append(g.features[n][:, c - tb:c - tb + T].T)
                    sdates.append(t)
    out = (np.asarray(sensor_ids), np.asarray(dates, dtype="datetime64[m]"), np.asarray(flags))
    if timeseries_out:
        return out + (np.asarray(series), np.asarray(sdates))
    return out


def timeseries_figure(predicted, true, sensor_timeseries, sensor_id, dates, outdir, anomaly_time_ind,
                      model_config=None, ds_type="cml", alpha: Optional[float] = None):
    """One window: the flagged sensor's channels, the centre step shaded by outcome."""
    alpha = alpha if alpha is not None else float(((model_config or {}).get("plotting") or {}).get("alpha", 0.2))
    os.makedirs(outdir, exist_ok=True)
    dates = np.asarray(dates).astype("datetime64[m]").astype(object)
    sensor_timeseries = np.asarray(sensor_timeseries, np.float64)
    fig, ax = plt.subplots(1, 1, figsize=(18, 3))
    ymin = np.floor(np.nanmin(sensor_timeseries))
    ymax = np.ceil(np.nanmax(sensor_timeseries))
    if ymin == ymax:
        ymax = ymin + 1
    ax.set_ylim([ymin, ymax])
    color = OUTCOME_COLORS[(int(predicted), int(true))]
    ax.fill_between(dates[anomaly_time_ind - 1:anomaly_time_ind + 1], ymin, ymax, alpha=alpha, color=color)
    legend = [mpatches.Patch(color=c, label=l, alpha=alpha) for c, l in
              (("green", "True Positive"), ("blue", "True Negative"), ("orange", "False Positive"),
               ("red", "False Negative"))]
    ax.plot(dates, sensor_timeseries[:, 0], color=LINE_COLORS[0])
    if ds_type == "cml":
        ax.plot(dates, sensor_timeseries[:, 1], color=LINE_COLORS[1])
        ax.xaxis.set_major_formatter(mdates.DateFormatter("%H:%M"))
        ax.set_ylabel("TL [dB]", fontsize=14)
    else:
        ax2 = ax.twinx()
        ax2.plot(dates, sensor_timeseries[:, -1], color=LINE_COLORS[1])
        ax2.set_ylabel("Battery voltage normalized", color=LINE_COLORS[1], fontsize=14)
        ax.xaxis.set_major_formatter(mdates.DateFormatter("%y-%m-%d %H:%M"))
        ax.set_ylabel("Soil moisture normalized", color=LINE_COLORS[0], fontsize=14)
    curr = dates[anomaly_time_ind]
    ax.set_title(f"{sensor_id} on {curr}", pad=12)
    ax.legend(handles=legend)
    outpath = os.path.join(outdir, f"{sensor_id}_{curr}_true_{int(true)}_pred_{int(predicted)}.png".replace(":", "-"))
    fig.savefig(outpath, bbox_inches="tight")
    plt.close(fig)
    return outpath


def plot_classified_samples(model, store, window_ids, model_config, preproc_config, threshold: float = 0.5,
                            baseline: bool = False, plot_example: bool = False, batch_size: int = 256):
    """Predict ``window_ids`` and write one :func:`timeseries_figure` per sample."""
    import torch
    out_dir = os.path.join(_outdir(model_config), "classified_validation_samples" + ("_baseline" if baseline else ""))
    ids = np.asarray(window_ids, np.int64)
    if plot_example:
        ids = ids[:3]
    preds = []
    model.eval()
    with torch.no_grad():
        for s in range(0, len(ids), batch_size):
            b = store.gather(torch.as_tensor(ids[s:s + batch_size], device=store.device))
            preds.append(model(b.model_inputs(store.ds_type, baseline)).reshape(b.y.shape).float().cpu().numpy())
    pred = np.concatenate(preds)
    sids, _, flags, series, sdates = extract_target_info(store.windows, ids, timeseries_out=True)
    if store.ds_type != "cml":
        pred = np.concatenate([p[m > 0] for p, m in zip(pred, store.win_valid[torch.as_tensor(ids)].cpu().numpy())])
    cls = (pred.reshape(-1) > threshold).astype(int)
    tb = int(round(store.windows.timestep_before / store.windows.freq))
    paths = []
    for i in range(len(cls)):
        paths.append(timeseries_figure(cls[i], flags[i], series[i], sids[i], sdates[i], out_dir, tb, model_config,
                                       store.ds_type))
    return paths


def _strip(ax, dates, pred, true, lo, hi, alpha, tn_color="white", empty="grey", label=True):
    for (p, t), col, name in (((1, 1), "green", "True Positive"), ((0, 0), tn_color, "True Negative"),
                              ((0, 1), "red", "False Negative"), ((1, 0), "orange", "False Positive")):
        ax.fill_between(dates, lo, hi, where=(pred == p) & (true == t), alpha=alpha, color=col,
                        label=name if label else None, step="mid")
    ax.fill_between(dates, lo, hi, where=np.isnan(true), alpha=alpha, color=empty, label="No data" if label else None,
                    step="mid")


def plot_results(sensor_ids, anomaly_dates, anomaly_flags_pred, anomaly_flags_true, predictions, preproc_config,
                 model_config, windows=None, comparison: bool = False, sensor_ids_baseline=None,
                 anomaly_dates_baseline=None, anomaly_flags_pred_baseline=None, anomaly_flags_true_baseline=None,
                 predictions_baseline=None, labels=("GCN", "baseline"), interval: Optional[float] = None,
                 plot_example: bool = False, max_figures: int = 5) -> List[str]:
    """Per-sensor panels: flagged-sensor series on top, outcome strip(s) below, one
    figure per ``interval`` hours (``plotting.plot_time_range``)."""
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    alpha = float(pl.get("alpha", 0.2))
    interval = float(interval if interval is not None else pl.get("plot_time_range", 144))
    out_dir = os.path.join(_outdir(model_config), "classified_timeseries" + ("_comparison" if comparison else ""))
    os.makedirs(out_dir, exist_ok=True)
    sensor_ids = np.asarray(sensor_ids)
    anomaly_dates = np.asarray(anomaly_dates).astype("datetime64[m]")
    groups = {str(g.group_id): g for g in windows.groups} if windows is not None else {}
    paths: List[str] = []
    for sid in np.unique(sensor_ids):
        sel = np.nonzero(sensor_ids == sid)[0]
        d = anomaly_dates[sel]
        start, end = d.min(), d.max()
        step = np.timedelta64(int(interval * 60), "m")
        t0 = start
        while t0 <= end and len(paths) < max_figures:
            t1 = t0 + step
            inwin = sel[(anomaly_dates[sel] >= t0) & (anomaly_dates[sel] < t1)]
            if len(inwin) == 0:
                t0 = t1
                continue
            order = inwin[np.argsort(anomaly_dates[inwin])]
            dts = anomaly_dates[order].astype(object)
            nrows = 2
            fig, ax = plt.subplots(nrows, 1, sharex="all", height_ratios=[2, 1], figsize=(18, 4.5))
            g = groups.get(str(sid))
            if g is not None:
                tt = g.time
                m = (tt >= t0) & (tt < t1)
                feats = g.features[g.anomalous_pos if g.anomalous_pos >= 0 else 0][:, m]
                for j in range(min(2, feats.shape[0])):
                    ax[0].plot(tt[m].astype(object), feats[j], linewidth=2, color=LINE_COLORS[j])
            else:
                ax[0].plot(dts, np.asarray(predictions)[order], color=LINE_COLORS[0])
            ax[0].set_ylabel("TL [dB]" if preproc_config.ds_type == "cml" else "Soil moisture", fontsize=14)
            base = 0.5 if comparison else 0.0
            _strip(ax[1], dts, np.asarray(anomaly_flags_pred)[order].astype(float),
                   np.asarray(anomaly_flags_true)[order].astype(float), base, 1, alpha)
            if comparison and sensor_ids_baseline is not None:
                sb = np.nonzero(np.asarray(sensor_ids_baseline) == sid)[0]
                db = np.asarray(anomaly_dates_baseline).astype("datetime64[m]")
                sb = sb[(db[sb] >= t0) & (db[sb] < t1)]
                sb = sb[np.argsort(db[sb])]
                _strip(ax[1], db[sb].astype(object), np.asarray(anomaly_flags_pred_baseline)[sb].astype(float),
                       np.asarray(anomaly_flags_true_baseline)[sb].astype(float), 0, 0.5, alpha, label=False)
                ax[1].axhline(0.5, color="black", alpha=alpha)
                ax[1].text(-0.05, 0.25, labels[1], transform=ax[1].transAxes, fontsize=12)
            ax[1].text(-0.05, 0.5 + base / 2, labels[0], transform=ax[1].transAxes, fontsize=12)
            ax[1].set_axis_off()
            ax[1].legend(loc=10, bbox_to_anchor=(0.5, -0.1), ncols=6)
            fig.suptitle(str(sid), y=0.99)
            p = os.path.join(out_dir, f"{sid}_{t0}_{t1}.png".replace(":", "-"))
            fig.savefig(p, bbox_inches="tight")
            plt.close(fig)
            paths.append(p)
            t0 = t1
            if plot_example:
                break
    return paths


__all__ = ["plot_roc_curves", "extract_target_info", "timeseries_figure", "plot_classified_samples", "plot_results"]
