"""Evaluation plots (reference ``libs/visualize.py``).

* :func:`plot_roc_curves` - several ROC curves + the chosen-threshold markers
  (``:17-47``);
* :func:`extract_target_info` - sensor ids, centre dates, true flags (and series) of
  a window-id list (``:50-92``) straight from the window index - no dataset replay;
* :func:`timeseries_figure` - one classified window (``:95-149``);
* :func:`plot_classified_samples` - predict + plot validation windows (``:152-177``);
* :func:`plot_results` - per-sensor strips of TP/TN/FP/FN along time, optional
  GCN-vs-baseline comparison (``:180-417``);
* :func:`classified_timeseries_figure` / :func:`plot_classified_timeseries` - a sensor's raw
  series over ``plot_time_range``-hour intervals, shaded by outcome at every classified step
  (``xai/libs/visualize.py:17-69, 72-133``);
* :func:`classified_timeseries_figure_with_neighbours` /
  :func:`plot_classified_timeseries_with_neighbours` - the flagged sensor and its neighbours
  stacked, each with the flagged sensor's outcome shading, neighbour distances in the titles
  (``xai/libs/visualize.py:243-312``).

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
        if windows.per_sensor:
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
    """One window: the flagged sensor's channels, the centre step shaded by outcome. ``outdir``
    with a file extension is the output path itself (``libs/visualize.py:201-206``)."""
    alpha = alpha if alpha is not None else float(((model_config or {}).get("plotting") or {}).get("alpha", 0.2))
    target = outdir if os.path.splitext(str(outdir))[1] else None
    outdir = (os.path.dirname(target) or ".") if target else outdir
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
    outpath = target or os.path.join(outdir,
                                     f"{sensor_id}_{curr}_true_{int(true)}_pred_{int(predicted)}.png".replace(":", "-"))
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
    if not store.per_sensor:
        pred = np.concatenate([p[m > 0] for p, m in zip(pred, store.win_valid[torch.as_tensor(ids)].cpu().numpy())])
    cls = (pred.reshape(-1) > threshold).astype(int)
    tb = int(round(store.windows.timestep_before / store.windows.freq))
    paths = []
    for i in range(len(cls)):
        paths.append(timeseries_figure(cls[i], flags[i], series[i], sids[i], sdates[i], out_dir, tb, model_config,
                                       store.ds_type))
    return paths


def _strip(ax, dates, pred, true, lo, hi, alpha, tn_color="white", empty="grey", label=True, no_data=True):
    for (p, t), col, name in (((1, 1), "green", "True Positive"), ((0, 0), tn_color, "True Negative"),
                              ((0, 1), "red", "False Negative"), ((1, 0), "orange", "False Positive")):
        ax.fill_between(dates, lo, hi, where=(pred == p) & (true == t), alpha=alpha, color=col,
                        label=name if label else None, step="mid")
    if no_data:
        ax.fill_between(dates, lo, hi, where=np.isnan(true), alpha=alpha, color=empty,
                        label="No data" if label else None, step="mid")


def soilnet_plot_series(raw, interpolation_max: str = "60min"):
    """What ``plot_results`` draws for SoilNet from the raw dataset (``libs/visualize.py:200-215``):
    gap-interpolated moisture and battery voltage [sensor, time] and the automatic-flag state:
    1 where ``moisture_flag_Auto:{BattV,Range,Spike}`` is set, NaN where the step is unlabelled
    (``moisture_flag_no_label``) and no automatic flag is set, 0 otherwise."""
    from ..data.interp import interpolate_gaps
    t = np.asarray(raw.time)
    moist = interpolate_gaps(np.asarray(raw["moisture"].values, np.float64), t, interpolation_max)
    battv = interpolate_gaps(np.asarray(raw["battv"].values, np.float64), t, interpolation_max)
    auto = np.where(np.asarray(raw["moisture_flag_no_label"].values, bool), np.nan, 0.0)
    hit = np.zeros(auto.shape, bool)
    for k in ("moisture_flag_Auto:BattV", "moisture_flag_Auto:Range", "moisture_flag_Auto:Spike"):
        if k in raw:
            hit |= np.asarray(raw[k].values, bool)
    auto[hit] = 1.0
    return {"sensor_ids": np.asarray(raw.sensor_ids).astype(str), "time": t.astype("datetime64[m]"),
            "moisture": moist, "battv": battv, "automatic_flags": auto}


def _soil_strip(ax, dates, pred, true, auto, lo, hi, alpha, label=True):
    """Outcome bands plus the reference's two SoilNet bands (``libs/visualize.py:351-359``):
    'Automatic flag' where the automatic-flag state is not 0 - which, as in the reference (its
    ``where=`` casts the NaN of unlabelled steps to True), includes unlabelled steps - and
    'No data' where a labelled step has no prediction."""
    _strip(ax, dates, pred, true, lo, hi, alpha, label=label, no_data=False)
    ax.fill_between(dates, lo, hi, where=(auto != 0), alpha=alpha, color="blue",
                    label="Automatic flag" if label else None, step="mid")
    ax.fill_between(dates, lo, hi, where=np.isnan(true) & (auto == 0), alpha=alpha, color="grey",
                    label="No data" if label else None, step="mid")


def plot_results(sensor_ids, anomaly_dates, anomaly_flags_pred, anomaly_flags_true, predictions, preproc_config,
                 model_config, windows=None, comparison: bool = False, sensor_ids_baseline=None,
                 anomaly_dates_baseline=None, anomaly_flags_pred_baseline=None, anomaly_flags_true_baseline=None,
                 predictions_baseline=None, labels=("GCN", "baseline"), interval: Optional[float] = None,
                 plot_example: bool = False, max_figures: int = 5, raw=None) -> List[str]:
    """Per-sensor panels: flagged-sensor series on top, outcome strip(s) below, one
    figure per ``interval`` hours (``plotting.plot_time_range``; at most ``max_figures``,
    the reference stops after 5, ``libs/visualize.py:219,235``).

    SoilNet with the ``raw`` dataset (``libs/visualize.py:200-215,285-291,316-322,351-389``):
    the raw time axis of the range, moisture on the left axis (limits floor(min) .. ceil(min(60,
    max))), battery voltage [V] on a twin axis, the outcomes placed at their window centres, and
    the 'Automatic flag' / 'No data' bands of :func:`_soil_strip`."""
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    alpha = float(pl.get("alpha", 0.2))
    interval = float(interval if interval is not None else pl.get("plot_time_range", 144))
    out_dir = os.path.join(_outdir(model_config), "classified_timeseries" + ("_comparison" if comparison else ""))
    os.makedirs(out_dir, exist_ok=True)
    sensor_ids = np.asarray(sensor_ids)
    anomaly_dates = np.asarray(anomaly_dates).astype("datetime64[m]")
    groups = {str(g.group_id): g for g in windows.groups} if windows is not None else {}
    soil = soilnet_plot_series(raw) if (raw is not None and preproc_config.ds_type == "soilnet") else None
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
            if soil is not None and str(sid) in set(soil["sensor_ids"]):
                paths.append(_plot_soil_range(soil, str(sid), t0, t1, order, anomaly_dates, anomaly_flags_pred,
                                              anomaly_flags_true, alpha, out_dir, labels, comparison,
                                              sensor_ids_baseline, anomaly_dates_baseline,
                                              anomaly_flags_pred_baseline, anomaly_flags_true_baseline))
                t0 = t1
                if plot_example:
                    break
                continue
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


def _place(plot_dates, dates, values):
    """values at ``dates`` spread onto ``plot_dates`` (NaN elsewhere), as the reference's intersect1d."""
    out = np.full(len(plot_dates), np.nan)
    _, pi, ai = np.intersect1d(plot_dates, dates, return_indices=True)
    out[pi] = np.asarray(values, np.float64)[ai]
    return out


def _plot_soil_range(soil, sid, t0, t1, order, anomaly_dates, pred, true, alpha, out_dir, labels, comparison,
                     sids_b, dates_b, pred_b, true_b):
    k = int(np.nonzero(soil["sensor_ids"] == sid)[0][0])
    tt = soil["time"]
    m = (tt >= t0) & (tt <= t1)
    plot_dates = tt[m]
    moist, batt, auto = soil["moisture"][k, m], soil["battv"][k, m] / 1000.0, soil["automatic_flags"][k, m]
    p_ts = _place(plot_dates, anomaly_dates[order], np.asarray(pred)[order])
    t_ts = _place(plot_dates, anomaly_dates[order], np.asarray(true)[order])
    fig, ax = plt.subplots(2, 1, sharex="all", height_ratios=[1.2, 1] if comparison else [2, 1],
                           figsize=(18, 6 if comparison else 4.5))
    pd_obj = plot_dates.astype(object)
    ax[0].plot(pd_obj, moist, linewidth=2, color=LINE_COLORS[0])
    fin = moist[np.isfinite(moist)]
    if fin.size:
        ax[0].set_ylim([int(np.floor(fin.min())), int(np.ceil(min(60.0, fin.max())))])
    ax[0].set_ylabel("Soil moisture [%]", color=LINE_COLORS[0], fontsize=14)
    ax2 = ax[0].twinx()
    ax2.plot(pd_obj, batt, linewidth=2, color=LINE_COLORS[1], zorder=1)
    ax2.set_ylabel("Battery voltage [V]", color=LINE_COLORS[1], fontsize=14)
    ax2.locator_params(axis="y", nbins=4)
    ax[0].xaxis.set_major_formatter(mdates.DateFormatter("%Y-%m-%d %H:%M"))
    base = 0.5 if comparison else 0.0
    _soil_strip(ax[1], pd_obj, p_ts, t_ts, auto, base, 1, alpha)
    if comparison and sids_b is not None:
        sb = np.nonzero(np.asarray(sids_b) == sid)[0]
        db = np.asarray(dates_b).astype("datetime64[m]")
        sb = sb[(db[sb] >= t0) & (db[sb] <= t1)]
        _soil_strip(ax[1], pd_obj, _place(plot_dates, db[sb], np.asarray(pred_b)[sb]),
                    _place(plot_dates, db[sb], np.asarray(true_b)[sb]), auto, 0, 0.5, alpha, label=False)
        ax[1].axhline(0.5, color="black", alpha=alpha)
        ax[1].text(-0.05, 0.25, labels[1], transform=ax[1].transAxes, fontsize=12)
    ax[1].text(-0.05, 0.5 + base / 2, labels[0], transform=ax[1].transAxes, fontsize=12)
    ax[1].set_axis_off()
    ax[1].legend(loc=10, bbox_to_anchor=(0.5, -0.1), ncols=6)
    fig.suptitle(sid, y=0.99)
    p = os.path.join(out_dir, f"{sid}_{t0}_{t1}.png".replace(":", "-"))
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    return p


_OUTCOMES = (((1, 1), "green", "True Positive"), ((0, 0), "blue", "True Negative"),
             ((0, 1), "red", "False Negative"), ((1, 0), "orange", "False Positive"))


def _shade(ax, dates, pred, true, lo, hi, alpha, label=True):
    """Outcome shading at the steps where both flags are defined (NaN elsewhere)."""
    pred = np.asarray(pred, np.float64)
    true = np.asarray(true, np.float64)
    for (p, t), col, name in _OUTCOMES:
        ax.fill_between(dates, lo, hi, where=(pred == p) & (true == t), alpha=alpha, color=col,
                        label=name if label else None)


def _stamp(d) -> str:
    return str(np.datetime64(d, "m")).replace(":", "-")


def classified_timeseries_figure(sensor_id, features, dates, anomaly_flags_true, anomaly_flags_pred, model_config,
                                 probabilities=None, outdir=None):
    """One sensor over one time range: its raw channels (``features``: list of [T] arrays), shaded
    TP / TN / FN / FP where a window centred on that step was classified (flags NaN elsewhere),
    optional probability trace on a twin axis. Returns the PNG path."""
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    alpha = float(pl.get("alpha", 0.2))
    outdir = outdir or os.path.join(_outdir(model_config), "classified_timeseries_raw")
    os.makedirs(outdir, exist_ok=True)
    d = np.asarray(dates).astype("datetime64[m]")
    dd = d.astype(object)
    feats = [np.asarray(f, np.float64) for f in features]
    allv = np.concatenate([f[np.isfinite(f)] for f in feats]) if feats else np.zeros(1)
    ymin = float(np.floor(allv.min())) if allv.size else 0.0
    ymax = float(np.ceil(allv.max())) if allv.size else 1.0
    if ymax <= ymin:
        ymax = ymin + 1.0
    fig, ax = plt.subplots(1, 1, figsize=(20, 4))
    ax.set_ylim([ymin, ymax])
    _shade(ax, dd, anomaly_flags_pred, anomaly_flags_true, ymin, ymax, alpha)
    for j, f in enumerate(feats):
        ax.plot(dd, f, color=LINE_COLORS[j % len(LINE_COLORS)], linewidth=1.5)
    if probabilities is not None:
        ax2 = ax.twinx()
        ax2.set_ylim([0, 1])
        ax2.plot(dd, np.asarray(probabilities, np.float64), "k", linewidth=0.5, label="probability")
    ax.set_title(str(sensor_id), pad=10)
    ax.legend(loc="upper right")
    ax.margins(x=0.001)
    outpath = os.path.join(outdir, f"{sensor_id}_start_{_stamp(d[0])}_end_{_stamp(d[-1])}.png")
    fig.savefig(outpath, bbox_inches="tight")
    plt.close(fig)
    return outpath


def _predict_windows(model, store, ids, baseline, batch_size=256):
    import torch
    preds = []
    was = model.training
    model.eval()
    with torch.no_grad():
        for s in range(0, len(ids), batch_size):
            b = store.gather(torch.as_tensor(ids[s:s + batch_size], device=store.device))
            preds.append(model(b.model_inputs(store.ds_type, baseline)).reshape(b.y.shape).float().cpu().numpy())
    if was:
        model.train()
    pred = np.concatenate(preds)
    if not store.per_sensor:
        valid = store.win_valid[torch.as_tensor(ids)].cpu().numpy()
        pred = np.concatenate([p[m > 0] for p, m in zip(pred, valid)])
    return pred.reshape(-1)


def _node_series(windows, sensor_id):
    """(group, node position) holding ``sensor_id``'s raw series (CML: the group it is flagged in)."""
    for g in windows.groups:
        if windows.per_sensor:
            if str(g.group_id) == str(sensor_id):
                return g, max(g.anomalous_pos, 0)
        else:
            hit = np.nonzero(np.asarray(g.sensor_ids).astype(str) == str(sensor_id))[0]
            if len(hit):
                return g, int(hit[0])
    return None, -1


def plot_classified_timeseries(model, store, window_ids, model_config, predictions=None, start_date=None,
                               end_date=None, baseline: bool = False, threshold: float = 0.5,
                               interval: Optional[float] = None, max_figures: Optional[int] = None) -> List[str]:
    """Classify ``window_ids`` (or use ``predictions``, one per :func:`extract_target_info` row) and
    write, per sensor and ``plotting.plot_time_range``-hour interval, its raw series with the outcome
    of every window centred in it (``xai/libs/visualize.py:72-133``)."""
    ids = np.asarray(window_ids, np.int64)
    pred = np.asarray(predictions, np.float64).reshape(-1) if predictions is not None else \
        _predict_windows(model, store, ids, baseline)
    cls = (pred > threshold).astype(np.float64)
    sids, adates, flags = extract_target_info(store.windows, ids)
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    interval = float(interval if interval is not None else pl.get("plot_time_range", 144))
    step = np.timedelta64(int(interval * 60), "m")
    out_dir = os.path.join(_outdir(model_config), "classified_timeseries_raw" + ("_baseline" if baseline else ""))
    paths: List[str] = []
    for sid in np.unique(sids):
        g, pos = _node_series(store.windows, sid)
        if g is None:
            continue
        sel = np.nonzero(sids == sid)[0]
        t_lo = np.datetime64(start_date, "m") if start_date is not None else g.time.min()
        t_hi = np.datetime64(end_date, "m") if end_date is not None else g.time.max()
        t0 = t_lo
        while t0 <= t_hi:
            t1 = t0 + step
            m = (g.time >= t0) & (g.time <= t1)
            cur = sel[(adates[sel] >= t0) & (adates[sel] <= t1)]
            if len(cur) and m.any():
                plot_dates = g.time[m]
                pser = np.full(plot_dates.shape[0], np.nan)
                tser = pser.copy()
                _, pi, ai = np.intersect1d(plot_dates, adates[cur], return_indices=True)
                pser[pi] = cls[cur][ai]
                tser[pi] = flags[cur][ai]
                feats = [g.features[pos][c][m] for c in range(g.features.shape[1])]
                if store.ds_type != "cml":
                    feats = feats[:1]          # soil moisture (the reference plots moisture only)
                paths.append(classified_timeseries_figure(sid, feats, plot_dates, tser, pser, model_config,
                                                          outdir=out_dir))
                if max_figures is not None and len(paths) >= max_figures:
                    return paths
            t0 = t1
    return paths


def classified_timeseries_figure_with_neighbours(sensor_ids, all_features_timeseries, feature_timeseries_dates,
                                                 anomaly_flags_true, anomaly_flags_pred, model_config, flags,
                                                 probabilities=None, distances=None, ymin=None, ymax=None,
                                                 outdir=None):
    """Stacked panels, one per sensor (``all_features_timeseries`` [S, T, C]): each shaded with the
    flagged sensor's outcomes, the flagged one titled 'Anomalous sensor', the others 'Neighbouring
    sensor' with their distance. Per-panel y range min - 1 .. min + 24 unless given
    (``xai/libs/visualize.py:243-312``). Returns the PNG path."""
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    alpha = float(pl.get("alpha", 0.2))
    feats = np.asarray(all_features_timeseries, np.float64)
    S = feats.shape[0]
    d = np.asarray(feature_timeseries_dates).astype("datetime64[m]")
    dd = d.astype(object)
    fig, axes = plt.subplots(S, 1, figsize=(20, S * 3.5), sharex="all", squeeze=False)
    axes = axes[:, 0]
    flagged = str(sensor_ids[int(np.argmax(np.asarray(flags)))]) if np.any(flags) else str(sensor_ids[0])
    fixed = ymin is not None
    for i in range(S):
        f = feats[i]
        lo, hi = (ymin, ymax) if fixed else (float(np.nanmin(f)) - 1.0, float(np.nanmin(f)) + 24.0)
        if not np.isfinite(lo):
            lo, hi = 0.0, 25.0
        ax = axes[i]
        ax.set_ylim([lo, hi])
        _shade(ax, dd, anomaly_flags_pred, anomaly_flags_true, lo, hi, alpha, label=i == S - 1)
        if flags[i]:
            ax.set_title(f"Anomalous sensor: {sensor_ids[i]}", pad=10, fontweight="bold")
        elif distances is not None:
            ax.set_title(f"Neighbouring sensor: {sensor_ids[i]} distance: {float(distances[i]):.1f}", pad=10)
        else:
            ax.set_title(f"Neighbouring sensor: {sensor_ids[i]}", pad=10)
        if probabilities is not None:
            ax2 = ax.twinx()
            ax2.set_ylim([0, 1])
            ax2.plot(dd, np.asarray(probabilities, np.float64), "k", linewidth=0.5, label="probability")
        for c in range(f.shape[-1]):
            ax.plot(dd, f[:, c])
        ax.xaxis.set_major_formatter(mdates.DateFormatter("%Y-%m-%d %H:%M"))
        if i == S - 1:
            ax.legend()
    outdir = outdir or os.path.join(_outdir(model_config), "classification_with_neighbors")
    os.makedirs(outdir, exist_ok=True)
    outpath = os.path.join(outdir, f"{flagged}_start_{_stamp(d[0])}_end_{_stamp(d[-1])}_neighbours.png")
    fig.savefig(outpath, bbox_inches="tight")
    plt.close(fig)
    return outpath


def plot_classified_timeseries_with_neighbours(model, store, window_ids, model_config, predictions=None,
                                               baseline: bool = False, threshold: float = 0.5,
                                               interval: Optional[float] = None,
                                               max_figures: Optional[int] = 5) -> List[str]:
    """CML: per flagged sensor and interval, the flagged link and every neighbour of its graph
    (channels of the raw series), shaded by the flagged link's outcomes, with the classifier's
    probability trace and the neighbours' distances to the flagged link."""
    if not store.per_sensor:
        raise ValueError("neighbour figures need flagged-sensor neighbourhoods (CML, XAI SoilNet)")
    ids = np.asarray(window_ids, np.int64)
    pred = np.asarray(predictions, np.float64).reshape(-1) if predictions is not None else \
        _predict_windows(model, store, ids, baseline)
    cls = (pred > threshold).astype(np.float64)
    sids, adates, flags_true = extract_target_info(store.windows, ids)
    pl = (model_config.get("plotting") or {}) if model_config is not None else {}
    interval = float(interval if interval is not None else pl.get("plot_time_range", 144))
    step = np.timedelta64(int(interval * 60), "m")
    paths: List[str] = []
    for sid in np.unique(sids):
        g, pos = _node_series(store.windows, sid)
        if g is None:
            continue
        sel = np.nonzero(sids == sid)[0]
        t0 = adates[sel].min()
        while t0 <= adates[sel].max():
            t1 = t0 + step
            m = (g.time >= t0) & (g.time <= t1)
            cur = sel[(adates[sel] >= t0) & (adates[sel] <= t1)]
            if len(cur) and m.any():
                plot_dates = g.time[m]
                pser = np.full(plot_dates.shape[0], np.nan)
                tser = pser.copy()
                prob = pser.copy()
                _, pi, ai = np.intersect1d(plot_dates, adates[cur], return_indices=True)
                pser[pi] = cls[cur][ai]
                tser[pi] = flags_true[cur][ai]
                prob[pi] = pred[cur][ai]
                feats = np.transpose(g.features[:, :, m], (0, 2, 1))          # [S, T, C]
                fl = np.zeros(g.n_nodes, dtype=bool)
                fl[pos] = True
                paths.append(classified_timeseries_figure_with_neighbours(
                    [str(s) for s in g.sensor_ids], feats, plot_dates, tser, pser, model_config, fl,
                    probabilities=prob, distances=np.asarray(g.distances)[pos]))
                if max_figures is not None and len(paths) >= max_figures:
                    return paths
            t0 = t1
    return paths


__all__ = ["plot_roc_curves", "extract_target_info", "timeseries_figure", "plot_classified_samples", "plot_results",
           "classified_timeseries_figure", "plot_classified_timeseries",
           "classified_timeseries_figure_with_neighbours", "plot_classified_timeseries_with_neighbours"]
