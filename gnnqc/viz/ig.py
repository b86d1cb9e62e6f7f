"""Integrated-gradients figures (reference ``xai/libs/integrated_gradients.py:1415-2044``
and ``xai/libs/visualize.py``).

* :func:`plot_ig_heatmap` - flagged-sensor channels with their attribution painted as
  a time heatmap underneath, then one row per neighbour node (attributions scaled by
  ``plot.heatmap.scale_feature_gradients``), diverging colormap with the configured
  limits (``_plot_ig_heatmap``, ``:1612-1891``);
* :func:`plot_ig_heatmap_from_directory` - heatmaps of the sample directories written by the
  explainer, filtered by sensor / centre-time range and split over workers (``:1893-2044``);
* :func:`plot_gradient_saturation` - model output along the alpha path (``:1516-1610``);
* :func:`plot_interpolated_series` - every 10th interpolated input along the path (``:1415-1466``).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Optional

import numpy as np

import matplotlib

matplotlib.use("Agg")
import matplotlib.colors as mcolors  # noqa: E402
import matplotlib.pyplot as plt  # noqa: E402

CMAP = "RdBu_r"
CHANNEL_COLORS = [(1 / 255, 183 / 255, 1.0), (0.0, 117 / 255, 177 / 255), (0.2, 0.6, 0.2)]
STEMS = ("features_unwrapped", "anom_ts_unwrapped", "gradients_features_unwrapped", "gradients_anom_ts_unwrapped",
         "predictions_unwrapped", "anomaly_flag_true_unwrapped", "path_predictions_unwrapped")


def _cfg_get(cfg, path, default=None):
    cur = cfg
    for k in path.split("."):
        if cur is None or not hasattr(cur, "get"):
            return default
        cur = cur.get(k)
    return default if cur is None else cur


def _norm(limits, data):
    if isinstance(limits, (list, tuple)) and len(limits) == 2:
        return mcolors.Normalize(vmin=float(limits[0]), vmax=float(limits[1]))
    m = float(np.nanmax(np.abs(data))) if np.size(data) else 1.0
    m = m if m > 0 else 1.0
    return mcolors.Normalize(vmin=-m, vmax=m)


def plot_ig_heatmap(files: Dict[str, np.ndarray], rec: dict, xai_config=None, out_path: Optional[str] = None,
                    batch_id: Optional[int] = None, dpi: Optional[int] = None):
    hcfg = "integrated_gradients.plot.heatmap"
    scale_nb = float(_cfg_get(xai_config, hcfg + ".scale_feature_gradients", 25))
    limits = _cfg_get(xai_config, hcfg + ".cbar_limits", "auto")
    dpi = dpi or int(_cfg_get(xai_config, hcfg + ".dpi", 100))
    log_norm = _cfg_get(xai_config, hcfg + ".cbar_norm", "linear") == "log"
    anom = files.get("anom_ts_unwrapped")
    ganom = files.get("gradients_anom_ts_unwrapped")
    feats = files.get("features_unwrapped")
    gfeat = files.get("gradients_features_unwrapped")
    n_nb = 0 if gfeat is None else gfeat.shape[0]
    rows = (1 if anom is not None else 0) + n_nb
    rows = max(rows, 1)
    T = (anom if anom is not None else feats[0]).shape[0]
    x = np.arange(T)
    edges = np.linspace(-0.5, T - 0.5, T + 1)
    fig, axes = plt.subplots(rows, 1, figsize=(14, 1.2 + 1.1 * rows), sharex=True, squeeze=False)
    axes = axes[:, 0]
    all_g = [g for g in (ganom, None if gfeat is None else gfeat * scale_nb) if g is not None]
    norm = _norm(limits, np.concatenate([g.reshape(-1) for g in all_g])) if all_g else None
    if log_norm and norm is not None:
        norm = mcolors.SymLogNorm(linthresh=max(1e-6, abs(norm.vmax) * 1e-3), vmin=norm.vmin, vmax=norm.vmax)
    mesh = None
    r = 0

    def panel(ax, series, grads, label):
        nonlocal mesh
        C = series.shape[-1]
        lo, hi = np.nanmin(series), np.nanmax(series)
        pad = 0.1 * (hi - lo + 1e-6)
        lo, hi = lo - pad, hi + pad
        if grads is not None:
            yed = np.linspace(lo, hi, C + 1)
            mesh = ax.pcolormesh(edges, yed, grads.T, cmap=CMAP, norm=norm, shading="flat", alpha=0.85)
        for c in range(C):
            ax.plot(x, series[:, c], color=CHANNEL_COLORS[c % len(CHANNEL_COLORS)], linewidth=1.2)
        ax.set_ylim(lo, hi)
        ax.set_ylabel(label, rotation=0, ha="right", fontsize=8)

    if anom is not None:
        panel(axes[r], anom, ganom, "flagged")
        r += 1
    for j in range(n_nb):
        panel(axes[r], feats[j], gfeat[j] * scale_nb, f"node {j}")
        r += 1
    for ax in axes:
        ax.axvline((T - 1) * 2 / 3 if anom is None else _centre(T, rec), color="k", linewidth=0.6, alpha=0.6)
    title = f"{rec.get('sensor', '')} {rec.get('date', '')}  true={rec.get('true')} pred={rec.get('pred')} " \
            f"p={rec.get('score', float('nan')):.3f}"
    if batch_id is not None and _cfg_get(xai_config, hcfg + ".annotate_batch_id", True):
        title += f"  batch {batch_id}"
    axes[0].set_title(title, fontsize=10)
    if mesh is not None:
        fig.colorbar(mesh, ax=list(axes), shrink=0.8, label="integrated gradients")
    if out_path:
        os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
        fig.savefig(out_path, dpi=dpi, bbox_inches="tight")
    plt.close(fig)
    return out_path


def _centre(T: int, rec: dict) -> float:
    tb = rec.get("timestep_before_steps")
    return float(tb) if tb is not None else (T - 1) * 2 / 3


def _load_sample_dir(d: str) -> Dict[str, np.ndarray]:
    files = {}
    for stem in STEMS:
        hits = glob.glob(os.path.join(d, f"{stem}_*.npy"))
        # "features_unwrapped" is a suffix of "gradients_features_unwrapped": match the exact stem
        hits = [h for h in hits if os.path.basename(h).startswith(stem + "_")]
        if hits:
            files[stem] = np.load(hits[0])
    return files


def parse_sample_dir(name: str) -> dict:
    """``<sensor>_<YYYYmmdd>_<HHMMSS>_<true>_<pred>`` (sensor ids may contain ``_``)."""
    parts = name.rsplit("_", 4)
    if len(parts) != 5:
        raise ValueError(f"not a sample directory name: {name}")
    sensor, day, tod, true, pred = parts
    return {"sensor": sensor, "date": f"{day}_{tod}", "true": int(true), "pred": int(pred)}


def list_sample_dirs(directory: str, sensors=None, time_from=None, time_to=None) -> list:
    """Sample directories ``<directory>/<sensor>/<sample>`` of an explainer run, as
    ``(sensor, sample)`` pairs sorted by sample name (``integrated_gradients.py:1903-1936``): the
    sensor directories (all but ``log`` and dot files, or the given ``sensors``), then, with both
    ``time_from`` and ``time_to``, only samples whose centre time (parsed from the name) lies in
    [time_from, time_to]."""
    import pandas as pd
    if sensors is None:
        sensors = sorted(os.listdir(directory)) if os.path.isdir(directory) else []
    sensors = [str(s) for s in sensors if s != "log" and not str(s).startswith(".")]
    pairs = []
    for sensor in sensors:
        d = os.path.join(directory, sensor)
        if not os.path.isdir(d):
            continue
        for dn in os.listdir(d):
            if os.path.isdir(os.path.join(d, dn)):
                pairs.append((sensor, dn))
    pairs.sort(key=lambda p: p[1])
    if time_from is not None and time_to is not None:
        lo, hi = pd.to_datetime(time_from), pd.to_datetime(time_to)
        keep = []
        for sensor, dn in pairs:
            try:
                t = pd.to_datetime(parse_sample_dir(dn)["date"], format="%Y%m%d_%H%M%S")
            except ValueError:
                continue
            if lo <= t <= hi:
                keep.append((sensor, dn))
        pairs = keep
    return pairs


def plot_ig_heatmap_from_directory(directory: str, xai_config=None, overwrite: bool = False, sensors=None,
                                   time_from=None, time_to=None, workerid: Optional[int] = None,
                                   n_worker: Optional[int] = None, stem: Optional[str] = None):
    """Heatmaps of every saved sample (``integrated_gradients.py:1893-2044``): selected by sensor and
    centre-time range (:func:`list_sample_dirs`), split round-robin over ``n_worker`` workers
    (SLURM array / ``--shard``), written as ``ig_heatmap_<stem>_<sample>.png`` next to the sample's
    arrays (``stem`` = ``<project>_<ds_type>_<dataset>``; default: taken from the array names).
    Existing heatmaps are kept unless ``overwrite``. Returns the written paths."""
    samples = list_sample_dirs(directory, sensors, time_from, time_to)
    if workerid is not None and n_worker:
        samples = [s for i, s in enumerate(samples) if i % n_worker == workerid]
    out = []
    for sensor, dn in samples:
        d = os.path.join(directory, sensor, dn)
        try:
            rec = parse_sample_dir(dn)
        except ValueError:
            continue
        files = _load_sample_dir(d)
        if "features_unwrapped" not in files:      # (the reference skips samples without features)
            continue
        if "predictions_unwrapped" in files:
            rec["score"] = float(np.asarray(files["predictions_unwrapped"]).reshape(-1)[0])
        st = stem
        if st is None:
            hit = [f for f in os.listdir(d) if f.startswith("features_unwrapped_") and f.endswith(f"_{dn}.npy")]
            st = hit[0][len("features_unwrapped_"):-len(f"_{dn}.npy")] if hit else None
        name = f"ig_heatmap_{st}_{dn}.png" if st else f"ig_heatmap_{dn}.png"
        p = os.path.join(d, name)
        if os.path.exists(p) and not overwrite:
            continue
        out.append(plot_ig_heatmap(files, rec, xai_config, p))
    return out


def plot_gradient_saturation(path_pred: np.ndarray, out_path: str, normalize: bool = False):
    alphas = np.linspace(0, 1, len(path_pred))
    y = np.asarray(path_pred, np.float64)
    if normalize and np.ptp(y) > 0:
        y = (y - y.min()) / np.ptp(y)
    fig, ax = plt.subplots(1, 2, figsize=(10, 3.5))
    ax[0].plot(alphas, y)
    ax[0].set_xlabel("alpha")
    ax[0].set_title("Target class predicted \n probability over alpha")
    ax[1].plot(alphas[1:], np.diff(y) * (len(y) - 1))
    ax[1].set_xlabel("alpha")
    ax[1].set_title("d prediction / d alpha")
    fig.tight_layout()
    fig.savefig(out_path, bbox_inches="tight")
    plt.close(fig)
    return out_path


def plot_interpolated_series(series: np.ndarray, alphas: np.ndarray, out_path: str, every: int = 10,
                             max_steps: int = 500):
    """Every ``every``-th interpolated input of one sample along the alpha path, one row each
    (``_plot_interpolated_data_element_series``, ``integrated_gradients.py:1415-1466``):
    ``series`` [m+1, T, C] (flagged series) or [m+1, N, T, C] (node features: node 0 drawn)."""
    series = np.asarray(series)
    if series.ndim == 4:
        series = series[:, 0]
    sel = list(range(0, len(alphas), every))
    ymin, ymax = float(np.min(series)), float(np.max(series))
    fig = plt.figure(figsize=(20, 10))
    for k, i in enumerate(sel):
        ax = fig.add_subplot(len(sel), 1, k + 1)
        ax.set_title(f"alpha: {alphas[i]:.1f}")
        ax.plot(series[i][:max_steps])
        ax.set_ylim(ymin, ymax if ymax > ymin else ymin + 1)
    fig.tight_layout()
    fig.savefig(out_path, dpi=50)
    plt.close(fig)
    return out_path


__all__ = ["plot_ig_heatmap", "plot_ig_heatmap_from_directory", "plot_gradient_saturation",
           "plot_interpolated_series", "parse_sample_dir", "list_sample_dirs"]
