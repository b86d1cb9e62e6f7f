"""Analysis of saved integrated-gradients results (SURVEY L7;
reference ``xai/libs/integrated_gradients_analyser.py``, class ``IntegrateGradientsAnalyser``).

Works on the directory tree written by :class:`gnnqc.xai.ig.IntegratedGradientsExplainer`::

    <output_dir>/integrated_gradients/<project>/<ds>/<dataset>/<sensor>/<sensor>_<YYYYmmdd_HHMMSS>_<t>_<p>/
        gradients_features_unwrapped_<stem>.npy   [n_nodes, T, C]
        gradients_anom_ts_unwrapped_<stem>.npy    [T, C]
        features_unwrapped_<stem>.npy, anom_ts_unwrapped_<stem>.npy, predictions_unwrapped_<stem>.npy, ...

Methods mirror the reference: :meth:`get_overview` (``:343-529``: sample table, time-range
scatter and confusion bar plots, selection by confusion class with ``keep_surrounding``
context samples), :meth:`spatial_aggregate_gradients` (``:531-695``),
:meth:`plot_spatial_aggregated_gradients` (``:811-964``), :meth:`concatenate_images`
(``:697-731``), :meth:`create_videos` (GIF via PIL; ``:185-308,733-809``),
:meth:`plot_agg_samples_over_time` (``:1169-1710``), :meth:`scale_gradients_with_input`
(``:992-1074``), :meth:`rename_based_on_threshold` (``:1076-1120``). Work is split by
sensor over SLURM array tasks or ``torch.distributed`` ranks.

Differences on purpose: sample directory names are parsed from the right
(``rsplit``), so sensor ids need not have exactly four ``_``-separated parts
(``get_sensor_id``/``get_datetime``, ``:310-327``); the ``dont_scale.txt`` exclusion
list is optional.
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import pandas as pd

import matplotlib

matplotlib.use("Agg")
import matplotlib.colors as mcolors  # noqa: E402
import matplotlib.pyplot as plt  # noqa: E402

from .. import config as C  # noqa: E402
from ..viz.ig import parse_sample_dir  # noqa: E402
from .ig import CONFUSION  # noqa: E402

COLOR_MAP = {(0, 0): "white", (0, 1): "orange", (1, 0): "red", (1, 1): "green"}
TL_COLORS = [(1 / 255, 183 / 255, 1.0), (0.0, 117 / 255, 177 / 255), (0.2, 0.6, 0.2), (0.5, 0.5, 0.5)]
COLOR_NAMES = {(0, 0): "True Negative", (0, 1): "False Positive", (1, 0): "False Negative", (1, 1): "True Positive"}
STEM_GF, STEM_GA = "gradients_features_unwrapped", "gradients_anom_ts_unwrapped"
STEM_F, STEM_A = "features_unwrapped", "anom_ts_unwrapped"
STEM_P, STEM_Y = "predictions_unwrapped", "anomaly_flag_true_unwrapped"


class IntegrateGradientsAnalyser:
    def __init__(self, preproc_config, model_config=None, xai_config=None):
        load = lambda c: C.load(c) if isinstance(c, str) else c  # noqa: E731
        self.preproc_config = C.normalize_preproc(load(preproc_config))
        self.model_config = load(model_config) if model_config is not None else None
        self.xai_config = load(xai_config) if xai_config is not None else C.default("xai_ig")
        ig = self.xai_config.integrated_gradients
        self.ig = ig
        self.an = ig.analyser
        self.ds_type = self.preproc_config.ds_type
        self.dp_results_parent = os.path.join(self.xai_config.output_dir, "integrated_gradients",
                                              self.xai_config.project, self.ds_type, ig.dataset)
        self.stem = f"{self.xai_config.project}_{self.ds_type}_{ig.dataset}"
        self.conf_matrix_string = "_".join(sorted(str(x) for x in self.an.which_samples))
        from ..parallel import dist as D
        if "SLURM_ARRAY_TASK_ID" in os.environ:
            self.workerid = int(os.environ["SLURM_ARRAY_TASK_ID"])
            self.n_worker = int(os.environ["SLURM_ARRAY_TASK_COUNT"])
        elif D.world_size() > 1:
            self.workerid, self.n_worker = D.rank(), D.world_size()
        else:
            self.workerid = self.n_worker = None
        self.output_dir_analysis = os.path.join(
            os.path.dirname(self.dp_results_parent),
            f"{ig.dataset}_analysis_{self.an.concat_images_scale}_{self.an.video.video_fps}")
        self.df = self.df_unfiltered = None
        self.selected_sensors: List[str] = []

    # ----------------------------------------------------------------- helpers
    def get_filename(self, stem: str, dn_sample: str) -> str:
        return f"{stem}_{self.stem}_{dn_sample}"

    def _load(self, row, stem: str) -> Optional[np.ndarray]:
        p = os.path.join(row["path"], self.get_filename(stem, row["sample_name"]) + ".npy")
        return np.load(p) if os.path.exists(p) else None

    @staticmethod
    def _split_work(items, workerid, n_worker):
        return [it for i, it in enumerate(items) if i % n_worker == workerid]

    # ----------------------------------------------------------------- overview
    def get_overview(self, plots: bool = True) -> pd.DataFrame:
        os.makedirs(self.output_dir_analysis, exist_ok=True)
        rows = []
        if os.path.isdir(self.dp_results_parent):
            for sensor in sorted(os.listdir(self.dp_results_parent)):
                dsens = os.path.join(self.dp_results_parent, sensor)
                if sensor in ("log",) or sensor.startswith(".") or not os.path.isdir(dsens):
                    continue
                for dn in sorted(os.listdir(dsens)):
                    if not os.path.isdir(os.path.join(dsens, dn)):
                        continue
                    try:
                        info = parse_sample_dir(dn)
                    except ValueError:
                        continue
                    rows.append({"sensor_id": sensor, "sample_name": dn,
                                 "date_time": pd.to_datetime(info["date"], format="%Y%m%d_%H%M%S"),
                                 "true": info["true"], "pred": info["pred"], "path": os.path.join(dsens, dn)})
        df = pd.DataFrame(rows, columns=["sensor_id", "sample_name", "date_time", "true", "pred", "path"])
        self.df_unfiltered = df.copy()
        which_sensors = self.an.which_sensors
        self.selected_sensors = list(df["sensor_id"].unique()) if which_sensors in ("all", None) else \
            [str(s) for s in which_sensors]
        df = df[df["sensor_id"].isin(self.selected_sensors)]
        if self.workerid is not None:
            self.selected_sensors = self._split_work(self.selected_sensors, self.workerid, self.n_worker)
        df = df.sort_values("date_time").reset_index(drop=True)
        if len(df):
            df["color"] = [COLOR_MAP[(t, p)] for t, p in zip(df["true"], df["pred"])]
            df["confusion_matrix"] = [COLOR_NAMES[(t, p)] for t, p in zip(df["true"], df["pred"])]
            df["confusion_matrix_abbr"] = [CONFUSION[(t, p)] for t, p in zip(df["true"], df["pred"])]
            if plots:
                self._overview_plots(df)
            # selection + surrounding context samples
            sel = df["confusion_matrix_abbr"].isin(list(self.an.which_samples)).to_numpy()
            surr = int(self.an.get("keep_surrounding", 0) or 0)
            keep = sel.copy()
            for i in np.nonzero(sel)[0]:
                keep[max(0, i - surr): i + surr + 1] = True
            df = df[keep].reset_index(drop=True)
        else:
            print("NoSamplesError: no IG sample directories found under", self.dp_results_parent)
        self.df = df
        return df

    def _overview_plots(self, df):
        fig, ax = plt.subplots(figsize=(12, 8))
        for sid in df["sensor_id"].unique():
            sub = df[df["sensor_id"] == sid]
            ax.scatter(sub["date_time"], [sid] * len(sub), c=sub["color"], s=12, marker="|")
        ax.set_xlabel("Date and Time")
        ax.set_ylabel("sensor ID")
        ax.set_title("Analysed Samples per sensor ID")
        ax.legend(handles=[plt.Line2D([0], [0], color=COLOR_MAP[k], label=COLOR_NAMES[k]) for k in COLOR_MAP])
        fig.savefig(os.path.join(self.output_dir_analysis, "sensor_samples_time_range.png"), bbox_inches="tight")
        plt.close(fig)
        counts = df.groupby("sensor_id")["confusion_matrix"].value_counts().unstack().fillna(0)
        colors = [COLOR_MAP[k] for k in COLOR_MAP if COLOR_NAMES[k] in counts.columns]
        counts = counts[[COLOR_NAMES[k] for k in COLOR_MAP if COLOR_NAMES[k] in counts.columns]]
        ax = counts.plot(kind="barh", stacked=True, color=colors, alpha=0.6, edgecolor="k")
        ax.get_legend().set_title(None)
        ax.figure.savefig(os.path.join(self.output_dir_analysis, "sensor_samples_confusion_matrix.png"),
                          bbox_inches="tight")
        plt.close(ax.figure)

    # ----------------------------------------------------------------- aggregation
    def _spatial_mean(self, sid, classes, normalize: bool):
        """(node-mean feature gradients [T, C], anomalous-series gradients [T, C], n) averaged over
        the samples of sensor ``sid`` whose confusion class is in ``classes``; each sample optionally
        normalised by its max |gradient| first."""
        sub = self.df[(self.df["sensor_id"] == sid) & self.df["confusion_matrix_abbr"].isin(classes)]
        sf = sa = None
        n = 0
        for _, row in sub.iterrows():
            gf, ga = self._load(row, STEM_GF), self._load(row, STEM_GA)
            if gf is None and ga is None:
                continue
            if normalize:
                parts = [np.abs(a).reshape(-1) for a in (gf, ga) if a is not None]
                m = float(np.max(np.concatenate(parts))) if parts else 0.0
                if m > 0:
                    gf = gf / m if gf is not None else None
                    ga = ga / m if ga is not None else None
            f = gf.sum(0) / gf.shape[0] if gf is not None else None      # neighbour count varies: node mean
            sf = f if sf is None else sf + f
            sa = ga if sa is None else (sa + ga if ga is not None else sa)
            n += 1
        if n == 0:
            return None, None, 0
        return (sf / n if sf is not None else None), (sa / n if sa is not None else None), n

    def spatial_aggregate_gradients(self) -> dict:
        """Per sensor: mean over the selected samples (``spatial_aggregation.which_samples``) of the
        node-mean feature gradients and the anomalous-series gradients, optionally normalised per
        sample by the max |gradient| (``integrated_gradients_analyser.py`` spatial aggregation), saved
        as ``spatial_aggregated_gradients_{features,anom_ts}_<classes>.npy``; the per-class means the
        figure draws are kept too."""
        if self.df is None:
            self.get_overview(plots=False)
        which = list(self.an.spatial_aggregation.which_samples)
        normalize = bool(self.an.spatial_aggregation.normalize)
        out = {}
        for sid in self.selected_sensors:
            sf, sa, n = self._spatial_mean(sid, which, normalize)
            if n == 0:
                print("No samples found for", sid)
                continue
            d = os.path.join(self.output_dir_analysis, str(sid))
            os.makedirs(d, exist_ok=True)
            res = {"n_samples": n, "per_class": {}}
            if sf is not None:
                res["features"] = sf
                np.save(os.path.join(d, f"spatial_aggregated_gradients_features_{self.conf_matrix_string}.npy"), sf)
            if sa is not None:
                res["anom_ts"] = sa
                np.save(os.path.join(d, f"spatial_aggregated_gradients_anom_ts_{self.conf_matrix_string}.npy"), sa)
            for cls in which:
                cf, ca, cn = self._spatial_mean(sid, [cls], normalize)
                if cn:
                    res["per_class"][cls] = {"features": cf, "anom_ts": ca, "n_samples": cn}
            out[sid] = res
        self.spatial = out
        return out

    def plot_spatial_aggregated_gradients(self) -> List[str]:
        """The reference's figure (``integrated_gradients_analyser.py:811-964``): per confusion class of
        ``which_samples`` four banded rows - TL1 and TL2 of the flagged sensor's own series, then TL1
        and TL2 of the neighbours ("N", feature gradients scaled by ``scale_feature_gradients``) - on
        one fixed symmetric ``coolwarm`` scale (``spatial_aggregation.cbar_limit``, default the
        reference's 0.1), rows stacked without spacing, colour bar on the left. Saved as
        ``<sensor>/spatial_aggregated_gradients_<sensor>[_norm].png`` by the ``normalize`` flag, so the
        two normalisation runs keep both figures. Difference: every class's rows show that class's
        own mean (the reference draws the all-classes mean in each class's rows)."""
        if not hasattr(self, "spatial"):
            self.spatial_aggregate_gradients()
        sp = self.an.spatial_aggregation
        scale = float(sp.scale_feature_gradients)
        lim = float(sp.get("cbar_limit", 0.1) or 0.1)
        norm = mcolors.Normalize(vmin=-lim, vmax=lim)
        which = list(sp.which_samples)
        suffix = "_norm" if bool(sp.normalize) else ""
        n_rows = 4
        paths = []
        for sid, res in self.spatial.items():
            fig, ax = plt.subplots(len(which) * n_rows, 1, figsize=(16, 8), sharex=True, squeeze=False)
            ax = ax[:, 0]
            for a in ax:
                a.set_yticklabels([])
                a.tick_params(axis="y", labelrotation=90)
            pcol = None

            def band(v, a):
                v = np.asarray(v, dtype=np.float64)
                xs = np.arange(v.shape[0] + 1) - 0.5
                return a.pcolormesh(xs, np.array([0.0, 1.0]), v[None, :], norm=norm, alpha=0.8, cmap="coolwarm")

            for i, cls in enumerate(which):
                d = res["per_class"].get(cls)
                if d is None:
                    continue
                rows = []
                if d["anom_ts"] is not None:
                    rows += [(d["anom_ts"][:, k], lbl) for k, lbl in ((0, "TL1"), (1, "TL2")) if k < d["anom_ts"].shape[1]]
                if d["features"] is not None:
                    rows += [(d["features"][:, k] * scale, lbl) for k, lbl in ((0, "TL1\nN"), (1, "TL2\nN"))
                             if k < d["features"].shape[1]]
                for j, (v, lbl) in enumerate(rows[:n_rows]):
                    a = ax[i * n_rows + j]
                    pcol = band(v, a)
                    a.set_ylabel(lbl)
                    a.text(0.03, 0.5, cls, ha="center", va="center", transform=a.transAxes, fontsize=16)
            if pcol is None:
                plt.close(fig)
                print("No data for plotting found.")
                continue
            cbar_ax = fig.add_axes([0.07, 0.2, 0.01, 0.6])
            cbar = fig.colorbar(pcol, cax=cbar_ax, orientation="vertical", location="left")
            cbar.set_label("Attention")
            fig.text(0.5, 0.95, "Spatially Averaged Attention for sensor " + str(sid), fontsize=16, ha="center",
                     va="center")
            fig.subplots_adjust(hspace=0)
            p = os.path.join(self.output_dir_analysis, str(sid), f"spatial_aggregated_gradients_{sid}{suffix}.png")
            fig.savefig(p)
            plt.close(fig)
            paths.append(p)
        return paths

    def plot_agg_samples_over_time(self, sensor: str, time_from=None, time_to=None, agg_type: Optional[str] = None,
                                   norm_by_prediction: Optional[bool] = None, cbar_limits=None) -> Optional[str]:
        """Spatio-temporal attribution map of one sensor (``integrated_gradients_analyser.py:1169-1710``).

        Frames sit on a regular grid of ``aggregate_sample_along_time.interval`` seconds from
        ``time_from`` to ``time_to`` (default: the sensor's first / last sample); a grid time with
        no saved sample is a NaN frame (a gap stays a gap). Per frame: the flagged channels and
        every neighbour's channels at the window centre, the prediction, the outcome, and each
        series' attribution aggregated over the window's time steps (``agg_type``), optionally
        divided by the prediction (``norm_by_prediction``) - drawn as coloured bands under the
        series. A frame whose neighbour count differs from the first frame's is NaN, as in the
        reference. Written as ``agg_samples_over_time_<sensor>_<from>-<to>_<agg>[_norm].png`` in
        the analysis directory (the paper's script draws each range with and without the
        normalisation, ``run_integrated_gradients_analyser_20240318.py:25-36``)."""
        cfg = self.an.aggregate_sample_along_time
        agg_type = agg_type or cfg.agg_type
        norm_by_prediction = bool(cfg.norm_by_prediction if norm_by_prediction is None else norm_by_prediction)
        cbar_limits = cbar_limits if cbar_limits is not None else cfg.cbar_limits
        if self.df_unfiltered is None:
            self.get_overview(plots=False)
        sub = self.df_unfiltered[self.df_unfiltered["sensor_id"] == str(sensor)].sort_values("date_time")
        # each bound applies on its own; a missing one is the sensor's first / last sample
        if time_from is not None:
            time_from = pd.to_datetime(time_from)
            sub = sub[sub["date_time"] >= time_from]
        if time_to is not None:
            time_to = pd.to_datetime(time_to)
            sub = sub[sub["date_time"] <= time_to]
        if not len(sub):
            return None
        if time_from is None:
            time_from = sub["date_time"].min()
        if time_to is None:
            time_to = sub["date_time"].max()
        grid = pd.date_range(start=time_from, end=time_to, freq=pd.Timedelta(int(cfg.interval), unit="s"))
        if not len(grid):
            return None
        agg = {"mean": np.nanmean, "sum": np.nansum, "max": np.nanmax, "min": np.nanmin}[agg_type]
        tb = int(round(self.preproc_config.timestep_before / max(1, int(self.preproc_config.get("freq", 1) or 1))))
        scale = cfg.scale_feature_gradients
        by_time = {pd.Timestamp(r["date_time"]): r for _, r in sub.iterrows()}
        frames = []
        shape_nb = None
        for t in grid:
            row = by_time.get(pd.Timestamp(t))
            if row is None:
                frames.append(None)
                continue
            a, ga, gf, f = (self._load(row, k) for k in (STEM_A, STEM_GA, STEM_GF, STEM_F))
            p, y = self._load(row, STEM_P), self._load(row, STEM_Y)
            if a is None or ga is None or gf is None or f is None:
                frames.append(None)
                continue
            score = float(np.asarray(p).reshape(-1)[0]) if p is not None else np.nan
            if norm_by_prediction:
                ga, gf = ga / score, gf / score
            gf = gf / gf.shape[0] * 2 if scale == "auto" else gf * float(scale)
            if shape_nb is None:
                shape_nb = gf.shape
            if gf.shape != shape_nb:                   # the neighbour set changed: a missing frame
                frames.append(("nb", a, score, y))
                continue
            frames.append((a[min(tb, a.shape[0] - 1)], score, float(np.asarray(y).reshape(-1)[0]) if y is not None
                           else float(row["true"]), agg(ga, axis=0), agg(gf, axis=1), f[:, min(tb, f.shape[1] - 1)]))
        if shape_nb is None:
            return None
        n_nb, C = shape_nb[0], shape_nb[2]
        S = len(grid)
        anom_c = np.full((S, C), np.nan)
        pred = np.full(S, np.nan)
        flag = np.full(S, np.nan)
        ga_agg = np.full((S, C), np.nan)
        gf_agg = np.full((S, n_nb, C), np.nan)
        feat_c = np.full((S, n_nb, C), np.nan)
        for i, fr in enumerate(frames):
            if fr is None:
                continue
            if isinstance(fr[0], str):                 # neighbour set changed: series / score, no attribution
                _, a, score, y = fr
                anom_c[i] = a[min(tb, a.shape[0] - 1)]
                pred[i] = score
                continue
            anom_c[i], pred[i], flag[i], ga_agg[i], gf_agg[i], feat_c[i] = fr
        if isinstance(cbar_limits, (list, tuple)):
            vmin, vmax = float(cbar_limits[0]), float(cbar_limits[1])
        else:
            vmin, vmax = float(np.nanmin(gf_agg)), float(np.nanmax(gf_agg))
            if not np.isfinite(vmin) or vmin == vmax:
                vmin, vmax = -1.0, 1.0
        norm = mcolors.Normalize(vmin=vmin, vmax=vmax)
        group = bool(cfg.get("group_tl_channels", True))
        if group:
            import warnings
            with warnings.catch_warnings():           # (NaN frames: all-NaN rows are expected)
                warnings.simplefilter("ignore", RuntimeWarning)
                gf_rows = [(f"N{j} TL", feat_c[:, j, :], np.nanmean(gf_agg[:, j, :], axis=1)) for j in range(n_nb)]
        else:
            gf_rows = [(f"N{j} TL{c + 1}", feat_c[:, j, c:c + 1], gf_agg[:, j, c]) for j in range(n_nb) for c in range(C)]
        thr = float(self.ig.threshold)
        pred_cls = np.where(pred > thr, 1.0, np.where(np.isnan(pred), np.nan, 0.0))
        cval = {(0, 0): 0.0, (0, 1): 0.33, (1, 0): 0.66, (1, 1): 1.0}
        cvals = np.array([0.0 if (np.isnan(t) or np.isnan(q)) else cval[(int(t), int(q))]
                          for t, q in zip(flag, pred_cls)])
        cmap_cm = mcolors.LinearSegmentedColormap.from_list(
            "confusion", list(zip([0.0, 0.33, 0.66, 1.0], ["white", "orange", "red", "green"])))
        rows = 1 + C + len(gf_rows)
        fig, axes = plt.subplots(rows, 1, figsize=(max(8.0, S / 300), 2 + 0.5 + 0.9 * rows), sharex=True,
                                 squeeze=False)
        axes = axes[:, 0]
        X = np.linspace(-0.5, S - 0.5, S + 1)
        x = X[:-1] + 0.5
        ylims = cfg.ylims
        fixed = isinstance(ylims, (list, tuple))

        def band(ax, series, z):
            lo, hi = (float(ylims[0]), float(ylims[1])) if fixed else (np.nanmin(anom_c), np.nanmax(anom_c))
            if not np.isfinite(lo) or lo == hi:
                lo, hi = 0.0, 1.0
            m = ax.pcolormesh(X, [lo, hi], np.reshape(z, (1, S)), norm=norm, alpha=0.8, cmap="RdBu_r")
            for c in range(series.shape[1]):
                ax.plot(x, series[:, c], color=TL_COLORS[c % len(TL_COLORS)], linewidth=0.8)
            ax.set_ylim(lo, hi)
            return m

        top = axes[0]
        top.pcolormesh(X, [0, 1], cvals.reshape(1, S), alpha=0.2, cmap=cmap_cm, vmin=0, vmax=1)
        top.plot(x, pred, color="k", linewidth=0.8)
        top.set_ylim(0, 1)
        top.set_ylabel("Prediction")
        top.legend(handles=[plt.Rectangle((0, 0), 1, 1, facecolor=c, edgecolor="grey", alpha=0.2, label=l)
                            for c, l in zip(["white", "orange", "red", "green"], ["TN", "FP", "FN", "TP"])],
                   loc="upper center", bbox_to_anchor=(0.5, -0.05), ncol=4, frameon=False, fontsize=7)
        mesh = None
        for c in range(C):
            mesh = band(axes[1 + c], anom_c[:, c:c + 1], ga_agg[:, c])
            axes[1 + c].set_ylabel(f"TL {c + 1}", rotation=0, labelpad=30)
        axes[1].set_title("Flagged Sensor", fontsize=9)
        for k, (name, series, z) in enumerate(gf_rows):
            mesh = band(axes[1 + C + k], series, z)
            axes[1 + C + k].set_ylabel(name, rotation=0, labelpad=30, fontsize=7)
        if gf_rows:
            axes[1 + C].set_title("Self Reference Cycle and Neighbouring Sensors", fontsize=9)
        tick = max(1, S // 8)
        axes[-1].set_xlim(x[0], x[-1] if S > 1 else x[0] + 1)
        axes[-1].set_xticks(x[::tick])
        axes[-1].set_xticklabels([t.strftime("%m-%d %H:%M") for t in grid][::tick], rotation=30)
        if mesh is not None:
            fig.colorbar(mesh, ax=list(axes[1:]), shrink=0.6, orientation="vertical", label="Attribution")
        self.last_agg = {"times": grid, "prediction": pred, "flag_true": flag, "anom": anom_c,
                         "gradients_anom": ga_agg, "gradients_features": gf_agg, "features": feat_c}
        os.makedirs(self.output_dir_analysis, exist_ok=True)
        name = (f"agg_samples_over_time_{sensor}_{pd.Timestamp(time_from).strftime('%Y%m%d-%H%M%S')}-"
                f"{pd.Timestamp(time_to).strftime('%Y%m%d-%H%M%S')}_{agg_type}{'_norm' if norm_by_prediction else ''}.png")
        p = os.path.join(self.output_dir_analysis, name)
        fig.savefig(p, bbox_inches="tight")
        plt.close(fig)
        return p

    # ----------------------------------------------------------------- images / videos
    def concatenate_images(self) -> List[str]:
        """Stack each sample's heatmap over its classified-series plot (if both exist)."""
        from PIL import Image
        out = []
        scale = float(self.an.concat_images_scale)
        for _, row in (self.df if self.df is not None else self.get_overview(plots=False)).iterrows():
            imgs = sorted(p for p in os.listdir(row["path"]) if p.endswith(".png") and not p.startswith("concat_"))
            if len(imgs) < 2:
                continue
            dst = os.path.join(row["path"], f"concat_{row['sample_name']}.png")
            if os.path.exists(dst) and not self.an.overwrite_concat_images:
                continue
            ims = [Image.open(os.path.join(row["path"], p)).convert("RGB") for p in imgs]
            w = max(i.width for i in ims)
            canvas = Image.new("RGB", (w, sum(i.height for i in ims)), "white")
            y = 0
            for im in ims:
                canvas.paste(im, (0, y))
                y += im.height
            if scale != 1.0:
                canvas = canvas.resize((int(canvas.width * scale), int(canvas.height * scale)))
            canvas.save(dst)
            out.append(dst)
        return out

    def create_videos(self, sensor=None, time_from=None, time_to=None) -> List[str]:
        """Animated GIF per sensor of the IG heatmaps in time order (PIL; the reference
        also writes mp4 through imageio/ffmpeg, which this image does not ship)."""
        from PIL import Image, ImageDraw
        if self.df is None:
            self.get_overview(plots=False)
        fps = float(self.an.video.video_fps)
        sensors = [sensor] if sensor is not None else self.selected_sensors
        out = []
        for sid in sensors:
            sub = self.df[self.df["sensor_id"] == str(sid)]
            if time_from is not None:
                sub = sub[sub["date_time"] >= pd.to_datetime(time_from)]
            if time_to is not None:
                sub = sub[sub["date_time"] <= pd.to_datetime(time_to)]
            frames = []
            prefix = "concat_" if self.an.video.videos_from_concat_images else "ig_heatmap_"
            for k, (_, row) in enumerate(sub.iterrows()):
                cand = [p for p in os.listdir(row["path"]) if p.startswith(prefix) and p.endswith(".png")]
                if not cand:
                    continue
                im = Image.open(os.path.join(row["path"], cand[0])).convert("RGB")
                # progress bar coloured by the sample's outcome
                dr = ImageDraw.Draw(im)
                frac = (k + 1) / max(1, len(sub))
                dr.rectangle([0, im.height - 8, int(im.width * frac), im.height], fill=COLOR_MAP[(row["true"],
                                                                                                  row["pred"])])
                frames.append(im)
            if not frames:
                continue
            d = os.path.join(self.output_dir_analysis, str(sid))
            os.makedirs(d, exist_ok=True)
            p = os.path.join(d, f"ig_{sid}_{self.conf_matrix_string}.gif")
            frames[0].save(p, save_all=True, append_images=frames[1:], duration=int(1000 / fps), loop=0)
            out.append(p)
        return out

    # ----------------------------------------------------------------- maintenance
    def scale_gradients_with_input(self, dont_scale: Optional[List[str]] = None) -> int:
        """Multiply saved gradients by the saved inputs in place (zero baseline; for results
        produced with ``scale_gradients: false``)."""
        if self.df is None:
            self.get_overview(plots=False)
        skip = set(dont_scale or [])
        n = 0
        for _, row in self.df[self.df["sensor_id"].isin(self.selected_sensors)].iterrows():
            if row["sample_name"] in skip:
                continue
            for gs, fs in ((STEM_GF, STEM_F), (STEM_GA, STEM_A)):
                g, f = self._load(row, gs), self._load(row, fs)
                if g is None or f is None:
                    continue
                np.save(os.path.join(row["path"], self.get_filename(gs, row["sample_name"]) + ".npy"), g * f)
            n += 1
        return n

    def rename_based_on_threshold(self, threshold: Optional[float] = None) -> int:
        """Re-derive the predicted class of each sample from its saved score and rename
        its directory / files (``..._<true>_<pred>``)."""
        thr = float(self.ig.threshold if threshold is None else threshold)
        if self.df is None:
            self.get_overview(plots=False)
        n = 0
        for _, row in self.df_unfiltered[self.df_unfiltered["sensor_id"].isin(self.selected_sensors)].iterrows():
            p = self._load(row, STEM_P)
            if p is None:
                continue
            cls = int(float(np.asarray(p).reshape(-1)[0]) > thr)
            if cls == row["pred"]:
                continue
            old = row["sample_name"]
            new = old[:-1] + str(cls)
            for f in os.listdir(row["path"]):
                if old in f:
                    os.rename(os.path.join(row["path"], f), os.path.join(row["path"], f.replace(old, new)))
            os.rename(row["path"], os.path.join(os.path.dirname(row["path"]), new))
            n += 1
        self.get_overview(plots=False)
        return n


def run_analyser(args):
    import json
    from ..cli.common import load_configs
    pc, mc = load_configs(args)
    xc = C.load(args.xai_config) if args.xai_config else C.default("xai_ig")
    xc["output_dir"] = args.xai_dir
    an = IntegrateGradientsAnalyser(pc, mc, xc)
    df = an.get_overview()
    agg = an.spatial_aggregate_gradients()
    plots = an.plot_spatial_aggregated_gradients()
    for s in an.selected_sensors[:4]:
        an.plot_agg_samples_over_time(s)
    print(json.dumps({"samples": int(len(df)), "sensors": len(an.selected_sensors), "aggregated": len(agg),
                      "plots": len(plots), "output_dir": an.output_dir_analysis}))


__all__ = ["IntegrateGradientsAnalyser", "run_analyser", "COLOR_MAP", "COLOR_NAMES"]
