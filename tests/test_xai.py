"""Integrated gradients engine, explainer output layout, analyser, plots."""
import os

import numpy as np
import pytest
import torch

from gnnqc import config as C
from gnnqc.data.preprocessing import create_windows_dataset
from gnnqc.data.store import DeviceStore
from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
from gnnqc.models import create_model
from gnnqc.xai.ig import IntegratedGradients, IntegratedGradientsExplainer, completeness_gap, trapezoid_weights


@pytest.fixture(scope="module")
def cml_small():
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    ws = create_windows_dataset(pc, raw=make_cml_raw(n_sensors=8, n_minutes=2 * 1440, seed=5))
    return pc, ws, DeviceStore(ws, "rolling_median", pc.graph)


def _sharp(model, gain=40.0):
    """Random-init outputs sit at ~0.5; scale the output layer so IG has something to explain."""
    with torch.no_grad():
        model.dense_out.kernel.mul_(gain)
    return model.eval()


def _sequential_ig(model, batch, m):
    """Reference semantics (``integrated_gradients.py:955-1015``): one pass per alpha."""
    xs, gx, ga = batch.x, [], []
    for a in torch.linspace(0, 1, m + 1):
        x = (a * batch.x).requires_grad_(True)
        an = (a * batch.anom).requires_grad_(True)
        y = model((x, an, batch.adj, batch.node_mask, batch.anom_pos)).reshape(-1)
        g1, g2 = torch.autograd.grad(y.sum(), [x, an])
        gx.append(g1)
        ga.append(g2)
    gx, ga = torch.stack(gx), torch.stack(ga)
    ix = ((gx[:-1] + gx[1:]) / 2).mean(0) * xs
    ia = ((ga[:-1] + ga[1:]) / 2).mean(0) * batch.anom
    return ix, ia


def test_trapezoid_weights():
    w = trapezoid_weights(4)
    g = torch.arange(5.0)
    assert torch.isclose((w * g).sum(), ((g[:-1] + g[1:]) / 2).mean())


def test_alpha_batched_matches_sequential(cml_small):
    pc, ws, store = cml_small
    torch.manual_seed(1)
    model = _sharp(create_model(C.default("model_cml"), pc))
    for p in model.parameters():
        p.requires_grad_(False)
    b = store.gather(torch.arange(0, 40, 8))
    ix, ia = _sequential_ig(model, b, 6)
    for max_rows in (5, 12, 10_000):            # alpha chunking must not change the result
        r = IntegratedGradients(model, "cml", m_steps=6, max_rows=max_rows).attribute(b)
        torch.testing.assert_close(r["grad_x"], ix, atol=1e-6, rtol=1e-4)
        torch.testing.assert_close(r["grad_anom"], ia, atol=1e-6, rtol=1e-4)
    # weights left trainable state untouched by the engine
    assert all(not p.requires_grad for p in model.parameters())


def test_completeness_improves_with_steps(cml_small):
    pc, ws, store = cml_small
    torch.manual_seed(2)
    model = _sharp(create_model(C.default("model_cml"), pc, baseline=True), 60.0)
    b = store.gather(torch.arange(0, 60, 6))
    gaps = []
    for m in (4, 64):
        r = IntegratedGradients(model, "cml", m_steps=m).attribute(b)
        delta = (r["path_pred"][-1] - r["path_pred"][0]).abs()
        gaps.append(float(completeness_gap(r).abs().max() / delta.max().clamp(min=1e-6)))
    assert gaps[1] < 0.05 and gaps[1] <= gaps[0] + 1e-6


def test_soilnet_target_node():
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    pc["timestep_before"], pc["timestep_after"] = 360, 60         # T = 29 survives three pool-3 stages
    pc = C.normalize_preproc(pc)
    ws = create_windows_dataset(pc, raw=make_soilnet_raw(n_boxes=4, n_time=6 * 96, seed=2))
    store = DeviceStore(ws, "scale_range", pc.graph)
    torch.manual_seed(0)
    model = _sharp(create_model(C.default("model_soilnet"), pc))
    b = store.gather(torch.arange(3))
    r = IntegratedGradients(model, "soilnet", m_steps=4).attribute(b)
    assert r["grad_x"].shape == b.x.shape and r["target"].shape == (3,)
    assert bool((b.node_mask.gather(1, r["target"][:, None]) > 0).all())


def test_explainer_writes_reference_layout_and_analyser(cml_small, tmp_path):
    from gnnqc.ckpt import save_model
    from gnnqc.xai.analyse import IntegrateGradientsAnalyser
    pc, ws, _ = cml_small
    torch.manual_seed(3)
    mc = C.default("model_cml")
    model = _sharp(create_model(mc, pc))
    mdir = str(tmp_path / "model")
    save_model(model, mdir, preproc_config=pc)
    mc["model_path"] = mdir
    xc = C.default("xai_ig")
    xc["output_dir"] = str(tmp_path / "xplain")
    ig = xc.integrated_gradients
    ig["m_steps"], ig["dataset"], ig["threshold"], ig["plot_heatmap"] = 4, "all", 0.5, True
    ig["plot_gradient_saturation"] = True
    pc2 = C.Config(dict(pc))
    pc2["batch_size"] = 16
    ex = IntegratedGradientsExplainer(pc2, mc, xc, windows=ws, device="cpu")
    ex.prepare_data()
    ex.sample_ids = ex.sample_ids[:32]
    res = ex.get_gradients()
    assert len(res) == 32                       # all four confusion classes selected
    r0 = res[0]
    stem = r0["file_stem"]
    for k in ("gradients_features_unwrapped", "gradients_anom_ts_unwrapped", "features_unwrapped",
              "anom_ts_unwrapped", "predictions_unwrapped", "anomaly_flag_true_unwrapped"):
        assert os.path.exists(os.path.join(r0["dir"], f"{k}_{stem}.npy")), k
    gf = np.load(os.path.join(r0["dir"], f"gradients_features_unwrapped_{stem}.npy"))
    f = np.load(os.path.join(r0["dir"], f"features_unwrapped_{stem}.npy"))
    assert gf.shape == f.shape and gf.shape[1] == ws.seq_len     # [n_nodes, T, C]
    assert os.path.exists(os.path.join(r0["dir"], f"ig_heatmap_{stem}.png"))
    assert os.path.basename(r0["dir"]).startswith(r0["sensor"] + "_")
    assert os.path.exists(os.path.join(ex.output_dir, "log", "log.txt"))

    xc.integrated_gradients.analyser["which_samples"] = ["TP", "FP", "TN", "FN"]
    xc.integrated_gradients.analyser.spatial_aggregation["which_samples"] = ["TP", "FP", "TN", "FN"]
    an = IntegrateGradientsAnalyser(pc2, mc, xc)
    df = an.get_overview()
    assert len(df) == 32
    agg = an.spatial_aggregate_gradients()
    sid = r0["sensor"]
    assert agg[sid]["features"].shape == (ws.seq_len, 2) and agg[sid]["anom_ts"].shape == (ws.seq_len, 2)
    assert an.plot_spatial_aggregated_gradients()
    assert an.plot_agg_samples_over_time(sid) is not None
    gifs = an.create_videos()
    assert gifs and os.path.getsize(gifs[0]) > 0
    # re-threshold: everything above 0 becomes positive -> directories renamed to *_1
    n = an.rename_based_on_threshold(threshold=0.0)
    assert n >= 0 and (an.df_unfiltered["pred"] == 1).all()


def test_roc_and_result_plots(cml_small, tmp_path):
    from gnnqc.eval.metrics import roc_curve
    from gnnqc.viz import extract_target_info, plot_results, plot_roc_curves
    pc, ws, store = cml_small
    rng = np.random.default_rng(0)
    y = rng.integers(0, 2, 300)
    p = np.clip(y * 0.4 + rng.random(300) * 0.6, 0, 1)
    fpr, tpr, thr = roc_curve(y, p)
    out = plot_roc_curves([fpr], [tpr], None, [thr], [0.5], str(tmp_path / "roc.png"), ["GCN"])
    assert os.path.getsize(out) > 0
    ids = np.arange(min(200, ws.n_windows))
    sids, dates, flags = extract_target_info(ws, ids)
    assert len(sids) == len(ids) == len(dates)
    mc = C.Config({"plotting": {"outdir": str(tmp_path / "plots"), "alpha": 0.2, "plot_time_range": 24}})
    paths = plot_results(sids, dates, (rng.random(len(ids)) > 0.5).astype(int), flags, rng.random(len(ids)), pc, mc,
                         windows=ws)
    assert paths and all(os.path.exists(q) for q in paths)


def test_explainer_shards_partition_batches(cml_small, tmp_path):
    """--shard i/n splits the batches round-robin like the SLURM array path; the shards
    together cover exactly the unsharded sample set."""
    from gnnqc.ckpt import save_model
    pc, ws, _ = cml_small
    torch.manual_seed(3)
    mc = C.default("model_cml")
    model = _sharp(create_model(mc, pc))
    mdir = str(tmp_path / "model")
    save_model(model, mdir, preproc_config=pc)
    mc["model_path"] = mdir
    pc2 = C.Config(dict(pc))
    pc2["batch_size"] = 8

    def run(shard, out):
        xc = C.default("xai_ig")
        xc["output_dir"] = str(tmp_path / out)
        ig = xc.integrated_gradients
        ig["m_steps"], ig["dataset"], ig["threshold"] = 2, "all", 0.5
        ex = IntegratedGradientsExplainer(pc2, mc, xc, windows=ws, device="cpu", shard=shard)
        ex.prepare_data()
        ex.sample_ids = ex.sample_ids[:24]
        return {(r["sensor"], r["file_stem"]) for r in ex.get_gradients()}

    full = run(None, "all")
    a, b = run("0/2", "s0"), run("1/2", "s1")
    assert a and b and not (a & b)
    assert a | b == full
    with pytest.raises(ValueError):
        run("2/2", "bad")


def test_classified_timeseries_plots(cml_small, tmp_path):
    """plot_classified_timeseries (raw series shaded per classified step) and the neighbours figure
    (flagged link + every neighbour of its graph, distances in the titles), from a real model's
    predictions and from given ones."""
    from gnnqc.viz import (classified_timeseries_figure_with_neighbours, plot_classified_timeseries,
                           plot_classified_timeseries_with_neighbours)
    pc, ws, store = cml_small
    torch.manual_seed(0)
    mc = C.default("model_cml")
    mc["plotting"] = {"outdir": str(tmp_path / "plots"), "alpha": 0.2, "plot_time_range": 24}
    model = create_model(mc, pc)
    ids = np.arange(min(120, ws.n_windows))
    paths = plot_classified_timeseries(model, store, ids, mc, max_figures=3)
    assert paths and all(os.path.getsize(q) > 0 for q in paths)
    rng = np.random.default_rng(1)
    paths2 = plot_classified_timeseries(None, store, ids, mc, predictions=rng.random(len(ids)), max_figures=2)
    assert paths2 and all(os.path.exists(q) for q in paths2)
    pn = plot_classified_timeseries_with_neighbours(model, store, ids, mc, max_figures=2)
    assert pn and all(os.path.getsize(q) > 0 for q in pn) and all("_neighbours.png" in q for q in pn)
    # direct call: 3 sensors x 50 steps x 2 channels, the middle one flagged
    d = np.arange("2019-07-01T00:00", "2019-07-01T00:50", dtype="datetime64[m]")
    feats = rng.normal(size=(3, 50, 2))
    true = np.where(rng.random(50) > 0.5, 1.0, 0.0)
    pred = np.where(rng.random(50) > 0.5, 1.0, 0.0)
    q = classified_timeseries_figure_with_neighbours(["a", "b", "c"], feats, d, true, pred, mc, [False, True, False],
                                                     probabilities=rng.random(50), distances=[1.5, 0.0, 3.2])
    assert os.path.getsize(q) > 0 and os.path.basename(q).startswith("b_")


def test_reference_run_scripts_golden(cml_small, tmp_path):
    """The call sequences of xai/notebooks/run_integrated_gradients_20240318.py and
    run_integrated_gradients_analyser_20240318.py on a synthetic explainer run: per-sensor,
    per-time-range heatmaps (no overwrite, round-robin worker split), the optional per-sample plots,
    and the analyser's aggregated-over-time figures for both normalisation modes on an
    ``interval`` grid with a missing sample (NaN frame), each under its own file name."""
    import pandas as pd
    from gnnqc.ckpt import save_model
    from gnnqc.viz.ig import list_sample_dirs
    from gnnqc.xai.analyse import IntegrateGradientsAnalyser
    pc, ws, _ = cml_small
    torch.manual_seed(4)
    mc = C.default("model_cml")
    mc["plotting"] = {"outdir": str(tmp_path / "plots"), "alpha": 0.2}
    model = _sharp(create_model(mc, pc))
    mdir = str(tmp_path / "model")
    save_model(model, mdir, preproc_config=pc)
    mc["model_path"] = mdir
    pc2 = C.Config(dict(pc))
    pc2["batch_size"] = 16

    def xcfg():
        xc = C.default("xai_ig")
        xc["output_dir"] = str(tmp_path / "xplain")
        ig = xc.integrated_gradients
        ig["m_steps"], ig["dataset"], ig["threshold"] = 4, "all", 0.5
        ig["plot_interpolated_data_element_series"] = True
        ig["plot_classified_timeseries_sample"] = True
        return xc

    ex = IntegratedGradientsExplainer(pc2, mc, xcfg(), windows=ws, device="cpu")
    ex.prepare_data()
    ex.sample_ids = ex.sample_ids[:48]
    res = ex.get_gradients()
    assert len(res) == 48
    for bid in range(3):
        for k in (1, 2):
            assert os.path.exists(os.path.join(ex.output_dir, f"interpolated_data_element_{k}_batch_{bid}.png"))
    for r in res:
        assert os.path.exists(os.path.join(r["dir"], f"anomalous_ts_{r['file_stem']}.png"))
    # the script: two sensors, each with its own time range
    sensors = sorted({r["sensor"] for r in res})
    s1 = sensors[0]
    t1 = sorted(pd.to_datetime(r["date"], format="%Y%m%d_%H%M%S") for r in res if r["sensor"] == s1)
    lo, hi = t1[len(t1) // 4], t1[3 * len(t1) // 4]
    want = {os.path.basename(r["dir"]) for r in res if r["sensor"] == s1
            and lo <= pd.to_datetime(r["date"], format="%Y%m%d_%H%M%S") <= hi}
    out = ex.plot_ig_heatmap_from_directory(sensors=[s1], time_from=str(lo), time_to=str(hi))
    assert {os.path.basename(os.path.dirname(p)) for p in out} == want and len(out) == len(want)
    stem = ex._file_name()
    for p in out:
        d = os.path.basename(os.path.dirname(p))
        assert os.path.basename(p) == f"ig_heatmap_{stem}_{d}.png"
    assert ex.plot_ig_heatmap_from_directory(sensors=[s1], time_from=str(lo), time_to=str(hi)) == []  # no overwrite
    assert len(ex.plot_ig_heatmap_from_directory(sensors=[s1], time_from=str(lo), time_to=str(hi),
                                                 overwrite=True)) == len(want)
    # SLURM-style split of the same selection: disjoint, together the whole set
    parts = []
    for i in range(2):
        exi = IntegratedGradientsExplainer(pc2, mc, xcfg(), windows=ws, device="cpu", shard=f"{i}/2")
        parts.append({os.path.dirname(p) for p in exi.plot_ig_heatmap_from_directory(overwrite=True)})
    allp = {os.path.join(ex.output_dir, s, d) for s, d in list_sample_dirs(ex.output_dir)}
    assert parts[0] and parts[1] and not (parts[0] & parts[1]) and parts[0] | parts[1] == allp

    # analyser script: overview, spatial aggregation, videos, both normalisation modes
    xc = xcfg()
    xc.integrated_gradients.analyser["which_sensors"] = [s1]
    xc.integrated_gradients.analyser.spatial_aggregation["which_samples"] = ["TP", "FP", "TN", "FN"]
    an = IntegrateGradientsAnalyser(pc2, mc, xc)
    an.get_overview()
    an.spatial_aggregate_gradients()
    (pn,) = an.plot_spatial_aggregated_gradients()
    assert os.path.basename(pn) == f"spatial_aggregated_gradients_{s1}_norm.png"
    # the script's second pass with normalize off writes its own figure (both are kept)
    xc.integrated_gradients.analyser.spatial_aggregation["normalize"] = False
    an = IntegrateGradientsAnalyser(pc2, mc, xc)
    an.get_overview(plots=False)
    an.spatial_aggregate_gradients()
    (pr,) = an.plot_spatial_aggregated_gradients()
    assert os.path.basename(pr) == f"spatial_aggregated_gradients_{s1}.png"
    assert os.path.exists(pn) and os.path.exists(pr) and os.path.dirname(pn) == os.path.dirname(pr)
    res = an.spatial[s1]
    assert set(res["per_class"]) <= {"TP", "FP", "TN", "FN"} and res["per_class"]
    assert sum(d["n_samples"] for d in res["per_class"].values()) == res["n_samples"]
    assert an.create_videos(sensor=s1, time_from=str(lo), time_to=str(hi))
    # a gap: one sample of the range removed -> its grid frame is NaN
    gap = sorted(want)[1]
    import shutil
    shutil.rmtree(os.path.join(ex.output_dir, s1, gap))
    an.get_overview(plots=False)
    p0 = an.plot_agg_samples_over_time(sensor=s1, time_from=str(lo), time_to=str(hi), agg_type="mean",
                                       norm_by_prediction=False, cbar_limits=(-0.015, 0.015))
    agg0 = an.last_agg
    p1 = an.plot_agg_samples_over_time(sensor=s1, time_from=str(lo), time_to=str(hi), agg_type="mean",
                                       norm_by_prediction=True, cbar_limits=(-0.015, 0.015))
    fmt = "%Y%m%d-%H%M%S"
    rng_s = f"{pd.Timestamp(lo).strftime(fmt)}-{pd.Timestamp(hi).strftime(fmt)}"
    assert os.path.basename(p0) == f"agg_samples_over_time_{s1}_{rng_s}_mean.png"
    assert os.path.basename(p1) == f"agg_samples_over_time_{s1}_{rng_s}_mean_norm.png"
    assert os.path.exists(p0) and os.path.exists(p1)
    grid = agg0["times"]
    assert len(grid) == int((hi - lo) / pd.Timedelta(60, unit="s")) + 1
    gt = pd.to_datetime(parse_gap := gap.rsplit("_", 4)[1] + "_" + gap.rsplit("_", 4)[2], format="%Y%m%d_%H%M%S")
    k = list(grid).index(gt)
    assert np.isnan(agg0["prediction"][k]) and np.isnan(agg0["gradients_features"][k]).all()
    assert np.isfinite(agg0["prediction"]).sum() == len(want) - 1
    assert parse_gap


def test_soilnet_result_plots_automatic_flags(tmp_path):
    """SoilNet plot_results with the raw dataset: the automatic-flag state (Auto flags -> 1,
    unlabelled -> NaN, else 0), the 'Automatic flag' / 'No data' bands with the reference's NaN
    semantics, and the battery-voltage twin axis (libs/visualize.py:200-215,285-291,351-359)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from gnnqc.viz import extract_target_info, plot_results
    from gnnqc.viz.results import _soil_strip, soilnet_plot_series
    raw = make_soilnet_raw(n_boxes=3, n_time=20 * 96, seed=4)
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    pc["min_date"], pc["max_date"] = str(raw.time[0]), str(raw.time[-1])
    ws = create_windows_dataset(pc, raw=raw)
    sp = soilnet_plot_series(raw)
    nl = np.asarray(raw["moisture_flag_no_label"].values, bool)
    au = np.zeros_like(nl)
    for k in ("moisture_flag_Auto:BattV", "moisture_flag_Auto:Range", "moisture_flag_Auto:Spike"):
        au |= np.asarray(raw[k].values, bool)
    a = sp["automatic_flags"]
    assert au.any() and (a[au] == 1).all()
    assert np.isnan(a[nl & ~au]).all() and (a[~nl & ~au] == 0).all()
    # the strip: automatic band covers auto-flagged AND unlabelled steps; 'No data' only labelled ones
    fig, ax = plt.subplots()
    d = np.arange("2014-08-01T00:00", "2014-08-01T02:00", 15, dtype="datetime64[m]").astype(object)
    auto = np.array([1.0, np.nan, 0.0, 0.0, 0.0, 0.0, 1.0, np.nan])
    true = np.array([np.nan, np.nan, np.nan, 0.0, 1.0, 1.0, 0.0, np.nan])
    pred = np.array([np.nan, np.nan, np.nan, 0.0, 1.0, 0.0, 1.0, np.nan])
    _soil_strip(ax, d, pred, true, auto, 0, 1, 0.2)
    labels = [c.get_label() for c in ax.collections]
    assert "Automatic flag" in labels and "No data" in labels and "True Positive" in labels
    plt.close(fig)
    ids = np.arange(0, ws.n_windows, max(1, ws.n_windows // 30))
    sids, dates, flags = extract_target_info(ws, ids)
    rng = np.random.default_rng(0)
    mc = C.Config({"plotting": {"outdir": str(tmp_path / "plots"), "alpha": 0.2, "plot_time_range": 72}})
    paths = plot_results(sids, dates, (rng.random(len(sids)) > 0.5).astype(int), flags, rng.random(len(sids)), pc, mc,
                         windows=ws, raw=raw, max_figures=3)
    assert paths and all(os.path.getsize(q) > 0 for q in paths)
