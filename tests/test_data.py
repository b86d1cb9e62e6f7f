"""Preprocessing golden tests."""
import numpy as np
import pandas as pd
import pytest
import torch

from gnnqc import config as C
from gnnqc.data import geo
from gnnqc.data.interp import interpolate_gaps
from gnnqc.data.raw_io import SensorData, read_netcdf, write_netcdf
from gnnqc.data.preprocessing import create_windows_dataset
from gnnqc.data.splits import chronological_split, kfold_split, monthly_random_split
from gnnqc.data.stats import rolling_stats
from gnnqc.data.synthetic import make_cml_raw, make_soilnet_raw
from gnnqc.data.targets import create_target
from gnnqc.data.windows import build_window_index, SensorGroup


def test_config_roundtrip_and_overrides(tmp_path):
    c = C.default("preprocessing_cml")
    c = C.normalize_preproc(c)
    assert c.dataset.train_fraction == c.train_fraction
    C.parse_overrides(c, ["graph.max_sample_distance=15", "batch_size=64"])
    assert c.graph.max_sample_distance == 15 and c.batch_size == 64
    p = tmp_path / "c.yml"
    C.save(c, str(p))
    c2 = C.load(str(p))
    assert c2.graph.max_sample_distance == 15
    assert C.sequence_length(c2) == 181
    s = C.normalize_preproc(C.default("preprocessing_soilnet"))
    assert C.sequence_length(s) == 337
    merged = {**C.default("preprocessing_cml"), **C.default("model_cml")}   # reference merges like this
    assert "epochs" in merged and "ds_type" in merged


def test_vincenty_known_distances():
    # 1 degree of latitude at the equator on WGS84 = 110574.4 m
    d = geo.vincenty_inverse(0.0, 0.0, 1.0, 0.0)
    assert abs(d - 110574.389) < 0.01
    # Flinders Peak -> Buninyong (Vincenty 1975 test): 54972.271 m
    d = geo.vincenty_inverse(-37.95103342, 144.42486789, -37.65282114, 143.92649554)
    assert abs(d - 54972.271) < 0.01
    m = geo.geodesic_distance_matrix([51.0, 51.1, 51.0], [7.0, 7.0, 7.1], unit="km")
    assert np.allclose(m, m.T) and np.all(np.diag(m) == 0)


def test_utm_roundtrip():
    lat, lon = np.array([51.35, 51.36]), np.array([12.43, 12.41])
    e, n = geo.wgs84_to_utm(lat, lon, 33)
    lat2, lon2 = geo.utm_to_wgs84(e, n, 33)
    assert np.allclose(lat, lat2, atol=1e-9) and np.allclose(lon, lon2, atol=1e-9)


def test_interpolation_max_gap():
    t = np.arange(np.datetime64("2019-07-01T00:00"), np.datetime64("2019-07-01T00:20"), np.timedelta64(1, "m"))
    x = np.arange(20, dtype=float)
    x[[0, 3, 4, 5, 6, 10, 11, 12, 13, 14, 15, 19]] = np.nan
    y = interpolate_gaps(x[None], t, np.timedelta64(5, "m"))[0]
    assert np.isnan(y[0]) and np.isnan(y[19])                  # no extrapolation
    assert np.allclose(y[3:7], [3, 4, 5, 6])                    # gap 2->7 = 5 min: filled
    assert np.isnan(y[10:16]).all()                             # gap 9->16 = 7 min: kept


@pytest.mark.parametrize("w", [1, 7, 50])
def test_rolling_stats_match_pandas(w):
    rng = np.random.default_rng(0)
    x = rng.normal(size=(5, 300)).astype(np.float32)
    x[1, 20:60] = np.nan
    x[2, :5] = np.nan
    r = rolling_stats(x, w)
    p = rolling_stats(x, w, backend="pandas")
    for k in r:
        assert np.array_equal(np.isnan(r[k]), np.isnan(p[k]))
        assert np.nanmax(np.abs(r[k] - p[k])) < 1e-4


def test_cml_target_and_netcdf_roundtrip(tmp_path):
    ds = make_cml_raw(n_sensors=6, n_minutes=1440, seed=2)
    tgt = create_target(ds, ds_type="cml")
    # recompute by definition: >=3 of 4 experts in any variable
    manual = np.zeros_like(tgt)
    for k in ("Jump", "Dew", "Fluctuation", "Unknown anomaly"):
        manual |= ds[k].data.sum(0) >= 3
    assert np.array_equal(tgt, manual)
    p = str(tmp_path / "raw.nc")
    write_netcdf(ds, p)
    ds2 = read_netcdf(p)
    assert np.array_equal(ds2.sensor_ids, ds.sensor_ids)
    assert np.array_equal(ds2.time, ds.time)
    assert np.array_equal(ds2["Unknown anomaly"].data, ds["Unknown anomaly"].data)
    assert np.allclose(ds2["TL_1"].data, ds["TL_1"].data, equal_nan=True)


def test_soilnet_target_rules():
    ds = make_soilnet_raw(n_boxes=3, n_time=400, seed=1)
    t = create_target(ds, ds_type="soilnet")
    m = ds["moisture"].data
    ok = ds["moisture_flag_OK"].data
    man = ds["moisture_flag_Manual"].data
    inr = (m > 0) & (m < 100)
    assert np.all(t[ok & inr & ~man] == 0)
    assert np.all(t[man & inr] == 1)
    assert np.all(np.isnan(t[~((ok | man) & inr)]))


def _toy_group():
    T = 40
    time = np.arange(np.datetime64("2019-07-01T00:00"), np.datetime64("2019-07-01T00:00") + np.timedelta64(T, "m"))
    feats = np.ones((3, 2, T), np.float32)
    feats[0, 0, 25] = np.nan      # flagged sensor NaN at t=25
    feats[2, 1, 8] = np.nan       # neighbour NaN at t=8
    target = np.zeros(T, bool)
    target[12] = True
    return SensorGroup("s0", "cml", np.array(["a", "b", "c"]), 0, ["TL_1", "TL_2"], feats, time, target,
                       np.zeros((3, 3)))


def test_cml_window_rules():
    g = _toy_group()
    ix = build_window_index(g, 0, timestep_before=4, timestep_after=2, freq=1)
    c = ix.center
    assert c.min() == 4 and c.max() == 37                      # window must fit in the series
    assert not np.any((c >= 23) & (c <= 29))                   # flagged NaN at 25 -> skipped
    row = np.nonzero(c == 10)[0][0]
    assert ix.node_valid[row].tolist() == [True, True, False]  # neighbour NaN at 8 dropped
    assert ix.labels[np.nonzero(c == 12)[0][0]] == 1


def test_splits():
    days = np.repeat(np.arange(np.datetime64("2019-07-01"), np.datetime64("2019-07-29")), 10)
    tr, va, te = chronological_split(days, 0.6, 0.2, 120, 60)
    assert tr.sum() and va.sum() and te.sum()
    assert days[tr].max() < days[va].min() < days[te].min()
    # one-day gap before validation (ceil(180/1440) = 1)
    assert (days[va].min() - days[tr].max()).astype(int) >= 2
    fn = np.arange(100)
    folds = [kfold_split(fn, 5, k)[1] for k in range(5)]
    assert np.all(np.sum(folds, axis=0) == 1)                   # every file in exactly one test fold
    tr0, te0 = kfold_split(fn, 5, 0, gap=3)
    assert not tr0[te0].any() and not tr0[20:23].any()
    mdays = np.arange(np.datetime64("2014-01-01"), np.datetime64("2015-01-01"))
    a, b, c = monthly_random_split(mdays, 0.6, 0.2, 4320, 720, seed=1)
    assert not (a & b).any() and not (a & c).any() and not (b & c).any()


def test_store_and_sharded_loader(cml_windows):
    from gnnqc.data.store import DeviceLoader, DeviceStore
    pc, ws = cml_windows
    st = DeviceStore(ws, "rolling_median", pc.graph)
    ids = np.arange(st.n_windows)
    # shards of 3 ranks are disjoint and cover everything
    seen = []
    for r in range(3):
        L = DeviceLoader(st, ids, 16, shuffle=True, seed=1, rank=r, world_size=3)
        rows = L.batch_ids()
        assert rows.shape[1] == 16
        seen.append(rows[rows >= 0])
    allw = torch.cat(seen)
    assert allw.numel() == st.n_windows and torch.unique(allw).numel() == st.n_windows
    b = st.gather(torch.tensor([0, 3, -1]))
    assert b.x.shape == (3, 181, st.n_nodes, 2)
    assert b.y_mask.tolist() == [1.0, 1.0, 0.0]
    assert float(b.x[2].abs().sum()) == 0.0
    # normalisation: rolling median at the centre subtracted per node
    g = ws.groups[0]
    c = int(ws.indices[0].center[3])
    med = g.stats["TL_1_rolling_median"][:, c]
    raw = g.features[:, 0, c]
    valid = b.node_mask[1].numpy() > 0
    n = g.n_nodes
    got = b.x[1, ws.timestep_before, :n, 0].numpy()
    assert np.allclose(got[valid[:n]], (raw - med)[valid[:n]], atol=1e-4)
    # adjacency restricted to valid nodes, with self loops
    A = b.adj[1].numpy()
    assert np.all(np.diag(A)[valid] == 1) and np.all(A[~valid] == 0)


def test_soilnet_windows_and_store():
    from gnnqc.data.preprocessing import create_windows_dataset
    from gnnqc.data.store import DeviceStore
    pc = C.normalize_preproc(C.default("preprocessing_soilnet"))
    pc.timestep_before, pc.timestep_after = 300, 60
    ws = create_windows_dataset(pc, raw=make_soilnet_raw(n_boxes=4, n_time=600, seed=3))
    assert ws.n_windows > 0
    st = DeviceStore(ws, "scale_range", pc.graph)
    b = st.gather(torch.arange(4))
    assert b.y.shape == b.node_mask.shape
    assert torch.all(b.y_mask <= b.node_mask)
    # scale_range: moisture/60
    g = ws.groups[0]
    c = int(ws.indices[0].center[0])
    tb = 300 // 15
    n0 = int(torch.nonzero(b.node_mask[0])[0])
    assert abs(float(b.x[0, tb, n0, 0]) - g.features[n0, 0, c] / 60.0) < 1e-5


@pytest.mark.parametrize("ds", ["cml", "soilnet"])
def test_tfrecord_roundtrip_matches_device_store(ds, tmp_path):
    """Windows written as SequenceExample TFRecords (reference ``create_example`` layout)
    and read back give the same normalised node tensors / adjacency / labels as the
    device-resident gather path."""
    import torch
    from gnnqc.data.store import DeviceStore
    from gnnqc.data.synthetic import make_soilnet_raw
    from gnnqc.data.tfrecord import TFRecordWindows, read_tfrecord, write_window_records
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds}"))
    raw = (make_cml_raw(n_sensors=10, n_minutes=2 * 1440, seed=3) if ds == "cml"
           else make_soilnet_raw(n_boxes=6, n_time=20 * 96, seed=3))
    ws = create_windows_dataset(pc, raw=raw)
    files = write_window_records(ws, str(tmp_path), max_records=64, graph_cfg=pc.graph)
    assert sum(1 for f in files for _ in read_tfrecord(f)) == 64
    tw = TFRecordWindows(str(tmp_path), ds)
    order = np.argsort(ws.window_keys(), kind="stable")[:16]
    b = DeviceStore(ws, tw.normalization, pc.graph).gather(torch.as_tensor(order))
    rb = next(tw.batches(16))
    for i in range(16):
        v = b.node_mask[i] > 0
        n = int(v.sum())
        torch.testing.assert_close(b.x[i][:, v], rb.x[i][:, :n], atol=1e-4, rtol=1e-5)
        assert torch.equal(b.adj[i][v][:, v], rb.adj[i][:n, :n])
        if ds == "soilnet":
            assert torch.equal(b.y[i][v], rb.y[i][:n])
    if ds == "cml":
        assert torch.equal(b.y, rb.y)
        torch.testing.assert_close(b.anom, rb.anom, atol=1e-4, rtol=1e-5)


def test_tfrecord_crc_detects_corruption(tmp_path):
    from gnnqc.data.tfrecord import TFRecordWriter, read_tfrecord
    p = str(tmp_path / "x.tfrec")
    with TFRecordWriter(p) as w:
        w.write(b"hello")
        w.write(b"world" * 10)
    assert list(read_tfrecord(p)) == [b"hello", b"world" * 10]
    raw = bytearray(open(p, "rb").read())
    raw[14] ^= 1
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        list(read_tfrecord(p))


def test_soilnet_spatial_faults_are_locally_plausible():
    """The neighbour-only fault types of the SoilNet generator (missed / phantom wetting) stay
    within the sensor's own range and trip none of the automatic range / spike flags: only the
    neighbours reveal them (the mechanism behind the reference's GCN > baseline)."""
    import numpy as np
    from gnnqc.data.synthetic import make_soilnet_raw
    ds = make_soilnet_raw(n_boxes=8, n_time=60 * 96, seed=4, spatial_fault_frac=1.0)
    m = np.asarray(ds["moisture"].data, np.float64)
    man = np.asarray(ds["moisture_flag_Manual"].data, bool)
    assert man.mean() > 0.02
    rng_flag = np.asarray(ds["moisture_flag_Auto:Range"].data, bool)
    spike = np.asarray(ds["moisture_flag_Auto:Spike"].data, bool)
    assert not (man & rng_flag).any()
    assert (man & spike).sum() <= 0.01 * man.sum()
    site = m[~man & np.isfinite(m)]
    lo, hi = site.min(), site.max()
    seg = m[man & np.isfinite(m)]
    assert seg.min() >= lo - 2 and seg.max() <= hi + 5      # inside the site's normal range
    for i in range(m.shape[0]):                              # and above each sensor's own floor
        ok = ~man[i] & np.isfinite(m[i])
        if man[i].any() and ok.any():
            s_ = m[i, man[i]]
            assert np.nanmin(s_) >= np.nanmin(m[i, ok]) - 2


def test_cml_groups_touch_only_needed_links_and_match_full_processing():
    """prepare_cml_groups computes distances, gap filling and targets for the neighbourhood links
    only; the groups equal a straightforward full-network computation (reference semantics)."""
    from gnnqc.data.graph import compute_distance_matrix, get_neighbors
    from gnnqc.data.preprocessing import prepare_cml_groups
    ds = make_cml_raw(n_sensors=40, n_flagged=3, n_minutes=2 * 1440, seed=11, extent_km=30.0)
    pc = C.normalize_preproc(C.default("preprocessing_cml"))
    groups = prepare_cml_groups(ds, pc)
    dist = compute_distance_matrix(ds, "cml")
    target = create_target(ds)
    X = np.stack([interpolate_gaps(np.where(ds[n].data >= 200, np.nan, ds[n].data), ds.time,
                                   np.timedelta64(5, "m")).astype(np.float32) for n in ("TL_1", "TL_2")], 1)
    flagged = np.nonzero(ds["flagged"].data)[0]
    assert len(groups) == 3 and len(flagged) == 3
    for g, s in zip(groups, flagged):
        nb = get_neighbors(dist, s, pc.graph.max_sample_distance, "cml")
        assert list(g.sensor_ids) == list(ds.sensor_ids[nb])
        np.testing.assert_array_equal(g.distances, dist[np.ix_(nb, nb)])
        np.testing.assert_array_equal(g.features, X[nb])
        np.testing.assert_array_equal(g.target, target[s])
        assert g.sensor_ids[g.anomalous_pos] == ds.sensor_ids[s]
