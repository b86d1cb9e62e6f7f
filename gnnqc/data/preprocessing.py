"""Reference-named preprocessing entry points (``libs/preprocessing_functions.py``).

Pipeline, MI355X-first:

    raw SensorData --prepare_groups--> [SensorGroup] --create_windows_dataset--> WindowSet
        --load_dataset / load_dataset_CV--> window-id splits
        --create_batched_dataset--> DeviceLoader (HBM-resident, GPU gather, static shapes)

``create_sensors_ncfiles`` / ``create_tfrecords_dataset`` keep the reference's on-disk
artefacts available: per-neighbourhood NetCDF files, a compact ``.npz`` window
index per (tb, ta), and (optionally) genuine TFRecord ``SequenceExample`` files via
:mod:`gnnqc.data.tfrecord`.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional

import numpy as np

from ..config import Config, freq_minutes, normalize_preproc
from .graph import compute_depth_matrix, compute_distance_matrix, get_neighbors, sensor_positions
from .interp import interpolate_gaps
from .raw_io import SensorData, read_netcdf, write_netcdf
from .splits import chronological_split, day_numbers, kfold_split, monthly_random_split
from .stats import calculate_statistics
from .targets import CML_FLAG_VARS, create_target
from .windows import SensorGroup, WindowSet, build_window_index

CML_FEATURES = ["TL_1", "TL_2"]
SOIL_FEATURES = ["moisture", "temp", "battv"]

# which statistics each normalisation needs (the reference computes all of them)
_NEEDS = {
    "rolling_median": ("median",), "rolling_median_fractional": ("median",),
    "rolling_mean": ("mean", "std"), "standarization": (), "scale": (), "median": (),
    "scale_range": (), "none": (),
}


def _interp(values, time, max_gap):
    return interpolate_gaps(values, time, max_gap).astype(np.float32)


def _cml_flagged_rows(lat, lon, flagged, unit: str) -> np.ndarray:
    """Rows ``flagged`` of the CML geodesic distance matrix ([F, S]), each pair evaluated in the
    (lower index, higher index) orientation :func:`geodesic_distance_matrix` uses, so the values are
    bit-identical to the full matrix's without computing its S^2 / 2 pairs."""
    from .geo import vincenty_inverse
    S = lat.shape[0]
    j = np.arange(S)
    rows = np.zeros((len(flagged), S), dtype=np.float64)
    scale = {"m": 1.0, "km": 1e-3}[unit]
    for r, s in enumerate(flagged):
        a, b = np.minimum(s, j), np.maximum(s, j)
        off = a != b
        rows[r, off] = vincenty_inverse(lat[a[off]], lon[a[off]], lat[b[off]], lon[b[off]])
    return rows * scale


def prepare_cml_groups(ds: SensorData, cfg) -> List[SensorGroup]:
    """CML part of ``create_sensors_ncfiles`` (``:79-120``) in memory.

    Only the links that end up in some neighbourhood are touched: distances are computed as the
    flagged links' rows plus the matrix of the needed links, and gap filling, masking and the
    expert-vote target run on those rows only. The result is identical to processing every link
    (the reference writes one NetCDF per flagged link), but the full-size network (3,904 links x
    133,920 minutes, 20 flagged; ``notebooks/prepare_raw_cml.ipynb``) needs a few hundred MB
    instead of tens of GB of host temporaries."""
    from .geo import geodesic_distance_matrix
    cfg = normalize_preproc(cfg)
    time = ds.time
    unit = cfg.get("distance_unit", "km")
    lat, lon = sensor_positions(ds, "cml")
    flagged = np.nonzero(np.asarray(ds["flagged"].data, bool))[0]
    max_dist = cfg.graph.max_sample_distance
    rows = _cml_flagged_rows(lat, lon, flagged, unit)
    nbs = [get_neighbors(rows, r, max_dist, "cml") for r in range(len(flagged))]
    needed = np.unique(np.concatenate(nbs + [flagged])) if len(flagged) else np.zeros(0, np.int64)
    pos = {int(s): i for i, s in enumerate(needed)}
    dist = geodesic_distance_matrix(lat[needed], lon[needed], unit=unit)      # [n_needed, n_needed]
    feats = []
    for name in CML_FEATURES:
        v = np.array(np.asarray(ds[name].data)[needed], dtype=np.float32)
        v[v >= 200] = np.nan          # "High (over 200 dB) values replaced with NaN"
        if cfg.interpolate:
            v = _interp(v, time, np.timedelta64(5, "m"))
        feats.append(v)
    X = np.stack(feats, axis=1)       # [n_needed, C, T]
    target = create_target(ds, CML_FLAG_VARS, 3, "cml", sensors=flagged)      # [F, T]
    groups = []
    ids = ds.sensor_ids
    for r, s in enumerate(flagged):
        nb = nbs[r]
        li = np.array([pos[int(k)] for k in nb], dtype=np.int64)
        coords = {k: np.asarray(ds[k].data)[nb] for k in ("site_a_latitude", "site_a_longitude",
                                                          "site_b_latitude", "site_b_longitude", "length")
                  if k in ds}
        groups.append(SensorGroup(
            group_id=str(ids[s]), ds_type="cml", sensor_ids=ids[nb],
            anomalous_pos=int(np.nonzero(nb == s)[0][0]), feature_names=list(CML_FEATURES),
            features=np.ascontiguousarray(X[li]), time=time, target=target[r].astype(bool),
            distances=dist[np.ix_(li, li)], lat=lat[nb], lon=lon[nb], coords=coords))
    return groups


def prepare_soilnet_groups(ds: SensorData, cfg) -> List[SensorGroup]:
    """SoilNet part of ``create_tfrecords_dataset`` (``:414-447``): one network-wide graph."""
    cfg = normalize_preproc(cfg)
    lat_all = np.asarray(ds["latitude"].data, np.float64)
    lon_all = np.asarray(ds["longitude"].data, np.float64)
    keep = ~(np.isnan(lat_all) | np.isnan(lon_all))
    ds = ds.isel(sensor_id=np.nonzero(keep)[0])
    time = ds.time
    feats = []
    for name in SOIL_FEATURES:
        v = np.array(ds[name].data, dtype=np.float32)
        if cfg.interpolate:
            v = _interp(v, time, np.timedelta64(60, "m"))
        feats.append(v)
    X = np.stack(feats, axis=1)
    target = create_target(ds, ds_type="soilnet", flags_type=cfg.get("flags_type", "manual"))
    dist = compute_distance_matrix(ds, "soilnet", unit=cfg.get("distance_unit", "m"))
    depths = compute_depth_matrix(ds)
    lat, lon = sensor_positions(ds, "soilnet")
    coords = {k: np.asarray(ds[k].data) for k in ("box_id", "level_id", "depth") if k in ds}
    return [SensorGroup(group_id="soilnet", ds_type="soilnet", sensor_ids=ds.sensor_ids, anomalous_pos=-1,
                        feature_names=list(SOIL_FEATURES), features=X, time=time, target=target,
                        distances=dist, depths=depths, lat=lat, lon=lon, coords=coords)]


def select_sensors(ds: SensorData, seed: int = 44) -> np.ndarray:
    """One sensor per box: the one with the most moisture observations, ties broken at random
    (``xai/libs/preprocessing_functions.py:1019-1025``; the reference seeds ``random`` with
    ``random_state`` in ``create_sensors_ncfiles`` ``:952``). Returns sensor positions."""
    import random
    rnd = random.Random(seed)
    box = np.asarray(ds["box_id"].data)
    n_obs = (~np.isnan(np.asarray(ds["moisture"].data, np.float64))).sum(axis=1)
    out = []
    for b in np.unique(box):             # xarray groupby order: sorted box ids
        pos = np.nonzero(box == b)[0]
        best = pos[n_obs[pos] == n_obs[pos].max()]
        out.append(int(rnd.choice(list(best))))
    return np.asarray(out, np.int64)


def prepare_soilnet_sensor_groups(ds: SensorData, cfg) -> List[SensorGroup]:
    """SoilNet of the XAI generation (``create_sensors_ncfiles`` ``xai/libs/preprocessing_functions.py:
    951-1016``): for one selected sensor per box, its depth-aware neighbourhood (same-depth sensors
    within ``max_sample_distance`` and the co-located sensors within ``graph.max_depth`` of depth,
    ``get_neighbors``), with that sensor's target series and the neighbourhood's distances and depth
    differences. Group ids are ``<box>_<sensor>`` like the reference's file names."""
    cfg = normalize_preproc(cfg)
    lat_all = np.asarray(ds["latitude"].data, np.float64)
    lon_all = np.asarray(ds["longitude"].data, np.float64)
    keep = ~(np.isnan(lat_all) | np.isnan(lon_all))
    ds = ds.isel(sensor_id=np.nonzero(keep)[0])
    time = ds.time
    flagged = select_sensors(ds, int(cfg.get("random_state", 44)))
    feats = []
    for name in SOIL_FEATURES:
        v = np.array(ds[name].data, dtype=np.float32)
        if cfg.interpolate:
            v = _interp(v, time, np.timedelta64(60, "m"))
        feats.append(v)
    X = np.stack(feats, axis=1)
    target = create_target(ds, ds_type="soilnet", flags_type=cfg.get("flags_type", "manual"))
    dist = compute_distance_matrix(ds, "soilnet", unit=cfg.get("distance_unit", "m"))
    depths = compute_depth_matrix(ds)
    lat, lon = sensor_positions(ds, "soilnet")
    ids = ds.sensor_ids
    box = np.asarray(ds["box_id"].data)
    max_dist = cfg.graph.max_sample_distance
    max_depth = cfg.graph.get("max_depth", cfg.graph.max_neighbour_depth)
    groups = []
    for s in flagged:
        nb = get_neighbors(dist, s, max_dist, "soilnet", depths=depths, max_depth=max_depth)
        coords = {k: np.asarray(ds[k].data)[nb] for k in ("box_id", "level_id", "depth") if k in ds}
        groups.append(SensorGroup(
            group_id=f"{box[s]}_{ids[s]}", ds_type="soilnet", sensor_ids=ids[nb],
            anomalous_pos=int(np.nonzero(nb == s)[0][0]), feature_names=list(SOIL_FEATURES),
            features=np.ascontiguousarray(X[nb]), time=time, target=target[s].astype(np.float32),
            distances=dist[np.ix_(nb, nb)], depths=depths[np.ix_(nb, nb)], lat=lat[nb], lon=lon[nb],
            coords=coords))
    return groups


def prepare_groups(ds: SensorData, cfg) -> List[SensorGroup]:
    if cfg["ds_type"] == "cml":
        return prepare_cml_groups(ds, cfg)
    if cfg.get("per_sensor", False):
        return prepare_soilnet_sensor_groups(ds, cfg)
    return prepare_soilnet_groups(ds, cfg)


def add_statistics(groups: List[SensorGroup], cfg, normalization: Optional[str] = None):
    """``calculate_statistics`` (``:123-173``) for what the normalisation needs."""
    cfg = normalize_preproc(cfg)
    norm = normalization or cfg.get("normalization") or ("rolling_median" if cfg.ds_type == "cml" else "scale_range")
    needs = _NEEDS.get(norm, ("mean", "std", "median"))
    for g in groups:
        feats = {n: g.features[:, i, :] for i, n in enumerate(g.feature_names)}
        g.stats = calculate_statistics(feats, int(cfg.window_length), which_rolling=needs)
    return groups


# ----------------------------------------------------------------- NetCDF files
def group_to_sensordata(g: SensorGroup) -> SensorData:
    ds = SensorData(attrs={"anomalous_sensor_id": g.group_id, "ds_type": g.ds_type})
    ds.set_coord("sensor_id", "sensor_id", g.sensor_ids)
    ds.set_coord("time", "time", g.time)
    for k, v in g.coords.items():
        ds.set_coord(k, "sensor_id", v)
    if g.lat is not None:
        ds.set_coord("lat", "sensor_id", g.lat)
        ds.set_coord("lon", "sensor_id", g.lon)
    for i, n in enumerate(g.feature_names):
        ds[n] = (("sensor_id", "time"), g.features[:, i, :])
    if g.per_sensor:
        ds["target"] = ("time", g.target.astype(bool) if g.ds_type == "cml" else g.target.astype(np.float32))
        flagged = np.zeros(g.n_nodes, bool)
        flagged[g.anomalous_pos] = True
        ds["flagged"] = ("sensor_id", flagged)
    else:
        ds["target"] = (("sensor_id", "time"), g.target.astype(np.float32))
    if g.depths is not None:
        ds["depths"] = (("sensor_id", "sensor_id1"), g.depths)
    ds["distances"] = (("sensor_id", "sensor_id1"), g.distances)
    return ds


def sensordata_to_group(ds: SensorData) -> SensorGroup:
    ds_type = ds.attrs.get("ds_type", "cml")
    names = CML_FEATURES if ds_type == "cml" else SOIL_FEATURES
    X = np.stack([np.asarray(ds[n].data, np.float32) for n in names], axis=1)
    coords = {k: v.data for k, v in ds.coords.items() if k not in ("sensor_id", "time", "lat", "lon")}
    if "flagged" in ds:                  # a flagged-sensor neighbourhood (CML, XAI SoilNet)
        flagged = np.asarray(ds["flagged"].data, bool)
        anom = int(np.nonzero(flagged)[0][0])
        target = np.asarray(ds["target"].data, bool if ds_type == "cml" else np.float32)
    else:
        anom = -1
        target = np.asarray(ds["target"].data, np.float32)
    depths = np.asarray(ds["depths"].data) if "depths" in ds else None
    return SensorGroup(group_id=str(ds.attrs.get("anomalous_sensor_id", "group")), ds_type=ds_type,
                       sensor_ids=ds.sensor_ids, anomalous_pos=anom, feature_names=list(names), features=X,
                       time=ds.time, target=target, distances=np.asarray(ds["distances"].data), depths=depths,
                       lat=ds["lat"].data if "lat" in ds else None, lon=ds["lon"].data if "lon" in ds else None,
                       coords=coords)


def create_sensors_ncfiles(ds: SensorData, preproc_config) -> List[str]:
    """Write one NetCDF per neighbourhood into ``ncfiles_dir`` (``:79-120``; XAI SoilNet:
    ``<box>_<sensor>.nc`` per selected sensor, ``xai/libs/preprocessing_functions.py:1005-1016``)."""
    cfg = normalize_preproc(preproc_config)
    out_dir = cfg.ncfiles_dir
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for g in prepare_groups(ds, cfg):
        p = os.path.join(out_dir, f"{g.group_id}.nc")
        write_netcdf(group_to_sensordata(g), p)
        paths.append(p)
    return paths


def load_sensor_groups(preproc_config) -> List[SensorGroup]:
    cfg = normalize_preproc(preproc_config)
    files = sorted(glob.glob(os.path.join(cfg.ncfiles_dir, "*.nc")))
    return [sensordata_to_group(read_netcdf(f)) for f in files]


# ----------------------------------------------------------------- windows
def create_windows_dataset(preproc_config, groups: Optional[List[SensorGroup]] = None,
                           raw: Optional[SensorData] = None, normalization: Optional[str] = None) -> WindowSet:
    """Compute statistics and the window index of every group (the work of
    ``create_tfrecords_dataset`` ``:343-482`` without serialising records)."""
    cfg = normalize_preproc(preproc_config)
    if groups is None:
        if raw is not None:
            groups = prepare_groups(raw, cfg)
        elif cfg.get("per_sensor", cfg.ds_type == "cml"):
            groups = load_sensor_groups(cfg)
        else:
            groups = prepare_groups(read_netcdf(cfg.raw_dataset_path), cfg)
    add_statistics(groups, cfg, normalization)
    f = freq_minutes(cfg.ds_type)
    min_date = cfg.get("min_date")
    max_date = cfg.get("max_date")
    indices = [build_window_index(g, i, cfg.timestep_before, cfg.timestep_after, f, min_date, max_date)
               for i, g in enumerate(groups)]
    return WindowSet(groups=groups, indices=indices, ds_type=cfg.ds_type,
                     timestep_before=int(cfg.timestep_before), timestep_after=int(cfg.timestep_after), freq=f)


def create_tfrecords_dataset(preproc_config, windows: Optional[WindowSet] = None, write_records: bool = False,
                             max_records: Optional[int] = None) -> str:
    """Persist the window index (and optionally real TFRecord files).

    Output dir: ``<tfrecords_dataset_dir>/<tb>_<ta>`` like ``:355-360``. The index is
    ``windows.npz``; with ``write_records`` every window is also written as a
    ``SequenceExample`` into ``<sensor>_<day>.tfrec`` / ``<day>.tfrec`` files.
    """
    cfg = normalize_preproc(preproc_config)
    if windows is None:
        windows = create_windows_dataset(cfg)
    out = os.path.join(cfg.tfrecords_dataset_dir, f"{cfg.timestep_before}_{cfg.timestep_after}")
    os.makedirs(out, exist_ok=True)
    arrays = {}
    for i, ix in enumerate(windows.indices):
        arrays[f"g{i}_center"] = ix.center
        arrays[f"g{i}_valid"] = ix.node_valid
        arrays[f"g{i}_labels"] = ix.labels
        if ix.label_valid is not None:
            arrays[f"g{i}_label_valid"] = ix.label_valid
    arrays["group_ids"] = np.array([g.group_id for g in windows.groups])
    np.savez_compressed(os.path.join(out, "windows.npz"), **arrays)
    if write_records:
        from .tfrecord import write_window_records
        write_window_records(windows, out, normalization=cfg.get("normalization"), max_records=max_records,
                             graph_cfg=cfg.graph)
    return out


# ----------------------------------------------------------------- splits
def load_dataset(preproc_config, windows: WindowSet):
    """(train_ids, val_ids, test_ids) window-id arrays (``:485-563``)."""
    cfg = normalize_preproc(preproc_config)
    days = windows.window_days()
    if windows.ds_type == "cml":            # (SoilNet of both generations: monthly random split)
        tr, va, te = chronological_split(days, cfg.train_fraction, cfg.val_fraction,
                                         cfg.timestep_before, cfg.timestep_after)
    else:
        tr, va, te = monthly_random_split(days, cfg.train_fraction, cfg.val_fraction,
                                          cfg.timestep_before, cfg.timestep_after, seed=cfg.random_state)
    ids = np.arange(windows.n_windows)
    return ids[tr], ids[va], ids[te]


def load_dataset_CV(preproc_config, windows: WindowSet, test_split: int = 0, gap_days: Optional[int] = None):
    """(train_ids, test_ids, cfg) for fold ``test_split`` (``xai/...:804-836``).

    File numbers are day numbers (one record file per group and day).
    """
    cfg = normalize_preproc(preproc_config)
    cfg.split = test_split
    k = int(cfg.dataset.get("split_numb", cfg.get("split_numb", 5)))
    fn = day_numbers(windows.window_days())
    gap = int(cfg.get("cv_gap_days", 0) if gap_days is None else gap_days)
    tr, te = kfold_split(fn, k, test_split, gap=gap)
    ids = np.arange(windows.n_windows)
    return ids[tr], ids[te], cfg


def create_batched_dataset(window_ids, preproc_config, store, shuffle: bool = True, baseline: bool = False,
                           rank: int = 0, world_size: int = 1, batch_size: Optional[int] = None):
    """DeviceLoader over ``window_ids`` + config + wrapping functions (``:936-965``).

    Like the reference, ``preproc_config.normalization`` is set from the loader's
    normalisation (``:941,964``).
    """
    from .store import DeviceLoader
    cfg = preproc_config
    loader = DeviceLoader(store, window_ids, batch_size or cfg["batch_size"], shuffle=shuffle,
                          seed=cfg.get("random_state", 44), rank=rank, world_size=world_size)
    cfg["normalization"] = store.normalization

    def wrap_model(batch):
        return batch.model_inputs(store.ds_type, baseline), batch.y

    def wrap_plot(batch):
        return (batch.model_inputs(store.ds_type, baseline), batch.wid), batch.y

    return loader, cfg, [wrap_model, wrap_plot]


__all__ = [
    "prepare_cml_groups", "prepare_soilnet_groups", "prepare_soilnet_sensor_groups", "select_sensors",
    "prepare_groups", "add_statistics",
    "create_sensors_ncfiles", "load_sensor_groups", "create_windows_dataset", "create_tfrecords_dataset",
    "load_dataset", "load_dataset_CV", "create_batched_dataset", "group_to_sensordata", "sensordata_to_group",
]
