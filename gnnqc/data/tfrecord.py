"""TFRecord / ``tf.train.SequenceExample`` codec without TensorFlow.

The reference persists every window as a ``SequenceExample`` in ``.tfrec`` files
(``libs/preprocessing_functions.py:176-340`` feature helpers + ``create_example``,
``:343-482`` writer loop). The training path of this framework does not need them
(windows are cut on the device from the resident series, :mod:`gnnqc.data.store`),
but the format is kept so that

* datasets can be exported for / imported from the reference tooling, and
* existing ``.tfrec`` files can be trained on (:class:`TFRecordWindows` -> ``Batch``).

Pieces:

* protobuf wire encoding/decoding of ``Feature`` / ``Features`` / ``FeatureList`` /
  ``FeatureLists`` / ``SequenceExample`` (packed float / int64 lists);
* TFRecord framing: ``uint64 len | masked_crc32c(len) | data | masked_crc32c(data)``
  (CRC32C from the native host library, SSE4.2);
* :func:`window_example` - the reference's ``create_example`` feature layout for a
  window of a :class:`~gnnqc.data.windows.WindowSet` (CML and SoilNet);
* :func:`write_window_records` - the reference file naming (``<sensor>_<day>.tfrec``,
  ``<day>.tfrec``);
* :func:`parse_window_example` / :class:`TFRecordWindows` - decode records back to
  node tensors, normalise like ``parse_*_tfrecord_fn`` and batch them statically.
"""
from __future__ import annotations

import glob
import os
import struct
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

import numpy as np

from ..utils.native import masked_crc32c

# ----------------------------------------------------------------- protobuf wire helpers


def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos: int) -> Tuple[int, int]:
    result = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _ld(field: int, payload: bytes) -> bytes:
    """Length-delimited field."""
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _fields(buf) -> Iterator[Tuple[int, int, object]]:
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _read_varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 2:
            ln, pos = _read_varint(buf, pos)
            yield fn, wt, buf[pos:pos + ln]
            pos += ln
        elif wt == 0:
            v, pos = _read_varint(buf, pos)
            yield fn, wt, v
        elif wt == 5:
            yield fn, wt, buf[pos:pos + 4]
            pos += 4
        elif wt == 1:
            yield fn, wt, buf[pos:pos + 8]
            pos += 8
        else:
            raise ValueError(f"bad wire type {wt}")


# Feature oneof: bytes_list = 1, float_list = 2, int64_list = 3; each *List has `value = 1`.
def feature_float(values) -> bytes:
    a = np.ascontiguousarray(np.asarray(values, dtype="<f4").reshape(-1))
    return _ld(2, _ld(1, a.tobytes()) if a.size else b"")


def feature_int64(values) -> bytes:
    a = np.asarray(values, dtype=np.int64).reshape(-1)
    return _ld(3, _ld(1, b"".join(_varint(int(v)) for v in a)) if a.size else b"")


def feature_bytes(values: Iterable) -> bytes:
    items = [v.encode() if isinstance(v, str) else bytes(v) for v in values]
    return _ld(1, b"".join(_ld(1, v) for v in items))


def _features(d: Dict[str, bytes]) -> bytes:
    # map<string, Feature> feature = 1  -> repeated entry {key = 1, value = 2}
    return b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, v)) for k, v in sorted(d.items()))


def _feature_lists(d: Dict[str, List[bytes]]) -> bytes:
    # map<string, FeatureList> feature_list = 1 ; FeatureList { repeated Feature feature = 1 }
    return b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, b"".join(_ld(1, f) for f in feats)))
                    for k, feats in sorted(d.items()))


def encode_sequence_example(context: Dict[str, bytes], feature_lists: Dict[str, List[bytes]]) -> bytes:
    """``context`` maps name -> encoded Feature, ``feature_lists`` name -> [encoded Feature]."""
    return _ld(1, _features(context)) + _ld(2, _feature_lists(feature_lists))


def decode_feature(buf) -> object:
    """Encoded Feature -> np.float32 array / np.int64 array / list of bytes."""
    for fn, _, payload in _fields(buf):
        if fn == 1:
            return [bytes(v) for f2, _, v in _fields(payload) if f2 == 1]
        if fn == 2:
            parts = []
            for f2, wt, v in _fields(payload):
                if f2 == 1:
                    parts.append(np.frombuffer(v, dtype="<f4") if wt == 2 else np.frombuffer(v, "<f4"))
            return np.concatenate(parts).astype(np.float32) if parts else np.zeros(0, np.float32)
        if fn == 3:
            vals = []
            for f2, wt, v in _fields(payload):
                if f2 != 1:
                    continue
                if wt == 2:
                    pos = 0
                    while pos < len(v):
                        x, pos = _read_varint(v, pos)
                        vals.append(x)
                else:
                    vals.append(v)
            a = np.array(vals, dtype=np.uint64).astype(np.int64) if vals else np.zeros(0, np.int64)
            return a
    return np.zeros(0, np.float32)


def decode_sequence_example(buf) -> Tuple[Dict[str, object], Dict[str, List[object]]]:
    ctx: Dict[str, object] = {}
    lists: Dict[str, List[object]] = {}
    for fn, _, payload in _fields(buf):
        for _f, _, entry in _fields(payload):
            key, val = None, b""
            for f2, _, v in _fields(entry):
                if f2 == 1:
                    key = bytes(v).decode()
                elif f2 == 2:
                    val = v
            if fn == 1:
                ctx[key] = decode_feature(val)
            elif fn == 2:
                lists[key] = [decode_feature(f) for f3, _, f in _fields(val) if f3 == 1]
    return ctx, lists


# ----------------------------------------------------------------- TFRecord framing
class TFRecordWriter:
    def __init__(self, path: str):
        self.f = open(path, "wb")

    def write(self, record: bytes):
        n = struct.pack("<Q", len(record))
        self.f.write(n + struct.pack("<I", masked_crc32c(n)) + record + struct.pack("<I", masked_crc32c(record)))

    def close(self):
        self.f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def read_tfrecord(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    mv = memoryview(data)
    while pos < len(data):
        if pos + 12 > len(data):
            raise ValueError(f"truncated record header in {path}")
        n = struct.unpack_from("<Q", data, pos)[0]
        if verify and struct.unpack_from("<I", data, pos + 8)[0] != masked_crc32c(data[pos:pos + 8]):
            raise ValueError(f"length crc mismatch in {path} at {pos}")
        rec = bytes(mv[pos + 12: pos + 12 + n])
        if verify and struct.unpack_from("<I", data, pos + 12 + n)[0] != masked_crc32c(rec):
            raise ValueError(f"data crc mismatch in {path} at {pos}")
        yield rec
        pos += 16 + n


# ----------------------------------------------------------------- window <-> example
_CML_NAMES = {"TL_1": "TRSL1", "TL_2": "TRSL2"}
_STATS = ("mean", "median", "std", "min", "max")
_ROLL = ("mean", "std", "median")


def _fl_rows(mat) -> List[bytes]:
    """FeatureList of float Features, one per row (``float_featurelist_from_list``)."""
    return [feature_float(r) for r in np.asarray(mat, np.float32)]


def _fl_scalars_f(vals) -> List[bytes]:
    return [feature_float([v]) for v in np.asarray(vals, np.float32).reshape(-1)]


def _fl_scalars_i(vals) -> List[bytes]:
    return [feature_int64([v]) for v in np.asarray(vals, np.int64).reshape(-1)]


def _stat(g, key, nodes, center=None):
    v = g.stats.get(key)
    if v is None:
        return np.full(len(nodes), np.nan, np.float32)
    v = np.asarray(v)
    if v.ndim == 2:            # rolling [N, T]
        return v[nodes, center].astype(np.float32)
    return v[nodes].astype(np.float32)


def window_example(ws, gi: int, li: int, graph_cfg=None) -> bytes:
    """Serialise window ``li`` of group ``gi`` like ``create_example`` (``:220-340``)."""
    from .graph import build_adjacency
    g = ws.groups[gi]
    ix = ws.indices[gi]
    T = ws.seq_len
    tb = int(round(ws.timestep_before / ws.freq))
    c = int(ix.center[li])
    t0, t1 = c - tb, c - tb + T
    nodes = np.nonzero(ix.node_valid[li])[0]
    if g.per_sensor and g.anomalous_pos not in nodes:
        nodes = np.sort(np.append(nodes, g.anomalous_pos))
    feats = g.features[nodes][:, :, t0:t1]                    # [n, C, T]
    dist = g.distances[np.ix_(nodes, nodes)]
    dep = g.depths[np.ix_(nodes, nodes)] if g.depths is not None else None
    if graph_cfg is None:
        graph_cfg = {"adjacency": "radius", "max_sample_distance": 6.0 if g.ds_type == "cml" else 30.0,
                     "max_neighbour_depth": 0.1}
    adj = build_adjacency(graph_cfg, dist, dep, g.ds_type) > 0
    src, dst = np.nonzero(adj)
    dates = np.datetime_as_string(g.time[t0:t1].astype("datetime64[s]"), unit="s")
    ctx: Dict[str, bytes] = {"node_numb": feature_int64([len(nodes)]), "link_numb": feature_int64([len(src)]),
                             "dates": feature_bytes(dates)}
    lists: Dict[str, List[bytes]] = {"nodes": _fl_scalars_i(src), "neighbours": _fl_scalars_i(dst),
                                     "distances": _fl_scalars_f(dist[adj])}
    if g.ds_type == "cml":
        ap = int(np.nonzero(nodes == g.anomalous_pos)[0][0])
        ctx["anomaly_ID"] = feature_bytes([str(g.group_id)])
        ctx["anomaly_flag"] = feature_int64([int(ix.labels[li])])
        ctx["CML_ids"] = feature_bytes([str(s) for s in g.sensor_ids[nodes]])
        for ci, name in enumerate(g.feature_names):
            rn = _CML_NAMES.get(name, name)
            ctx[f"{rn}_anomalous_cml"] = feature_float(feats[ap, ci])
            for s in _STATS:
                ctx[f"{rn}_{s}"] = feature_float(_stat(g, f"{name}_{s}", nodes))
            for s in _ROLL:
                ctx[f"{rn}_rolling_{s}"] = feature_float(_stat(g, f"{name}_rolling_{s}", nodes, c))
            lists[rn] = _fl_rows(feats[:, ci].T)                 # T entries of [n]
        for key in ("site_a_latitude", "site_b_latitude", "site_a_longitude", "site_b_longitude"):
            if key in g.coords:
                name = "cml_" + key.replace("site_", "").replace("latitude", "lat").replace("longitude", "lon")
                name = {"cml_a_lat": "cml_lat_a", "cml_b_lat": "cml_lat_b", "cml_a_lon": "cml_lon_a",
                        "cml_b_lon": "cml_lon_b"}[name]
                row = feature_float(np.asarray(g.coords[key], np.float32)[nodes])
                lists[name] = [row] * T                           # ``coordinates_featurelist``
    elif g.per_sensor:
        # XAI-generation SoilNet neighbourhood (xai/libs/preprocessing_functions.py:218-240): the
        # selected sensor's id, series and window label as context, every node's series as lists
        ap = int(np.nonzero(nodes == g.anomalous_pos)[0][0])
        sid = np.asarray(g.sensor_ids)
        ctx["anomaly_ID"] = feature_int64([int(sid[g.anomalous_pos])])
        ctx["sensor_ids"] = feature_int64(sid[nodes].astype(np.int64))
        ctx["anomaly_flag"] = feature_int64([int(ix.labels[li])])
        for ci, name in enumerate(g.feature_names):
            ctx[f"{name}_anomalous_sensor"] = feature_float(feats[ap, ci])
            for s in _STATS:
                ctx[f"{name}_{s}"] = feature_float(_stat(g, f"{name}_{s}", nodes))
            for s in _ROLL:
                ctx[f"{name}_rolling_{s}"] = feature_float(_stat(g, f"{name}_rolling_{s}", nodes, c))
            lists[name] = _fl_rows(feats[:, ci].T)
        lists["depths"] = _fl_scalars_f(dep[adj] if dep is not None else np.zeros(len(src)))
        if g.lat is not None:
            lists["sensor_lat"] = [feature_float(np.asarray(g.lat, np.float32)[nodes])] * T
            lists["sensor_lon"] = [feature_float(np.asarray(g.lon, np.float32)[nodes])] * T
    else:
        for ci, name in enumerate(g.feature_names):
            for s in _STATS:
                ctx[f"{name}_{s}"] = feature_float(_stat(g, f"{name}_{s}", nodes))
            for s in _ROLL:
                ctx[f"{name}_rolling_{s}"] = feature_float(_stat(g, f"{name}_rolling_{s}", nodes, c))
            lists[name] = _fl_rows(feats[:, ci].T)
        lab = ix.labels[li][nodes]
        lists["sensor_ids"] = _fl_scalars_i(np.asarray(g.sensor_ids)[nodes].astype(np.int64))
        lists["anomaly_flag"] = _fl_scalars_i(lab)
        lists["depths"] = _fl_scalars_f(dep[adj] if dep is not None else np.zeros(len(src)))
        if g.lat is not None:
            lists["sensor_lat"] = [feature_float(np.asarray(g.lat, np.float32)[nodes])] * T
            lists["sensor_lon"] = [feature_float(np.asarray(g.lon, np.float32)[nodes])] * T
    return encode_sequence_example(ctx, lists)


def write_window_records(ws, out_dir: str, normalization: Optional[str] = None, max_records: Optional[int] = None,
                         graph_cfg=None) -> List[str]:
    """One file per (flagged sensor, day) for CML / per day for SoilNet (``:392-393,452``)."""
    os.makedirs(out_dir, exist_ok=True)
    keys = ws.window_keys()
    wg, wl = ws.flat()
    order = np.argsort(keys, kind="stable")
    written: List[str] = []
    writer, cur = None, None
    for n, i in enumerate(order):
        if max_records is not None and n >= max_records:
            break
        if keys[i] != cur:
            if writer:
                writer.close()
            cur = keys[i]
            path = os.path.join(out_dir, f"{cur}.tfrec")
            writer = TFRecordWriter(path)
            written.append(path)
        writer.write(window_example(ws, int(wg[i]), int(wl[i]), graph_cfg))
    if writer:
        writer.close()
    return written


# ----------------------------------------------------------------- parsing back
def parse_window_example(buf: bytes, ds_type: str) -> Dict[str, object]:
    """Record -> dict(features [n, C, T] float32, anom_pos, src, dst, label(s), stats, ids, dates)."""
    ctx, lists = decode_sequence_example(buf)
    out: Dict[str, object] = {"dates": [d.decode() for d in ctx.get("dates", [])]}
    if ds_type == "cml":
        chans = ["TRSL1", "TRSL2"]
        feats = np.stack([np.stack(lists[c], 1) for c in chans], 1)          # [n, C, T]
        ids = [s.decode() for s in ctx["CML_ids"]]
        anom_id = ctx["anomaly_ID"][0].decode()
        out.update(features=feats, ids=ids, anom_pos=ids.index(anom_id) if anom_id in ids else 0,
                   label=int(ctx["anomaly_flag"][0]))
    elif "anomaly_ID" in ctx:          # XAI SoilNet per-sensor record (parse_soilnet_tfrecord_fn :419-509)
        chans = ["moisture", "temp", "battv"]
        feats = np.stack([np.stack(lists[c], 1) for c in chans], 1)
        ids = [int(v) for v in ctx["sensor_ids"]]
        aid = int(ctx["anomaly_ID"][0])
        out.update(features=feats, ids=ids, anom_pos=ids.index(aid) if aid in ids else 0,
                   label=int(ctx["anomaly_flag"][0]),
                   anom_series=np.stack([np.asarray(ctx[f"{c}_anomalous_sensor"], np.float32) for c in chans], 0))
    else:
        chans = ["moisture", "temp", "battv"]
        feats = np.stack([np.stack(lists[c], 1) for c in chans], 1)
        out.update(features=feats, ids=[int(v[0]) for v in lists["sensor_ids"]], anom_pos=-1,
                   labels=np.array([int(v[0]) for v in lists["anomaly_flag"]], np.float32))
    out["src"] = np.array([int(v[0]) for v in lists.get("nodes", [])], np.int64)
    out["dst"] = np.array([int(v[0]) for v in lists.get("neighbours", [])], np.int64)
    out["stats"] = {f"{c}_{s}": ctx[f"{c}_{s}"] for c in chans
                    for s in _STATS + tuple(f"rolling_{r}" for r in _ROLL) if f"{c}_{s}" in ctx}
    out["channels"] = chans
    return out


def _shift_scale(rec, normalization: str, ds_type: str):
    st, chans = rec["stats"], rec["channels"]
    n = rec["features"].shape[0]
    C = len(chans)

    def get(s):
        return np.stack([st[f"{c}_{s}"] for c in chans], -1).astype(np.float32)   # [n, C]

    if normalization == "scale_range":
        from .store import _SOIL_SCALE_RANGE
        sh = np.array([_SOIL_SCALE_RANGE[c][0] for c in chans], np.float32)
        sc = np.array([_SOIL_SCALE_RANGE[c][1] for c in chans], np.float32)
        return np.broadcast_to(sh, (n, C)), np.broadcast_to(sc, (n, C))
    if normalization == "rolling_median":
        return get("rolling_median"), np.ones((n, C), np.float32)
    if normalization == "rolling_median_fractional":
        m = get("rolling_median")
        return m, 1.0 / m
    if normalization == "rolling_mean":
        return get("rolling_mean"), 1.0 / get("rolling_std")
    if normalization == "standarization":
        return get("mean"), 1.0 / get("std")
    if normalization == "scale":
        mn = get("min")
        return mn, 1.0 / (get("max") - mn)
    if normalization == "median":
        m = get("median")
        return m, (1.0 / m if ds_type == "cml" else np.ones_like(m))
    return np.zeros((n, C), np.float32), np.ones((n, C), np.float32)


class TFRecordWindows:
    """Windows read from ``.tfrec`` files, batched into static-shape :class:`Batch` es.

    ``parse_*_tfrecord_fn`` + ``prepare_batch_*`` (``:566-933``) with the dense
    per-sample adjacency of :mod:`gnnqc.data.store` instead of a block-diagonal
    sparse matrix. Records are decoded once on the host and kept as padded arrays.
    """

    def __init__(self, files, ds_type: str, normalization: Optional[str] = None, max_nodes: Optional[int] = None):
        if isinstance(files, str):
            files = sorted(glob.glob(os.path.join(files, "*.tfrec"))) if os.path.isdir(files) else [files]
        self.ds_type = ds_type
        self.normalization = normalization or ("rolling_median" if ds_type == "cml" else "scale_range")
        recs = [parse_window_example(r, ds_type) for f in files for r in read_tfrecord(f)]
        if not recs:
            raise ValueError("no records")
        N = max_nodes or max(r["features"].shape[0] for r in recs)
        C, T = recs[0]["features"].shape[1:]
        W = len(recs)
        # one label per window (CML, XAI SoilNet) vs one per node (network-wide SoilNet)
        self.per_sensor = ds_type == "cml" or "label" in recs[0]
        per = self.per_sensor
        self.x = np.zeros((W, T, N, C), np.float32)
        self.adj = np.zeros((W, N, N), np.float32)
        self.mask = np.zeros((W, N), np.float32)
        self.anom_pos = np.full(W, -1, np.int64)
        self.y = np.zeros((W,) if per else (W, N), np.float32)
        self.y_mask = np.ones((W,), np.float32) if per else np.zeros((W, N), np.float32)
        for i, r in enumerate(recs):
            f = r["features"]
            n = f.shape[0]
            sh, sc = _shift_scale(r, self.normalization, ds_type)
            xi = (f.transpose(2, 0, 1) - sh[None]) * sc[None]
            self.x[i, :, :n] = np.nan_to_num(xi, nan=0.0, posinf=0.0, neginf=0.0)
            self.adj[i, r["src"], r["dst"]] = 1.0
            self.mask[i, :n] = 1.0
            self.anom_pos[i] = r["anom_pos"]
            if per:
                self.y[i] = r["label"]
            else:
                self.y[i, :n] = r["labels"]
                self.y_mask[i, :n] = 1.0
        self.n_windows, self.seq_len, self.n_nodes = W, T, N

    def batches(self, batch_size: int, device="cpu", shuffle: bool = False, seed: int = 0):
        import torch
        from .store import Batch
        order = np.random.default_rng(seed).permutation(self.n_windows) if shuffle else np.arange(self.n_windows)
        for s in range(0, self.n_windows, batch_size):
            idx = order[s:s + batch_size]
            pad = batch_size - len(idx)
            take = np.concatenate([idx, np.zeros(pad, np.int64)]) if pad else idx
            ok = np.concatenate([np.ones(len(idx)), np.zeros(pad)]).astype(np.float32)

            def t(a):
                return torch.from_numpy(np.ascontiguousarray(a)).to(device)
            x = self.x[take] * ok[:, None, None, None]
            mask = self.mask[take] * ok[:, None]
            anom = None
            if self.per_sensor:
                ap = np.clip(self.anom_pos[take], 0, None)
                anom = x[np.arange(len(take)), :, ap]
                y, ym = self.y[take] * ok, ok
            else:
                y, ym = self.y[take] * mask, self.y_mask[take] * ok[:, None]
            wid = np.concatenate([idx, np.full(pad, -1)]).astype(np.int64)
            yield Batch(x=t(x), adj=t(self.adj[take] * mask[:, :, None] * mask[:, None, :]), node_mask=t(mask),
                        anom=t(anom) if anom is not None else None, anom_pos=t(self.anom_pos[take]), y=t(y),
                        y_mask=t(ym), wid=t(wid), per_sensor=self.per_sensor)


__all__ = ["TFRecordWriter", "read_tfrecord", "encode_sequence_example", "decode_sequence_example",
           "feature_float", "feature_int64", "feature_bytes", "window_example", "write_window_records",
           "parse_window_example", "TFRecordWindows"]
