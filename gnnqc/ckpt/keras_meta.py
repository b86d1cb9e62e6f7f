"""``keras_metadata.pb`` of the Keras SavedModel layout.

The reference registers its custom layers (``Custom>TimeLayer``; ``libs/create_model.py:7,43``)
so that ``tf.keras.models.load_model(path, compile=False)`` can rebuild the model from
the per-layer JSON stored in ``keras_metadata.pb``. This module writes that file for
our models and reads it back:

* protobuf ``SavedMetadata { repeated SavedObject nodes = 1; }`` with
  ``SavedObject { int32 node_id = 2; string node_path = 3; string identifier = 4;
  string metadata = 5 (JSON); VersionDef version = 6; }`` (encoded by hand: no
  protobuf runtime needed);
* one node per Keras object the reference saves: the model (``_tf_keras_model``,
  with ``training_config`` / optimizer config), every layer (``_tf_keras_layer`` /
  ``_tf_keras_rnn_layer``), the LSTM cells, and the 9 compile metrics
  (``_tf_keras_metric``);
* node paths follow the reference's attribute names (``root.gcn_layer``,
  ``root.time_layer.time_layers.0.cell``, baseline ``root.time1`` ...), class names
  and configs follow Keras 2.11 serialisation, build shapes come from the window
  configuration (T = (tb + ta) / freq + 1, then / pool per stack).

``node_id`` values are assigned in traversal order (the reference's come from its
TrackableObjectGraph, which is not emitted): consumers key on ``node_path``.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

KERAS_VERSION = "2.11.0"
META_FILE = "keras_metadata.pb"
_VERSION_DEF = b"\x08\x02\x10\x01"    # VersionDef{producer: 2, min_consumer: 1}


# ------------------------------------------------------------------ protobuf helpers
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, data: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(data)) + data


def _read_varint(b: bytes, i: int):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield num, v


def encode_metadata(nodes: List[dict]) -> bytes:
    out = bytearray()
    for n in nodes:
        obj = bytearray()
        if n.get("node_id", 0):
            obj += _varint((2 << 3) | 0) + _varint(int(n["node_id"]))
        obj += _field_bytes(3, n["node_path"].encode())
        obj += _field_bytes(4, n["identifier"].encode())
        obj += _field_bytes(5, json.dumps(n["metadata"]).encode())
        obj += _field_bytes(6, _VERSION_DEF)
        out += _field_bytes(1, bytes(obj))
    return bytes(out)


def decode_metadata(data: bytes) -> List[dict]:
    nodes = []
    for num, v in _fields(data):
        if num != 1:
            continue
        d = {"node_id": 0}
        for f, x in _fields(v):
            if f == 2:
                d["node_id"] = int(x)
            elif f == 3:
                d["node_path"] = x.decode()
            elif f == 4:
                d["identifier"] = x.decode()
            elif f == 5:
                d["metadata"] = json.loads(x.decode())
        nodes.append(d)
    return nodes


def read_keras_metadata_pb(path: str) -> List[dict]:
    f = path if path.endswith(".pb") else os.path.join(path, META_FILE)
    with open(f, "rb") as fh:
        return decode_metadata(fh.read())


# ------------------------------------------------------------------ Keras JSON builders
class _Builder:
    def __init__(self):
        self.nodes: List[dict] = []
        self.shared = 0
        self.names = {}

    def sid(self) -> int:
        self.shared += 1
        return self.shared

    def name(self, prefix: str) -> str:
        k = self.names.get(prefix, 0)
        self.names[prefix] = k + 1
        return prefix if k == 0 else f"{prefix}_{k}"

    def init(self, cls: str, config: Optional[dict] = None) -> dict:
        return {"class_name": cls, "config": config or {}, "shared_object_id": self.sid()}

    def add(self, path: str, identifier: str, meta: dict):
        self.nodes.append({"node_id": len(self.nodes) and (10 + len(self.nodes)), "node_path": path,
                           "identifier": identifier, "metadata": meta})


def _shape(*items):
    return {"class_name": "TensorShape", "items": list(items)}


def _tuple(*items):
    return {"class_name": "__tuple__", "items": list(items)}


def _layer_meta(name, cls, config, build_shape, expects_training=False, input_spec=None, sid=None):
    m = {"name": name, "trainable": True, "expects_training_arg": expects_training, "dtype": "float32",
         "batch_input_shape": None, "stateful": False, "must_restore_from_config": False,
         "preserve_input_structure_in_config": False, "autocast": True, "class_name": cls,
         "config": {"name": name, "trainable": True, "dtype": "float32", **config}, "shared_object_id": sid}
    if input_spec is not None:
        m["input_spec"] = input_spec
    m["build_input_shape"] = build_shape
    return m


def _input_spec(b: _Builder, ndim=None, min_ndim=None, axes=None, shape=None):
    return {"class_name": "InputSpec", "config": {"dtype": None, "shape": shape, "ndim": ndim, "max_ndim": None,
                                                  "min_ndim": min_ndim, "axes": axes or {}},
            "shared_object_id": b.sid()}


def _dense(b: _Builder, path: str, d, in_features: int, activation: Optional[str] = None):
    name = b.name("dense")
    units = int(d.kernel.shape[1])
    cfg = {"units": units, "activation": activation or d.activation or "linear", "use_bias": d.bias is not None,
           "kernel_initializer": b.init("GlorotUniform", {"seed": None}), "bias_initializer": b.init("Zeros"),
           "kernel_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
           "kernel_constraint": None, "bias_constraint": None}
    sid = b.sid()
    b.add(path, "_tf_keras_layer", _layer_meta(name, "Dense", cfg, _shape(None, in_features), sid=sid,
                                               input_spec=_input_spec(b, min_ndim=2, axes={"-1": in_features})))


def _leaky(b: _Builder, path: str, alpha: float, width, ndim=2):
    name = b.name("leaky_re_lu")
    shape = _shape(None, width) if ndim == 2 else _shape(None, *width)
    b.add(path, "_tf_keras_layer", _layer_meta(name, "LeakyReLU", {"alpha": float(alpha)}, shape, sid=b.sid()))


def _lstm(b: _Builder, path: str, lstm, T: Optional[int], din: int):
    name = b.name("lstm")
    units = int(lstm.units)
    cell_cfg = {"units": units, "activation": lstm.activation, "recurrent_activation": "sigmoid", "use_bias": True,
                "kernel_initializer": b.init("GlorotUniform", {"seed": None}),
                "recurrent_initializer": b.init("Orthogonal", {"gain": 1.0, "seed": None}),
                "bias_initializer": b.init("Zeros"), "unit_forget_bias": True,
                "kernel_regularizer": _reg(lstm.regularizer), "recurrent_regularizer": _reg(lstm.regularizer),
                "bias_regularizer": None, "kernel_constraint": None, "recurrent_constraint": None,
                "bias_constraint": None, "dropout": 0.0, "recurrent_dropout": 0.0, "implementation": 2}
    cell_sid = b.sid()
    cfg = {"return_sequences": bool(lstm.return_sequences), "return_state": False, "go_backwards": False,
           "stateful": False, "unroll": False, "time_major": False, **{k: v for k, v in cell_cfg.items()
                                                                     if k != "kernel_regularizer"},
           "kernel_regularizer": cell_cfg["kernel_regularizer"], "activity_regularizer": None}
    spec = [_input_spec(b, ndim=3, shape=_tuple(None, None, din))]
    b.add(path, "_tf_keras_rnn_layer", _layer_meta(name, "LSTM", cfg, _shape(None, T, din), True, spec, b.sid()))
    cell_name = b.name("lstm_cell")
    b.add(path + ".cell", "_tf_keras_layer",
          _layer_meta(cell_name, "LSTMCell", cell_cfg, _tuple(None, din), True, sid=cell_sid))


def _conv(b: _Builder, path: str, conv, T: Optional[int], din: int):
    name = b.name("conv1d")
    k, _, filters = conv.kernel.shape
    cfg = {"filters": int(filters), "kernel_size": _tuple(int(k)), "strides": _tuple(1), "padding": conv.padding,
           "data_format": "channels_last", "dilation_rate": _tuple(1), "groups": 1, "activation": "linear",
           "use_bias": True, "kernel_initializer": b.init("GlorotUniform", {"seed": None}),
           "bias_initializer": b.init("Zeros"), "kernel_regularizer": _reg(conv.regularizer),
           "bias_regularizer": None, "activity_regularizer": None, "kernel_constraint": None,
           "bias_constraint": None}
    b.add(path, "_tf_keras_layer", _layer_meta(name, "Conv1D", cfg, _shape(None, T, din), sid=b.sid(),
                                               input_spec=_input_spec(b, min_ndim=3, axes={"-1": din})))


def _pool(b: _Builder, path: str, p: int, T: Optional[int], C: int):
    name = b.name("max_pooling1d")
    cfg = {"strides": _tuple(p), "pool_size": _tuple(p), "padding": "valid", "data_format": "channels_last"}
    b.add(path, "_tf_keras_layer", _layer_meta(name, "MaxPooling1D", cfg, _shape(None, T, C), sid=b.sid(),
                                               input_spec=_input_spec(b, ndim=3)))


def _reg(r):
    return None if not r else {"class_name": "L2", "config": {"l2": float(r)}}


def _timelayer_children(b: _Builder, prefix: str, tl, T0: Optional[int], din: int):
    """time1, time2, max_pooling, time4, then the lists (Keras tracks list items later)."""
    cnn = tl.layer_type != "lstm"
    seq = tl._sequence()
    # shapes through the stack
    shapes = []
    T, c = T0, din
    for mod in seq:
        shapes.append((T, c))
        if mod.__class__.__name__ == "MaxPooling1D":
            T = None if T is None else T // mod.pool_size
        else:
            c = int(mod.units) if hasattr(mod, "units") else int(mod.kernel.shape[2])
    idx = {id(m): s for m, s in zip(seq, shapes)}
    leaf = _conv if cnn else _lstm

    def emit(path, mod):
        T_, c_ = idx[id(mod)]
        if mod.__class__.__name__ == "MaxPooling1D":
            _pool(b, path, mod.pool_size, T_, c_)
        else:
            leaf(b, path, mod, T_, c_)

    emit(prefix + "time1", tl.time1)
    emit(prefix + "time2", tl.time2)
    emit(prefix + "max_pooling", tl.max_pooling)
    emit(prefix + "time4", tl.time4)
    if cnn:
        f1 = int(tl.time1.kernel.shape[2])
        _leaky(b, prefix + "leakyrelu1", tl.leakyrelu1.alpha, (idx[id(tl.time1)][0], f1), 3)
        _leaky(b, prefix + "leakyrelu2", tl.leakyrelu2.alpha, (idx[id(tl.time2)][0], f1), 3)
        _leaky(b, prefix + "leakyrelu3", tl.leakyrelu3.alpha, (idx[id(tl.time4)][0], tl.out_features), 3)
        b.add(prefix + "global_pooling", "_tf_keras_layer",
              _layer_meta(b.name("global_average_pooling1d"), "GlobalAveragePooling1D",
                          {"data_format": "channels_last", "keepdims": False},
                          _shape(None, idx[id(tl.time4)][0], tl.out_features), sid=b.sid()))
    return emit


def _timelayer_lists(b: _Builder, prefix: str, tl, emit):
    for i, mod in enumerate(tl.time_layers):
        emit(f"{prefix}time_layers.{i}", mod)
    for i, mod in enumerate(tl.pooling_layers):
        emit(f"{prefix}pooling_layers.{i}", mod)


_METRICS = [("Mean", "loss", {}), ("Recall", "recall", {"thresholds": None, "top_k": None, "class_id": None}),
            ("BinaryAccuracy", "binary_accuracy", {"threshold": 0.5}),
            ("Precision", "precision", {"thresholds": None, "top_k": None, "class_id": None}),
            ("AUC", "auc", {"num_thresholds": 200, "curve": "ROC", "summation_method": "interpolation",
                            "multi_label": False, "num_labels": None, "label_weights": None, "from_logits": False}),
            ("TruePositives", "tp", {"thresholds": None}), ("FalsePositives", "fp", {"thresholds": None}),
            ("TrueNegatives", "tn", {"thresholds": None}), ("FalseNegatives", "fn", {"thresholds": None})]


def _metric_specs(b: _Builder):
    specs = []
    for cls, name, cfg in _METRICS:
        specs.append({"class_name": cls, "name": name, "dtype": "float32",
                      "config": {"name": name, "dtype": "float32", **cfg}, "shared_object_id": b.sid()})
    return specs


def _seq_len(model) -> Optional[int]:
    try:
        return int((model.timestep_before + model.timestep_after) // model.freq + 1)
    except Exception:
        return None


def build_metadata(model, optimizer=None) -> List[dict]:
    """Keras metadata nodes for a :class:`GCNClassifier` or :class:`BaselineClassifier`."""
    b = _Builder()
    is_gcn = type(model).__name__ == "GCNClassifier"
    metrics = _metric_specs(b)
    T0 = _seq_len(model)
    F = int(getattr(model, "input_feature_numb", 2))
    lr = float(optimizer.lr) if optimizer is not None else float(getattr(model, "model_config", {}).get(
        "learning_rate", 1e-3) if hasattr(model, "model_config") else 1e-3)
    training_config = {
        "loss": "binary_crossentropy",
        "metrics": [[{k: v for k, v in m.items() if k != "name" and k != "dtype"} for m in metrics[1:]]],
        "weighted_metrics": None, "loss_weights": None,
        "optimizer_config": {"class_name": "Custom>Adam", "config": {
            "name": "Adam", "weight_decay": None, "clipnorm": None, "global_clipnorm": None, "clipvalue": None,
            "use_ema": False, "ema_momentum": 0.99, "ema_overwrite_frequency": None, "jit_compile": True,
            "is_legacy_optimizer": False, "learning_rate": lr, "beta_1": 0.9, "beta_2": 0.999, "epsilon": 1e-07,
            "amsgrad": False}}}
    cls = "GCNClassifier" if is_gcn else "BaselineClassifier"
    if is_gcn:
        build = _tuple(_shape(None, F), _shape(None, None, F), _shape(None, None), _shape(None), _shape(None))
    elif getattr(model, "ds_type", "cml") == "soilnet":
        build = _tuple(_shape(None, F), _shape(None))     # node rows + graph index -> graph_reshape (T fixed)
    else:
        T0 = None                                         # CML baseline: the window length is not fixed at build
        build = _shape(None, None, F)
    root = {"name": "gcn_classifier" if is_gcn else "baseline_classifier", "trainable": True,
            "expects_training_arg": False, "dtype": "float32", "batch_input_shape": None,
            "must_restore_from_config": False, "preserve_input_structure_in_config": False, "autocast": True,
            "class_name": cls, "config": {}, "shared_object_id": 0, "build_input_shape": build,
            "is_graph_network": False, "keras_version": KERAS_VERSION, "backend": "tensorflow",
            "model_config": {"class_name": cls, "config": {}}, "training_config": training_config}
    b.add("root", "_tf_keras_model", root)
    tl = model.time_layer
    units = int(model.dense.kernel.shape[1]) if is_gcn else int(model.dense1.kernel.shape[1])
    if is_gcn:
        g = model.gcn_layer
        gname = b.name("general_conv") if type(g).__name__ == "GeneralConv" else b.name(type(g).__name__.lower())
        prelu_sid = b.sid()
        gcfg = {"activation": {"class_name": "PReLU", "config": {
            "name": "p_re_lu", "trainable": True, "dtype": "float32", "alpha_initializer": b.init("Zeros"),
            "alpha_regularizer": None, "alpha_constraint": None, "shared_axes": None}, "shared_object_id": prelu_sid},
            "use_bias": True, "kernel_initializer": b.init("GlorotUniform", {"seed": None}),
            "bias_initializer": b.init("Zeros"), "kernel_regularizer": _reg(getattr(g, "regularizer", None)),
            "bias_regularizer": None, "kernel_constraint": None, "bias_constraint": None,
            "aggregate": getattr(g, "aggregate", "mean"), "channels": int(g.out_features),
            "prelu": getattr(g, "activation", "prelu") == "prelu"}
        b.add("root.gcn_layer", "_tf_keras_layer",
              _layer_meta(gname, type(g).__name__, gcfg, [_shape(None, F), _shape(None, None)], True, sid=b.sid()))
        tcfg = {"layer_type": tl.layer_type, "activation": getattr(tl.time1, "activation", "tanh"),
                "kernel_size": int(tl.time1.kernel_size) if tl.layer_type != "lstm" else None,
                "regularizer": getattr(tl.time1, "regularizer", None), "filter_1_size": tl.filter_1_size,
                "n_stacks": tl.n_stacks, "alpha": tl.alpha, "pool_size": tl.pool_size}
        din = int(tl.time1.kernel.shape[-2] if tl.layer_type != "lstm" else tl.time1.kernel.shape[0])
        b.add("root.time_layer", "_tf_keras_layer",
              _layer_meta(b.name("time_layer"), "Custom>TimeLayer", tcfg, _shape(None, T0, din), sid=b.sid()))
        _dense(b, "root.dense", model.dense, tl.out_features)
        _leaky(b, "root.leakyrelu4", model.leakyrelu4.alpha, units)
        _dense(b, "root.dense2", model.dense2, units)
        _leaky(b, "root.leakyrelu5", model.leakyrelu5.alpha, units)
        _dense(b, "root.dense_out", model.dense_out, units, "sigmoid")   # sigmoid applied outside (logit loss)
        if type(g).__name__ == "GeneralConv":
            ch = int(g.out_features)
            b.add("root.gcn_layer.activation", "_tf_keras_layer", _layer_meta(
                b.name("p_re_lu"), "PReLU", {"alpha_initializer": b.init("Zeros"), "alpha_regularizer": None,
                                             "alpha_constraint": None, "shared_axes": None},
                _shape(None, ch), sid=prelu_sid, input_spec=_input_spec(b, ndim=2)))
            b.add("root.gcn_layer.dropout", "_tf_keras_layer", _layer_meta(
                b.name("dropout"), "Dropout", {"rate": g.dropout, "noise_shape": None, "seed": None},
                _shape(None, ch), True, sid=b.sid()))
            b.add("root.gcn_layer.batch_norm", "_tf_keras_layer", _layer_meta(
                b.name("batch_normalization"), "BatchNormalization", {
                    "axis": [1], "momentum": g.momentum, "epsilon": g.eps, "center": True, "scale": True,
                    "beta_initializer": b.init("Zeros"), "gamma_initializer": b.init("Ones"),
                    "moving_mean_initializer": b.init("Zeros"), "moving_variance_initializer": b.init("Ones"),
                    "beta_regularizer": None, "gamma_regularizer": None, "beta_constraint": None,
                    "gamma_constraint": None}, _shape(None, ch), True, sid=b.sid(),
                input_spec=_input_spec(b, ndim=2, axes={"1": ch})))
        emit = _timelayer_children(b, "root.time_layer.", tl, T0, din)
    else:
        din = F
        emit = _timelayer_children(b, "root.", tl, T0, din)
        _dense(b, "root.dense1", model.dense1, tl.out_features)
        _leaky(b, "root.leakyrelu4", model.leakyrelu4.alpha, units)
        _dense(b, "root.dense2", model.dense2, units)
        _leaky(b, "root.leakyrelu5", model.leakyrelu5.alpha, units)
        _dense(b, "root.dense_out", model.dense_out, units, "sigmoid")   # sigmoid applied outside (logit loss)
    for i, m in enumerate(metrics):
        b.add(f"root.keras_api.metrics.{i}", "_tf_keras_metric", m)
    _timelayer_lists(b, "root.time_layer." if is_gcn else "root.", tl, emit)
    # LSTM cells are emitted right after their layer above; keep the reference's ordering:
    # layers, metrics, list items, then cells
    cells = [n for n in b.nodes if n["node_path"].endswith(".cell")]
    rest = [n for n in b.nodes if not n["node_path"].endswith(".cell")]
    nodes = rest + cells
    for i, n in enumerate(nodes):
        n["node_id"] = 0 if i == 0 else 10 + i
    return nodes


def write_keras_metadata(model, path: str, optimizer=None) -> str:
    os.makedirs(path, exist_ok=True)
    f = os.path.join(path, META_FILE)
    with open(f + ".tmp", "wb") as fh:
        fh.write(encode_metadata(build_metadata(model, optimizer)))
    os.replace(f + ".tmp", f)
    return f


__all__ = ["build_metadata", "write_keras_metadata", "read_keras_metadata_pb", "encode_metadata",
           "decode_metadata"]
