"""Keras SavedModel variable layout <-> gnnqc modules.

The reference saves ``model.save(path)`` directories whose TensorBundle keys are
``variables/<i>/.ATTRIBUTES/VARIABLE_VALUE`` in Keras' tracking order, plus the
non-trainable metadata variables ``model_info`` / ``model_type`` /
``model_normalization`` (GCN, ``libs/create_model.py:159-165``) or
``normalization`` (baseline, ``libs/create_model.py:276``), and Adam slots
``optimizer/_variables/{1..2n}`` interleaved (m, v) per trainable.

Our modules register their tensors in exactly that order (GeneralConv kernel,
bias, PReLU alpha, BN gamma/beta/moving stats; ``TimeLayer.time_layers[0..3]``
before ``time1/time2/time4``, ``libs/create_model.py:52-53``; dense heads), so
the mapping is positional over ``state_dict()`` minus the ``model_info`` buffer.
Shapes are checked entry by entry, so a layout drift fails loudly.

* :func:`load_keras_weights` - import a reference ``model_*`` directory (e.g.
  ``/root/reference/model_cml``) into a freshly built model;
* :func:`write_keras_variables` - export ours in the same layout.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .tensorbundle import read_bundle, write_bundle

SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"


def _var_key(i: int) -> str:
    return f"variables/{i}{SUFFIX}"


def ordered_variables(model) -> List[Tuple[str, torch.Tensor]]:
    """(state-dict name, tensor) in Keras ``model.variables`` order."""
    return [(k, v) for k, v in model.state_dict(keep_vars=True).items() if k != "model_info"]


def _is_baseline(model) -> bool:
    return type(model).__name__ == "BaselineClassifier"


def keras_tensors(model, optimizer=None) -> Dict[str, object]:
    out: Dict[str, object] = {}
    for i, (_, t) in enumerate(ordered_variables(model)):
        out[_var_key(i)] = t.detach().float().cpu().numpy()
    if hasattr(model, "model_info"):
        out["model_info" + SUFFIX] = model.model_info.detach().cpu().numpy().astype(np.int32)
    if _is_baseline(model):
        out["normalization" + SUFFIX] = str(model.normalization)
    else:
        out["model_type" + SUFFIX] = str(getattr(model, "model_type", model.ds_type))
        out["model_normalization" + SUFFIX] = str(model.model_normalization)
    if optimizer is not None:
        out["optimizer/_iterations" + SUFFIX] = np.asarray(int(optimizer.step_t.item()), dtype=np.int64)
        out["optimizer/_learning_rate" + SUFFIX] = np.asarray(optimizer.lr, dtype=np.float32)
        slots = optimizer.slots() if hasattr(optimizer, "slots") else []
        if len(slots) == 2:
            ms, vs = optimizer.views(slots[0]), optimizer.views(slots[1])
            for j, (m, v) in enumerate(zip(ms, vs)):
                out[f"optimizer/_variables/{2 * j + 1}{SUFFIX}"] = m.detach().cpu().numpy()
                out[f"optimizer/_variables/{2 * j + 2}{SUFFIX}"] = v.detach().cpu().numpy()
    return out


OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"


def trackable_tree(keys, full_names: Optional[Dict[str, str]] = None) -> List[dict]:
    """Node list of the object graph for a set of ``<path>/.ATTRIBUTES/VARIABLE_VALUE`` keys: node 0
    is the root, every path prefix (``variables``, ``variables/3``, ``optimizer/_variables``, ...) is a
    node whose ``children`` are ``(node_id, local_name)`` pairs, and a variable node carries
    ``attrs = [(name, full_name, checkpoint_key)]`` and ``key``. Node ids follow sorted key order, so
    the ``_CHECKPOINTABLE_OBJECT_GRAPH`` (:func:`object_graph`) and the ``SavedObjectGraph`` of
    ``saved_model.pb`` (:mod:`gnnqc.ckpt.saved_model`) number their nodes identically."""
    full_names = full_names or {}
    nodes = [{"children": [], "attrs": [], "path": (), "key": None}]
    index = {(): 0}
    for key in sorted(keys):
        if not key.endswith(SUFFIX):
            continue
        parts = tuple(key[: -len(SUFFIX)].split("/"))
        for d in range(1, len(parts) + 1):
            pre = parts[:d]
            if pre not in index:
                index[pre] = len(nodes)
                nodes.append({"children": [], "attrs": [], "path": pre, "key": None})
                nodes[index[parts[: d - 1]]]["children"].append((index[pre], parts[d - 1]))
        nodes[index[parts]]["attrs"].append(("VARIABLE_VALUE", full_names.get(key, "/".join(parts)), key))
        nodes[index[parts]]["key"] = key
    return nodes


def object_graph(keys, full_names: Optional[Dict[str, str]] = None) -> bytes:
    """``TrackableObjectGraph`` proto for a set of ``<path>/.ATTRIBUTES/VARIABLE_VALUE`` keys.

    Node 0 is the root; every path prefix (``variables``, ``variables/3``, ``optimizer/_variables``,
    ...) becomes a node whose ``children`` reference the next component by local name, and each
    variable node carries one ``SerializedTensor`` attribute (name ``VARIABLE_VALUE``, the
    checkpoint key) - the part of the reference's 600-node Keras graph
    (``model_cml/variables``, decoded in SURVEY §5.4) that object-based restore uses to map
    checkpoint keys to objects. Function / signature nodes are not emitted (no graph is saved).
    Field numbers follow tensorflow/core/protobuf/trackable_object_graph.proto."""
    from .tensorbundle import _pb_bytes, _pb_varint
    out = b""
    for n in trackable_tree(keys, full_names):
        body = b"".join(_pb_bytes(1, _pb_varint(1, nid) + _pb_bytes(2, name.encode())) for nid, name in n["children"])
        body += b"".join(_pb_bytes(2, _pb_bytes(1, a.encode()) + _pb_bytes(2, f.encode()) + _pb_bytes(3, k.encode()))
                         for a, f, k in n["attrs"])
        out += _pb_bytes(1, body)
    return out


def write_fingerprint(path: str):
    """``fingerprint.pb`` (``FingerprintDef``): 64-bit content hashes of what the directory holds
    (fields 1-5: saved-model checksum, graph hash, signature hash, object-graph hash, checkpoint
    hash; 6: version). Our hashes are blake2b-64 of the files, not TF's farmhash; saved_model.pb
    holds no ops or signatures, so the graph / signature hashes are of empty inputs."""
    import hashlib
    from .tensorbundle import _pb_bytes, _pb_varint

    def h(*blobs):
        d = hashlib.blake2b(digest_size=8)
        for b in blobs:
            d.update(b)
        return int.from_bytes(d.digest(), "little")

    var = os.path.join(path, "variables", "variables")
    with open(var + ".index", "rb") as f:
        idx = f.read()
    with open(var + ".data-00000-of-00001", "rb") as f:
        data = f.read()
    meta = b""
    mp = os.path.join(path, "keras_metadata.pb")
    if os.path.exists(mp):
        with open(mp, "rb") as f:
            meta = f.read()
    sm = b""
    sp = os.path.join(path, "saved_model.pb")
    if os.path.exists(sp):
        with open(sp, "rb") as f:
            sm = f.read()
    ck = h(idx, data)
    # saved-model checksum over saved_model.pb (+ the bundle and metadata), object-graph hash over the
    # SavedModel proto that carries the SavedObjectGraph (the bundle's index when none was written)
    fp = (_pb_varint(1, h(sm, idx, data, meta)) + _pb_varint(2, h(b"")) + _pb_varint(3, h(b""))
          + _pb_varint(4, h(sm) if sm else h(idx)) + _pb_varint(5, ck) + _pb_bytes(6, b""))
    with open(os.path.join(path, "fingerprint.pb"), "wb") as f:
        f.write(fp)


def trainable_keys(model) -> List[str]:
    """Checkpoint keys of the trainable ``variables/<i>`` (parameters; BN moving statistics are not)."""
    return [_var_key(i) for i, (_, t) in enumerate(ordered_variables(model))
            if isinstance(t, torch.nn.Parameter) and t.requires_grad]


def write_keras_variables(model, path: str, optimizer=None, saved_model: bool = True):
    """Write ``<path>/variables/variables.{index,data-00000-of-00001}`` (with the object graph) and,
    unless ``saved_model=False``, the best-effort ``<path>/saved_model.pb`` whose SavedObjectGraph
    mirrors that object graph node for node (:mod:`gnnqc.ckpt.saved_model`)."""
    t = keras_tensors(model, optimizer)
    t[OBJECT_GRAPH_KEY] = object_graph(list(t))
    write_bundle(os.path.join(path, "variables", "variables"), t)
    if saved_model:
        from .saved_model import write_saved_model
        write_saved_model(path, t, trainable_keys(model))


def _bundle_prefix(path: str) -> str:
    if os.path.exists(path + ".index"):
        return path
    p = os.path.join(path, "variables", "variables")
    if os.path.exists(p + ".index"):
        return p
    raise FileNotFoundError(f"no TensorBundle under {path}")


def read_keras_metadata(path: str) -> Dict[str, object]:
    """Metadata variables (model_info, model_type, normalization) of a saved model."""
    b = read_bundle(_bundle_prefix(path))
    meta = {}
    for name in ("model_info", "model_type", "model_normalization", "normalization"):
        v = b.get(name + SUFFIX)
        if v is None:
            continue
        meta[name] = v.decode() if isinstance(v, bytes) else v.tolist()
    return meta


def load_keras_weights(model, path: str, strict: bool = True) -> Dict[str, object]:
    """Copy the ``variables/<i>`` tensors of a Keras model directory into ``model``.

    Returns the metadata variables. Only tensors and strings are read (no pickles,
    nothing executed)."""
    b = read_bundle(_bundle_prefix(path))
    ours = ordered_variables(model)
    n_ref = sum(1 for k in b if k.startswith("variables/"))
    if strict and n_ref != len(ours):
        raise ValueError(f"variable count mismatch: checkpoint {n_ref}, model {len(ours)}")
    with torch.no_grad():
        for i, (name, t) in enumerate(ours):
            key = _var_key(i)
            if key not in b:
                if strict:
                    raise KeyError(key)
                continue
            arr = b[key]
            if tuple(arr.shape) != tuple(t.shape):
                raise ValueError(f"{key} -> {name}: shape {arr.shape} != {tuple(t.shape)}")
            t.copy_(torch.from_numpy(np.ascontiguousarray(arr)).to(t.dtype))
        mi = b.get("model_info" + SUFFIX)
        if mi is not None and hasattr(model, "model_info"):
            # the reference baseline stores only (tb, ta, batch_size) - an older code path
            n = min(mi.size, model.model_info.numel())
            model.model_info[:n].copy_(torch.from_numpy(mi[:n].astype(np.int64)).to(model.model_info.dtype))
    meta = read_keras_metadata(path)
    norm = meta.get("model_normalization", meta.get("normalization"))
    if norm is not None:
        if _is_baseline(model):
            model.normalization = norm
        else:
            model.model_normalization = norm
    return meta


def load_keras_optimizer(optimizer, path: str):
    """Restore Adam slots / iteration counter written by :func:`write_keras_variables`
    (the reference discards them on load; we can resume)."""
    b = read_bundle(_bundle_prefix(path))
    it = b.get("optimizer/_iterations" + SUFFIX)
    if it is not None:
        optimizer.iterations = int(it)
        optimizer.step_t.fill_(float(int(it)))
    lr = b.get("optimizer/_learning_rate" + SUFFIX)
    if lr is not None:
        optimizer.lr = float(lr)
    slots = optimizer.slots() if hasattr(optimizer, "slots") else []
    if len(slots) == 2:
        with torch.no_grad():
            for j, (m, v) in enumerate(zip(optimizer.views(slots[0]), optimizer.views(slots[1]))):
                km, kv = f"optimizer/_variables/{2 * j + 1}{SUFFIX}", f"optimizer/_variables/{2 * j + 2}{SUFFIX}"
                if km in b and b[km].shape == tuple(m.shape):
                    m.copy_(torch.from_numpy(b[km]))
                    v.copy_(torch.from_numpy(b[kv]))


def build_from_keras(path: str, ds_type: Optional[str] = None, baseline: Optional[bool] = None, device="cpu"):
    """Build the matching gnnqc model (packaged default configs) and load a reference
    Keras model directory into it."""
    from .. import config as C
    from ..models import create_model
    meta = read_keras_metadata(path)
    if baseline is None:
        baseline = "normalization" in meta and "model_type" not in meta
    if ds_type is None:
        ds_type = meta.get("model_type") or ("soilnet" if meta.get("normalization") == "scale_range" else "cml")
    pc = C.normalize_preproc(C.default(f"preprocessing_{ds_type}"))
    mc = C.default(f"model_{ds_type}")
    mi = meta.get("model_info")
    if mi:
        pc["timestep_before"], pc["timestep_after"], pc["batch_size"] = int(mi[0]), int(mi[1]), int(mi[2])
    pc["normalization"] = meta.get("model_normalization", meta.get("normalization"))
    model = create_model(mc, pc, baseline=baseline)
    load_keras_weights(model, path)
    return model.to(device), pc, mc


__all__ = ["write_keras_variables", "trainable_keys", "trackable_tree", "object_graph", "load_keras_weights", "load_keras_optimizer", "read_keras_metadata",
           "build_from_keras", "ordered_variables", "keras_tensors"]
