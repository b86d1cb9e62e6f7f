"""Checkpointing.

``save_model(model, path)`` writes a model directory:

* ``gnnqc_state.pt``   - tensors only (parameters, BN statistics, optimiser slots,
  step counters); loaded with ``torch.load(weights_only=True)``;
* ``gnnqc_meta.json``  - model/preprocessing config, class, epoch, RNG cursor;
* ``variables/variables.{index,data-00000-of-00001}`` (+ ``_CHECKPOINTABLE_OBJECT_GRAPH``),
  ``saved_model.pb``, ``keras_metadata.pb`` and ``fingerprint.pb`` - the Keras SavedModel layout
  (TensorBundle), object graph, best-effort SavedModel proto (meta graph tagged ``serve`` whose
  SavedObjectGraph mirrors the object graph), per-layer JSON and content fingerprint, see
  :mod:`gnnqc.ckpt.tensorbundle`, :mod:`gnnqc.ckpt.keras_layout`, :mod:`gnnqc.ckpt.saved_model`,
  :mod:`gnnqc.ckpt.keras_meta`.

``load_model(path)`` rebuilds the model from the metadata and restores the state;
``load_keras_weights`` imports the reference's trained ``model_*`` directories.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch

from ..config import Config

STATE_FILE = "gnnqc_state.pt"
META_FILE = "gnnqc_meta.json"


def _cfg_to_json(c):
    if c is None:
        return None
    return c.to_dict() if isinstance(c, Config) else dict(c)


def save_model(model, path: str, optimizer=None, epoch: Optional[int] = None, preproc_config=None,
               extra: Optional[dict] = None, keras_layout: bool = True):
    os.makedirs(path, exist_ok=True)
    state = {"model": {k: v.detach().cpu() for k, v in model.state_dict().items()}}
    if optimizer is not None:
        osd = optimizer.state_dict()
        state["optimizer"] = {k: (v.detach().cpu() if torch.is_tensor(v) else torch.tensor(v))
                              for k, v in osd.items()}
    tmp = os.path.join(path, STATE_FILE + ".tmp")
    torch.save(state, tmp)
    os.replace(tmp, os.path.join(path, STATE_FILE))
    meta = {
        "class": type(model).__name__,
        "ds_type": getattr(model, "ds_type", None),
        "model_config": _cfg_to_json(getattr(model, "model_config", None)),
        "preprocessing_config": _cfg_to_json(preproc_config),
        "epoch": epoch,
        "model_info": [int(x) for x in model.model_info.tolist()] if hasattr(model, "model_info") else None,
        "normalization": getattr(model, "model_normalization", getattr(model, "normalization", None)),
        **(extra or {}),
    }
    with open(os.path.join(path, META_FILE), "w") as f:
        json.dump(meta, f, indent=1, default=str)
    if keras_layout:
        from .keras_layout import write_keras_variables
        from .keras_meta import write_keras_metadata
        from .keras_layout import write_fingerprint
        write_keras_variables(model, path, optimizer)
        write_keras_metadata(model, path, optimizer)
        write_fingerprint(path)


def load_model(path: str, device="cpu", with_optimizer: bool = False):
    from ..models import BaselineClassifier, GCNClassifier
    with open(os.path.join(path, META_FILE)) as f:
        meta = json.load(f)
    mc = Config(meta["model_config"])
    pc = Config(meta["preprocessing_config"] or {})
    pc.setdefault("ds_type", meta.get("ds_type", "cml"))
    if meta.get("model_info"):
        tb, ta, bs, _ = meta["model_info"]
        pc.setdefault("timestep_before", tb)
        pc.setdefault("timestep_after", ta)
        pc.setdefault("batch_size", bs)
    pc.setdefault("normalization", meta.get("normalization"))
    cls = BaselineClassifier if meta["class"] == "BaselineClassifier" else GCNClassifier
    model = cls(mc, pc)
    state = torch.load(os.path.join(path, STATE_FILE), map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"])
    model.to(device)
    if with_optimizer:
        return model, state.get("optimizer"), meta
    return model


from .keras_layout import build_from_keras, load_keras_optimizer, load_keras_weights  # noqa: E402

__all__ = ["save_model", "load_model", "load_keras_weights", "load_keras_optimizer", "build_from_keras"]
