"""Configuration system.

The reference drives everything through OmegaConf YAML objects with attribute
access that are mutated at run time (``/root/reference/libs/config/*.yml``,
``notebooks/pipeline.ipynb`` nb:70-73, ``libs/preprocessing_functions.py:941,964``).
OmegaConf is not available here, so this module provides :class:`Config`, a
small attribute-access mapping on top of PyYAML with

* nested attribute access and mutation (``cfg.graph.max_sample_distance``),
* ``**cfg`` unpacking (the reference merges configs via ``{**pc, **mc}``,
  ``libs/fit_model.py:66``),
* dotted command line overrides (``trainer.lr=5e-4``),
* both schemas of the reference: the final flat preprocessing schema
  (``libs/config/preprocessing_config*.yml``) and the XAI-snapshot nested
  ``dataset:`` schema (``xai/libs/config/preprocessing_config_20240318.yml``).
  :func:`normalize_preproc` mirrors keys so code may read either spelling.
"""
from __future__ import annotations

import copy
import os
from typing import Any, Iterable, Mapping

import yaml

_DEFAULTS_DIR = os.path.join(os.path.dirname(__file__), "defaults")


class Config(dict):
    """A dict with attribute access; nested dicts become Configs."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        data = dict(*args, **kwargs)
        for k, v in data.items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, Config):
            return v
        if isinstance(v, Mapping):
            return Config(v)
        if isinstance(v, list):
            return [Config._wrap(x) for x in v]
        return v

    def __setitem__(self, key, value):
        super().__setitem__(key, Config._wrap(value))

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = value

    def __delattr__(self, key):
        del self[key]

    def __deepcopy__(self, memo):
        return Config(copy.deepcopy(dict(self), memo))

    def copy(self):
        return copy.deepcopy(self)

    def to_dict(self) -> dict:
        out = {}
        for k, v in self.items():
            if isinstance(v, Config):
                out[k] = v.to_dict()
            elif isinstance(v, list):
                out[k] = [x.to_dict() if isinstance(x, Config) else x for x in v]
            else:
                out[k] = v
        return out

    def select(self, dotted: str, default: Any = None) -> Any:
        node: Any = self
        for part in dotted.split("."):
            if isinstance(node, Mapping) and part in node:
                node = node[part]
            else:
                return default
        return node

    def set_dotted(self, dotted: str, value: Any) -> None:
        parts = dotted.split(".")
        node = self
        for part in parts[:-1]:
            if part not in node or not isinstance(node[part], Mapping):
                node[part] = Config()
            node = node[part]
        node[parts[-1]] = value


def load(path: str) -> Config:
    """Load a YAML file into a :class:`Config` (safe loader only)."""
    with open(path, "r") as f:
        data = yaml.safe_load(f) or {}
    return Config(data)


def save(cfg: Mapping, path: str) -> None:
    d = cfg.to_dict() if isinstance(cfg, Config) else dict(cfg)
    with open(path, "w") as f:
        yaml.safe_dump(d, f, sort_keys=False)


def merge(base: Mapping, other: Mapping) -> Config:
    """Recursive merge; values of ``other`` win."""
    out = Config(copy.deepcopy(dict(base)))
    for k, v in other.items():
        if k in out and isinstance(out[k], Mapping) and isinstance(v, Mapping):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def parse_overrides(cfg: Config, overrides: Iterable[str]) -> Config:
    """Apply ``a.b.c=value`` overrides; values are parsed as YAML scalars."""
    for ov in overrides or ():
        if "=" not in ov:
            raise ValueError(f"override must look like key=value, got {ov!r}")
        key, raw = ov.split("=", 1)
        cfg.set_dotted(key.strip(), yaml.safe_load(raw))
    return cfg


def default(name: str) -> Config:
    """Packaged default config by name, e.g. ``preprocessing_cml``."""
    return load(os.path.join(_DEFAULTS_DIR, f"{name}.yml"))


def available_defaults():
    return sorted(f[:-4] for f in os.listdir(_DEFAULTS_DIR) if f.endswith(".yml"))


# keys that live under ``dataset:`` in the XAI-snapshot schema and at top level in
# the final schema (libs/config/preprocessing_config.yml vs
# xai/libs/config/preprocessing_config_20240318.yml)
_DATASET_KEYS = (
    "raw_dataset_path", "create_nc_files", "ncfiles_dir", "create_tfrecords_dataset",
    "tfrecords_dataset_dir", "train_fraction", "val_fraction", "interpolate", "split_numb",
)


def normalize_preproc(cfg: Config) -> Config:
    """Make a preprocessing config readable through both reference schemas.

    Flat keys are mirrored into ``cfg.dataset`` and vice versa; missing keys get
    the reference defaults. Unknown keys are kept untouched.
    """
    cfg = Config(cfg)
    ds = cfg.get("dataset")
    if not isinstance(ds, Mapping):
        ds = Config()
    for k in _DATASET_KEYS:
        if k in cfg and k not in ds:
            ds[k] = cfg[k]
        elif k in ds and k not in cfg:
            cfg[k] = ds[k]
    cfg["dataset"] = ds
    cfg.setdefault("ds_type", "cml")
    cfg.setdefault("random_state", 44)
    cfg.setdefault("window_length", 4320 if cfg.ds_type == "cml" else 20160)
    cfg.setdefault("train_fraction", 0.6)
    cfg.setdefault("val_fraction", 0.2)
    cfg.setdefault("interpolate", True)
    cfg.setdefault("split_numb", 5)
    # SoilNet of the XAI generation: per-anomalous-sensor neighbourhoods (one flagged sensor per
    # box) instead of one network-wide graph (xai/libs/preprocessing_functions.py:951-1025)
    cfg.setdefault("per_sensor", cfg.ds_type == "cml")
    cfg.dataset.setdefault("split_numb", cfg.split_numb)
    g = cfg.get("graph")
    if not isinstance(g, Mapping):
        g = Config()
    g.setdefault("max_sample_distance", 20)
    g.setdefault("max_neighbour_distance", 10)
    g.setdefault("max_neighbour_depth", 0.1)
    # the XAI schema calls it ``max_depth`` (xai/libs/preprocessing_functions.py:955)
    g.setdefault("max_depth", g.max_neighbour_depth)
    g.setdefault("adjacency", "radius")   # 'radius' (reference) or 'knn'
    g.setdefault("k", 5)
    cfg["graph"] = g
    return cfg


def freq_minutes(ds_type: str) -> int:
    """Sampling interval: CML 1 min, SoilNet 15 min (libs/create_model.py:152-156)."""
    return 1 if ds_type == "cml" else 15


def sequence_length(cfg: Mapping) -> int:
    """T = (timestep_before + timestep_after)/freq + 1 (libs/create_model.py:12)."""
    f = freq_minutes(cfg["ds_type"])
    return int((cfg["timestep_before"] + cfg["timestep_after"]) / f + 1)


__all__ = [
    "Config", "load", "save", "merge", "parse_overrides", "default", "available_defaults",
    "normalize_preproc", "freq_minutes", "sequence_length",
]
