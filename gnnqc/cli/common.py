"""Shared CLI plumbing: configs, data sources, devices."""
from __future__ import annotations

import argparse
import os
from typing import Optional

from .. import config as C


def add_common(ap: argparse.ArgumentParser, ds_default: str = "cml"):
    ap.add_argument("--ds", choices=["cml", "soilnet"], default=ds_default, help="dataset type")
    ap.add_argument("--preproc", default=None, help="preprocessing YAML (default: packaged)")
    ap.add_argument("--model-config", default=None, help="model YAML (default: packaged)")
    ap.add_argument("--set", dest="overrides", action="append", default=[],
                    help="override: pre.<key>=v for preprocessing, model.<key>=v for the model config")
    ap.add_argument("--synthetic", action="store_true", help="generate synthetic raw data instead of reading it")
    ap.add_argument("--sensors", type=int, default=None, help="synthetic: number of sensors (CML links / soil boxes)")
    ap.add_argument("--days", type=float, default=None, help="synthetic: length in days")
    ap.add_argument("--flagged", type=int, default=None, help="synthetic CML: flagged links")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="auto")
    return ap


def load_configs(args):
    pc = C.load(args.preproc) if args.preproc else C.default(f"preprocessing_{args.ds}")
    mc = C.load(args.model_config) if args.model_config else C.default(f"model_{args.ds}")
    pre = [o[len("pre."):] for o in args.overrides if o.startswith("pre.")]
    mod = [o[len("model."):] for o in args.overrides if o.startswith("model.")]
    C.parse_overrides(pc, pre)
    C.parse_overrides(mc, mod)
    pc = C.normalize_preproc(pc)
    return pc, mc


def make_raw(args, pc):
    """Raw SensorData: read ``raw_dataset_path`` or generate synthetic data."""
    from ..data.raw_io import read_netcdf
    from ..data.synthetic import make_cml_raw, make_soilnet_raw
    path = pc.get("raw_dataset_path")
    if not args.synthetic and path and os.path.exists(path):
        return read_netcdf(path)
    if pc.ds_type == "cml":
        kw = dict(n_sensors=args.sensors or 23, n_flagged=args.flagged or 1,
                  n_minutes=int((args.days or 28) * 1440), seed=args.seed)
        ds = make_cml_raw(**kw)
        pc["min_date"], pc["max_date"] = str(ds.time[0]), str(ds.time[-1])
    else:
        kw = dict(n_boxes=args.sensors or 40, n_time=int((args.days or 89) * 96), seed=args.seed)
        ds = make_soilnet_raw(**kw)
        pc["min_date"], pc["max_date"] = str(ds.time[0]), str(ds.time[-1])
    return ds


def resolve_device(name: str):
    import torch
    from ..parallel import dist as D
    if name == "auto":
        return D.init_distributed()
    return D.init_distributed(device=name)


__all__ = ["add_common", "load_configs", "make_raw", "resolve_device"]
